set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5g; mkdir -p $O
(cd /tmp && timeout -k 5 90 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- $R/build/variants/gen_base --gens 200 --warmup 5 > $O/kt.log 2>&1) || { tail $O/kt.log; exit 1; }
timeout -k 5 60 build/examples/e1_onemax_float 200 || exit 1
timeout -k 5 120 python bench/bench_configs.py --only e1_sum100_refops || exit 1
PGA_TP_MIN_S=100000000 timeout -k 5 120 python bench/bench_configs.py --only e1_sum100_refops || exit 1
