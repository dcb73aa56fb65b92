#!/bin/bash
# Round-5 check of the rotated-MFMA / one-load roulette / REAL PD-4 /
# immigrate-bests build: targeted tests first, then the configs they move,
# the headline bench, migration cost, kernel traces, the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r5n}; mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_fused_hist.py tests/test_real.py tests/test_gpu_binary.py tests/test_jit.py tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_first.log 2>&1 || { tail -40 $O/pytest_first.log; exit 1; }
tail -2 $O/pytest_first.log
timeout -k 10 900 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot rastrigin30_jit onemax1024_roulette_2pt onemax1024_rank e1_sum100_refops > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl | cut -c1-220
timeout -k 5 60 build/examples/e1_onemax_float 200 > $O/e1_fnptr.log 2>&1 || { cat $O/e1_fnptr.log; exit 1; }
head -1 $O/e1_fnptr.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-200
PGA_OUT=$O/mig_epoch.json timeout -k 10 200 python bench/migration_cost.py > $O/mig_epoch.log 2>&1 || { tail -20 $O/mig_epoch.log; exit 1; }
cat $O/mig_epoch.json
PGA_RCCL_SELF=1 PGA_OUT=$O/mig_rccl_self.json timeout -k 10 400 python bench/migration_cost.py > $O/mig_rccl.log 2>&1 || { tail -20 $O/mig_rccl.log; exit 1; }
cat $O/mig_rccl_self.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mig --output-format csv -o run -- python3 $R/bench/migration_cost.py > $O/prof_mig.log 2>&1 || { tail -20 $O/prof_mig.log; exit 1; }
for c in rastrigin30_rot onemax1024_roulette_2pt e1_sum100_refops; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c --output-format csv -o run -- python3 $R/bench/bench_configs.py --only $c > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 1; }
done
cd $R
[ "${FULL:-1}" = 1 ] || exit 0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; exit $rc
