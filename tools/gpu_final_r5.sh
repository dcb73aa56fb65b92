#!/bin/bash
# Round-5 closing measurements (one call): smoke, the whole GPU suite,
# driver-shape bench, every BASELINE config, batched islands, kernel traces,
# migration cost (device epoch; RCCL self-exchange per transport), the
# migration host probe, E1 through its function pointer.  Each GPU step has
# its own limit; the chain stops at the first failure.  -> gpurun_out/final5/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/final5; mkdir -p $O
PART=${PART:-a}   # a: tests, bench, configs, islands; b: E1 fn-ptr, migration, host probe, kernel traces
if [ "$PART" = a ]; then
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-160
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 50 > $O/bench500.log 2>&1 || { cat $O/bench500.log; exit 1; }
tail -1 $O/bench500.log | cut -c1-160
timeout -k 10 900 python bench/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
echo configs done
for p in onemax rastrigin30 tsp128; do
  timeout -k 10 200 python bench/bench_islands.py --problem $p >> $O/islands.jsonl 2>> $O/islands.err || { tail -20 $O/islands.err; exit 1; }
done
echo islands done
exit 0
fi
timeout -k 5 60 build/examples/e1_onemax_float 200 > $O/e1_fnptr.log 2>&1 || { cat $O/e1_fnptr.log; exit 1; }
head -1 $O/e1_fnptr.log
PGA_OUT=$O/mig_epoch.json timeout -k 10 200 python bench/migration_cost.py > $O/mig_epoch.log 2>&1 || { tail -20 $O/mig_epoch.log; exit 1; }
PGA_RCCL_SELF=1 PGA_OUT=$O/mig_rccl_self.json timeout -k 10 400 python bench/migration_cost.py > $O/mig_rccl.log 2>&1 || { tail -20 $O/mig_rccl.log; exit 1; }
timeout -k 10 200 python bench/mig_host_probe.py > $O/mig_host_probe.json 2> $O/mig_host_probe.err || { tail -20 $O/mig_host_probe.err; exit 1; }
tail -1 $O/mig_host_probe.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_headline --output-format csv -o run -- \
  python3 $R/bench.py --steps 100 --warmup 10 > $O/prof_headline.log 2>&1 || { tail -20 $O/prof_headline.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mig --output-format csv -o run -- python3 $R/bench/migration_cost.py > $O/prof_mig.log 2>&1 || { tail -20 $O/prof_mig.log; exit 1; }
for c in onemax1024_rank onemax1024_roulette_2pt rastrigin30 rastrigin30_rot e1_sum100_refops tsp256_pmx; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c --output-format csv -o run -- \
    python3 $R/bench/bench_configs.py --only "$c" > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 1; }
done
echo all done
