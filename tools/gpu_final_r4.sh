#!/bin/bash
# Round-4 closing measurements (one call): smoke, driver-shape bench, headline
# phase clocks, every BASELINE config, batched islands, kernel traces of the
# headline and the rank / roulette / JIT / E2 configs, migration cost and the
# Python migration-epoch host probe.  Each GPU step has its own limit; the
# chain stops at the first failure.  -> gpurun_out/final/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 50 > $O/bench500.log 2>&1 || { cat $O/bench500.log; exit 1; }
tail -1 $O/bench500.log
if [ -x build/variants/gen_timing ]; then
  timeout -k 10 120 build/variants/gen_timing --gens 100 > $O/timing.json 2>&1 || { cat $O/timing.json; exit 1; }
fi
timeout -k 10 900 python bench/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
echo configs done
for p in onemax rastrigin30 tsp128; do
  timeout -k 10 200 python bench/bench_islands.py --problem $p >> $O/islands.jsonl 2>> $O/islands.err || { tail -20 $O/islands.err; exit 1; }
done
echo islands done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_headline" --output-format csv -o run -- \
  python3 "$R/bench.py" --steps 100 --warmup 10 > "$R/$O/prof_headline.log" 2>&1 || { tail -20 "$R/$O/prof_headline.log"; exit 1; }
for c in onemax1024_rank onemax1024_roulette_2pt onemax1024_jit rastrigin30_jit e2_knap_refops e1_sum100_refops; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$c" --output-format csv -o run -- \
    python3 "$R/bench/bench_configs.py" --only "$c" > "$R/$O/prof_$c.log" 2>&1 || { tail -20 "$R/$O/prof_$c.log"; exit 1; }
done
echo profiles done
cd "$R"
PGA_OUT=$O/mig_epoch.json timeout -k 10 120 python bench/migration_cost.py > $O/mig_epoch.log 2>&1 || { tail -20 $O/mig_epoch.log; exit 1; }
PGA_RCCL_SELF=1 PGA_OUT=$O/mig_rccl_self.json timeout -k 10 240 python bench/migration_cost.py > $O/mig_rccl.log 2>&1 || { tail -20 $O/mig_rccl.log; exit 1; }
timeout -k 10 200 python bench/mig_host_probe.py > $O/mig_host_probe.json 2> $O/mig_host_probe.err || { tail -20 $O/mig_host_probe.err; exit 1; }
echo all done
