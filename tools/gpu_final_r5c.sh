#!/bin/bash
# round-5 closing pass after the TSP kernel: GPU tests, islands, every config, bench.py, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final5c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for p in tsp128 onemax rastrigin30; do
  timeout -k 10 200 python bench/bench_islands.py --problem $p > $O/islands_$p.log 2>&1 || { tail -20 $O/islands_$p.log; exit 1; }
  grep '^{' $O/islands_$p.log >> $O/islands.jsonl
done
timeout -k 10 600 python bench/bench_configs.py --out $O/configs.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 500 --warmup 20 > $O/bench500.log 2>&1 || { tail -20 $O/bench500.log; exit 1; }
tail -1 $O/bench20.log; tail -1 $O/bench500.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
