#!/bin/bash
# branch-free TSP breed step + migration work on the transport stream: tests, configs, migration
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py tests/test_gpu_binary.py tests/test_fused_hist.py tests/test_parallel.py tests/test_local_islands.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench/bench_configs.py --only tsp256_ox tsp256_pmx tsp256_int_ox tsp256_euc_ox tsp256_asym_ox --out $O/configs.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
python -c "import json; [print(r['config'], round(r['ms_per_gen']*1e3,1), 'us/gen', round(r['gens_per_sec'])) for r in json.load(open('$O/configs.json'))]"
for p in onemax rastrigin30 tsp256; do
  MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 > $O/bench_self_$p.log 2>&1 || { tail -20 $O/bench_self_$p.log; exit 1; }
  grep '^{' $O/bench_self_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'self', round(d['ms_per_step']*1e3,2), 'us/gen', d['transport'], d['migrations_timed'], d['migrations_expected'])"
  timeout -k 10 120 python bench.py --problem $p --steps 300 --warmup 20 > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  grep '^{' $O/bench_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'nomig', round(d['ms_per_step']*1e3,2), 'us/gen')"
done
