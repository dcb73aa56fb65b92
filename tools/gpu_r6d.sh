#!/bin/bash
# f32 radix top-k: GPU tests, then the migration epoch per problem and the bench rccl-self lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_binary.py tests/test_fused_hist.py tests/test_local_islands.py tests/test_parallel.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in onemax rastrigin30 tsp256; do
  PGA_MIG_PROBLEM=$p timeout -k 10 120 python bench/migration_cost.py > $O/mig_$p.log 2>&1 || { tail -20 $O/mig_$p.log; exit 1; }
  grep '^{' $O/mig_$p.log | tail -1
  MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 > $O/bench_self_$p.log 2>&1 || { tail -20 $O/bench_self_$p.log; exit 1; }
  grep '^{' $O/bench_self_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'self', round(d['ms_per_step']*1e3,2), 'us/gen', d['transport'], d['migrations_timed'], d['migrations_expected'])"
  timeout -k 10 120 python bench.py --problem $p --steps 300 --warmup 20 > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  grep '^{' $O/bench_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'nomig', round(d['ms_per_step']*1e3,2), 'us/gen')"
done
