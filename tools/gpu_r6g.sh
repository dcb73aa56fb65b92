#!/bin/bash
# migration lag 2 + spin poll: island tests, bench rccl-self per problem, one timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parallel.py tests/test_fused_hist.py tests/test_capi_comm.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in onemax rastrigin30 tsp256; do
  MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 > $O/bench_self_$p.log 2>&1 || { tail -20 $O/bench_self_$p.log; exit 1; }
  grep '^{' $O/bench_self_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'self', round(d['ms_per_step']*1e3,2), 'us/gen', d['transport'], d['migrations_timed'], d['migrations_expected'])"
  timeout -k 10 120 python bench.py --problem $p --steps 300 --warmup 20 > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  grep '^{' $O/bench_$p.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', 'nomig', round(d['ms_per_step']*1e3,2), 'us/gen')"
done
MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl -- python bench.py --rccl-self --problem onemax --steps 60 --warmup 20 > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
f=$(find $O/tl -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
