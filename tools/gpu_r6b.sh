#!/bin/bash
# round 6: new GPU tests (perm sanitize, bench rccl-self), bench rccl-self lines, migration-epoch kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
: timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parallel.py tests/test_perm.py -k "sanitiz or rccl or stream_order" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for p in onemax tsp256 rastrigin30; do
  MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 200 --warmup 20 > $O/bench_self_$p.log 2>&1 || { tail -20 $O/bench_self_$p.log; exit 1; }
  grep '^{' $O/bench_self_$p.log | tail -1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_mig -o mig -- python bench/migration_cost.py > $O/prof_mig.log 2>&1 || { tail -20 $O/prof_mig.log; exit 1; }
find $O/prof_mig -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/mig_kernel_stats.csv
tail -1 $O/prof_mig.log
