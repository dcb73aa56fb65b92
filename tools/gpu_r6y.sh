#!/bin/bash
# roulette: covered guide buckets (no cumfit load); correctness, A/B vs PGA_ROUL_PACKED=0, kernel split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r6u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ -k "roulette or rank or headline_geometry or graph or real or perm" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  PGA_ROUL_PACKED=0 timeout -k 10 150 python bench/bench_configs.py --only onemax1024_roulette_2pt --out $O/off$i.json > $O/off$i.log 2>&1 || { tail -20 $O/off$i.log; exit 1; }
  timeout -k 10 150 python bench/bench_configs.py --only onemax1024_roulette_2pt --out $O/on$i.json > $O/on$i.log 2>&1 || { tail -20 $O/on$i.log; exit 1; }
  tail -1 $O/off$i.log; tail -1 $O/on$i.log
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o roul -- python3 $GRAFT_REPO_ROOT/bench/bench_configs.py --only onemax1024_roulette_2pt --scale 0.3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
