#!/bin/bash
# rank selection: fused tile counts (GEN kernel -> rank sort) correctness + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r6s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_binary.py tests/test_fused_hist.py -k "headline_geometry or rank or sort or topk or hist" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  PGA_RANK_FUSED=0 timeout -k 10 150 python bench/bench_configs.py --only onemax1024_rank --out $O/off$i.json > $O/off$i.log 2>&1 || { tail -20 $O/off$i.log; exit 1; }
  timeout -k 10 150 python bench/bench_configs.py --only onemax1024_rank --out $O/on$i.json > $O/on$i.log 2>&1 || { tail -20 $O/on$i.log; exit 1; }
  tail -1 $O/off$i.log; tail -1 $O/on$i.log
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o rank -- python3 $GRAFT_REPO_ROOT/bench/bench_configs.py --only onemax1024_rank --scale 0.3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
