#!/bin/bash
# final-tree kernel split of the driver-shape headline bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
O=$R/gpurun_out/r6z; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o head -- python3 $R/bench.py --gpus 1 --steps 50 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof ok
