#!/bin/bash
# round-6 opening pass: driver-shape bench, migration epoch + RCCL-self overhead baselines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 120 python bench/migration_cost.py > $O/mig.log 2>&1 || { tail -20 $O/mig.log; exit 1; }
tail -1 $O/mig.log
PGA_RCCL_SELF=1 PGA_OUT=$O/rccl_self.json timeout -k 10 200 python bench/migration_cost.py > $O/rself.log 2>&1 || { tail -20 $O/rself.log; exit 1; }
cat $O/rccl_self.json
