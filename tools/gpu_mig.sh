#!/bin/bash
# Island-migration cost on one GPU: device work per epoch, the real RCCL
# self-exchange overhead (clean JSON via PGA_OUT) and its kernel trace.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
PGA_OUT=gpurun_out/mig_epoch.json timeout -k 10 120 python bench/migration_cost.py > gpurun_out/mig_epoch.log 2>&1 || { tail -20 gpurun_out/mig_epoch.log; exit 1; }
cat gpurun_out/mig_epoch.json
PGA_RCCL_SELF=1 PGA_OUT=gpurun_out/mig_rccl_self.json timeout -k 10 240 python bench/migration_cost.py > gpurun_out/mig_rccl.log 2>&1 || { tail -20 gpurun_out/mig_rccl.log; exit 1; }
cat gpurun_out/mig_rccl_self.json
cd /tmp
PGA_RCCL_SELF=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/migprof" --output-format csv -o run -- python3 "$R/bench/migration_cost.py" > "$R/gpurun_out/migprof.log" 2>&1 || { tail -20 "$R/gpurun_out/migprof.log"; exit 1; }
echo migprof done
