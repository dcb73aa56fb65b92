#!/bin/bash
# RCCL self-exchange migration overhead (bench/migration_cost.py) plus a
# kernel trace of the same run; outputs under gpurun_out/mig/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/mig"
cd /tmp; export TMPDIR=/tmp
PGA_RCCL_SELF=1 PGA_OUT="$R/gpurun_out/mig/overhead.json" timeout -k 10 240 python3 "$R/bench/migration_cost.py" > "$R/gpurun_out/mig/run.log" 2>&1 || { tail -20 "$R/gpurun_out/mig/run.log"; exit 1; }
cat "$R/gpurun_out/mig/overhead.json"
PGA_RCCL_SELF=1 PGA_OUT="$R/gpurun_out/mig/overhead_traced.json" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/mig/trace" -o run -- python3 "$R/bench/migration_cost.py" > "$R/gpurun_out/mig/trace.log" 2>&1 || { tail -20 "$R/gpurun_out/mig/trace.log"; exit 1; }
