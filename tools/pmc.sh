#!/bin/bash
# PMC counter collection (kernel-trace only, never combined with sys/runtime trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters_list.txt" 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc/set$i" -o run -- python3 "$R/bench.py" --steps 30 --warmup 5 > "$R/gpurun_out/pmc/set$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc/set$i.log"; exit 1; }
done
