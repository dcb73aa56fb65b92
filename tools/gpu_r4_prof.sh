#!/bin/bash
# Kernel traces of named BASELINE configs (rocprofv3 --kernel-trace --stats),
# one run each: PROF_CFGS="e2_knap_refops ..." -> gpurun_out/$TAG/prof_<cfg>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r4}
cd /tmp && export TMPDIR=/tmp
for c in ${PROF_CFGS:-e2_knap_refops}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_$c" --output-format csv -o run -- \
    python3 "$R/bench/bench_configs.py" --only "$c" > "$O/prof_$c.log" 2>&1 || { tail -20 "$O/prof_$c.log"; exit 1; }
  tail -1 "$O/prof_$c.log"
done
