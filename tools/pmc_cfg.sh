#!/bin/bash
# PMC sets for selected bench_configs entries: tools/pmc_cfg.sh "<configs>" "<set1>" "<set2>" ...
# (kernel-trace only; outputs gpurun_out/pmc_cfg/set*/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
O="$R/gpurun_out/pmc_cfg"; rm -rf "$O"; mkdir -p "$O"
CFG=$1; shift
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/set$i" -o run -- \
    python3 "$R/bench/bench_configs.py" --only $CFG --scale 0.05 > "$O/set$i.log" 2>&1 || { tail -20 "$O/set$i.log"; exit 1; }
done
python3 "$R/tools/prof_summary.py" pmc "$O" > "$O/summary.md"
echo pmc_cfg done
