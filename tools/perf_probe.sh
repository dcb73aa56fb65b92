#!/bin/bash
# quick perf probes: GPU tests (subset), migration device cost, JIT eval, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x ${PROBE_K:+-k "$PROBE_K"} > gpurun_out/probe_tests.log 2>&1; rc=$?; tail -3 gpurun_out/probe_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/migration_cost.py > gpurun_out/migration_cost.json 2>gpurun_out/migration_cost.err || { cat gpurun_out/migration_cost.err; exit 1; }
cat gpurun_out/migration_cost.json; PGA_LOOPBACK=1 timeout -k 10 300 python bench/migration_cost.py || exit 1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/probe" -o run -- python3 "$R/bench/migration_cost.py" > "$R/gpurun_out/probe.log" 2>&1 || { tail -20 "$R/gpurun_out/probe.log"; exit 1; }


python3 "$R/tools/prof_summary.py" stats "$R/gpurun_out/probe/run_kernel_stats.csv"

