#!/bin/bash
# REAL encoding on one MI355X: GPU tests, then the Rastrigin-30D configs and
# their kernel stats.  A test failure (rc 1) still runs the benches; any other
# failure (fault, abort, time limit) ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-real}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_real.py tests/test_capi_comm.py -m gpu -q -x --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -25 "$O/tests.log"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot onemax1024 > "$O/configs.log" 2>&1 || { cat "$O/configs.log"; exit 1; }
cat "$O/configs.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench/bench_configs.py" --only rastrigin30 rastrigin30_rot --scale 0.3 > "$R/$O/prof.log" 2>&1 || { tail -20 "$R/$O/prof.log"; exit 1; }
for f in $(find "$R/$O/prof" -name "*kernel_stats.csv"); do head -8 "$f"; done
