#!/bin/bash
# Extra measurements of a round-4 session (tools/gpu_r4.sh EXTRA=...): the
# REAL size sweep on the default route and with the two-phase kernel forced,
# and the BASELINE configs named in $CFGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 200 python bench/real_size_sweep.py || exit 1
PGA_TP_MIN_S=0 timeout -k 10 200 python bench/real_size_sweep.py || exit 1
if [ -n "$CFGS" ]; then
  timeout -k 10 400 python bench/bench_configs.py --only $CFGS || exit 1
fi
