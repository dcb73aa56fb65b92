#!/bin/bash
# TSP-256 fast kernel: perm tests, then timing arms (tools/variants.sh csrc/kernels/perm.hip "pbase:")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5p
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py \
  > gpurun_out/r5p/pytest.log 2>&1 || { tail -30 gpurun_out/r5p/pytest.log; exit 1; }
tail -2 gpurun_out/r5p/pytest.log
fi
V=build/variants
P="--encoding perm --length 256 --pop 262144 --gens 100 --warmup 10 --elitism 1"
AB_TIMEOUT=120 tools/ab.sh 2 \
  "$V/gen_pbase $P --tsp f32" "$V/gen_pbase $P --tsp f32 --pmx 1" "PGA_PERM_PMX_TBL=0 $V/gen_pbase $P --tsp f32 --pmx 1" \
  "PGA_TSP_NO_LDS=1 $V/gen_pbase $P --tsp f32" \
  "$V/gen_pbase $P --tsp int --pmx 1" "$V/gen_pbase $P --tsp euc --pmx 1" \
  > gpurun_out/r5p/ab.txt 2>&1 && cat gpurun_out/r5p/ab.txt
