#!/bin/bash
# perm tests, then fast-kernel variants (tools/variants.sh csrc/kernels/perm.hip d0/d2/d0n + the previous kernel "old")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py \
  > gpurun_out/r5p/pytest.log 2>&1 || { tail -30 gpurun_out/r5p/pytest.log; exit 1; }
tail -1 gpurun_out/r5p/pytest.log
V=build/variants
P="--encoding perm --length 256 --pop 262144 --gens 100 --warmup 10 --elitism 1 --tsp f32"
AB_TIMEOUT=120 tools/ab.sh 2 \
  "$V/gen_old $P --pmx 1" "$V/gen_d0 $P --pmx 1" "$V/gen_d0n $P --pmx 1" \
  "PGA_PERM_PMX_TBL=0 $V/gen_d0 $P --pmx 1" \
  "$V/gen_old $P" "$V/gen_d0 $P" "$V/gen_d0n $P" "PGA_TSP_NO_LDS=1 $V/gen_d0 $P" \
  > gpurun_out/r5p/ab2.txt 2>&1 && cat gpurun_out/r5p/ab2.txt
