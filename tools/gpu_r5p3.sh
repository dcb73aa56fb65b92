#!/bin/bash
# PMX chain variants (tools/variants.sh csrc/kernels/perm.hip "e0:" "e3:-DPGA_PERM_CHAIN=3")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5p
V=build/variants
P="--encoding perm --length 256 --pop 262144 --gens 100 --warmup 10 --elitism 1"
AB_TIMEOUT=120 tools/ab.sh 2 \
  "$V/gen_e3 $P --tsp f32 --pmx 1" "$V/gen_e0 $P --tsp f32 --pmx 1" "PGA_PERM_PMX_TBL=0 $V/gen_e0 $P --tsp f32 --pmx 1" \
  "$V/gen_e0 $P --tsp int --pmx 1" "$V/gen_e0 $P --tsp euc --pmx 1" "$V/gen_e0 $P --tsp int" "$V/gen_e0 $P --tsp euc" \
  > gpurun_out/r5p/ab3.txt 2>&1 && cat gpurun_out/r5p/ab3.txt
