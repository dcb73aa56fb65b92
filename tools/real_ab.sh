#!/bin/bash
# REAL GPU tests, then A/B of the REAL GEN kernels on the REAL configs:
# generic fast kernel (PGA_REAL_PIPE=0) vs the pipelined kernel, and the
# 16x16x4 vs 4x4x1 wave-local MFMA rotation tile (PGA_ROT_4X4).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_real.py tests/test_graph.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/real_tests.log 2>&1; rc=$?; tail -3 gpurun_out/real_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in "PGA_REAL_PIPE=0" "PGA_ROT_4X4=0" "PGA_ROT_4X4=1"; do
  echo "== $v"; env $v timeout -k 10 300 python bench/bench_configs.py --only ${CFGS:-rastrigin30_rot} --scale 0.5 | cut -c1-200 || exit 1
done
done
