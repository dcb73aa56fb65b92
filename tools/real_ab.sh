#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_real.py tests/test_capi.py tests/test_jit.py -m gpu -q -x > gpurun_out/real_tests.log 2>&1; rc=$?; tail -3 gpurun_out/real_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "PGA_REAL_PIPE=0" "PGA_REAL_PIPE=1"; do
  echo "== $v"; env $v timeout -k 10 300 python bench/bench_configs.py --only rastrigin30 e1_sum100_refops --scale 0.5 | cut -c1-220 || exit 1
done
