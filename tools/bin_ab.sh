#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_binary.py -m gpu -q -x -k "bitexact or pipeline" > gpurun_out/bin_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bin_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --steps 1000 --warmup 100 | cut -c1-200 || exit 1; done
