#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
PGA_PERM_FAST=1 timeout -k 10 600 python -m pytest tests/test_perm.py -m gpu -q -x > gpurun_out/perm_tests.log 2>&1; rc=$?; tail -3 gpurun_out/perm_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "PGA_PERM_FAST=1"; do
  echo "== $v"; env $v timeout -k 10 300 python bench/bench_configs.py --only tsp256_ox tsp256_pmx tsp256_euc_ox tsp256_euc_pmx --scale 0.5 | cut -c1-220 || exit 1
done
