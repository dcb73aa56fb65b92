set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_real.py tests/test_capi.py -m gpu -q -x > gpurun_out/real_tests.log 2>&1; rc=$?; tail -3 gpurun_out/real_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "PGA_REAL_FAST=0" "PGA_REAL_U=1" "PGA_REAL_U=2" "PGA_REAL_U=4"; do
  echo "== $v"
  env $v timeout -k 10 300 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot e1_sum100_refops --scale 0.5 || exit 1
done
