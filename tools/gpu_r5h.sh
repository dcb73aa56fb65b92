set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O
timeout -k 5 60 build/examples/e1_onemax_float 200 || exit 1
PGA_TP_MIN_S=1000000000 timeout -k 5 60 build/examples/e1_onemax_float 200 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_capi.py tests/test_real.py tests/test_perm.py tests/test_jit.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; exit $rc
