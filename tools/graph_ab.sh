set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_graph.py tests/test_gpu_binary.py tests/test_real.py tests/test_perm.py -m gpu -q -x > gpurun_out/graph_tests.log 2>&1; rc=$?; tail -3 gpurun_out/graph_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== graph off"; PGA_GRAPH=0 timeout -k 10 300 python bench/bench_configs.py --only e2_knap_refops onemax64_gpu e1_sum100_refops || exit 1
echo "== graph on"; timeout -k 10 300 python bench/bench_configs.py --only e2_knap_refops onemax64_gpu e1_sum100_refops || exit 1
