#!/bin/bash
# One gpurun session: GPU tests, smoke, short bench, all BASELINE configs,
# the reference-semantics baseline, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
if [ "$STEP" = "all" ] || [ "$STEP" = "tests" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --maxfail=10 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "smoke" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-500} --warmup 50 > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
  cat gpurun_out/bench.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "configs" ]; then
  timeout -k 10 600 python bench/bench_configs.py --out gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { cat gpurun_out/configs.log; exit 1; }
  cat gpurun_out/configs.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "refsem" ]; then
  : > gpurun_out/refsem.log
  timeout -k 10 300 build/bench/refsem --objective onemax --pop 1048576 --length 1024 --gens 2 --warmup 1 >> gpurun_out/refsem.log 2>&1 &&
  timeout -k 10 300 build/bench/refsem --objective rastrigin --pop 1048576 --length 30 --gens 3 --warmup 1 >> gpurun_out/refsem.log 2>&1 &&
  timeout -k 10 300 build/bench/refsem --objective sum --pop 40000 --length 100 --gens 20 --warmup 2 >> gpurun_out/refsem.log 2>&1 &&
  timeout -k 10 300 build/bench/refsem --objective onemax --pop 1024 --length 64 --gens 50 --warmup 2 >> gpurun_out/refsem.log 2>&1
  rc=$?; cat gpurun_out/refsem.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "prof" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" --output-format csv -o run -- python3 "$R/bench.py" --steps 100 --warmup 10 > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  find "$R/gpurun_out/prof" -name "*kernel_stats.csv" | head -3
fi
