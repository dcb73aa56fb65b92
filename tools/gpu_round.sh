#!/bin/bash
# One round-status gpurun session: GPU tests, smoke, driver-shaped bench,
# every BASELINE config, rocprofv3 kernel stats of bench.py.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-round}; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 50 > $O/bench500.log 2>&1 || { cat $O/bench500.log; exit 1; }
tail -1 $O/bench500.log
timeout -k 10 600 python bench/bench_configs.py ${CFG:+--only $CFG} --out $O/configs.json > $O/configs.log 2>&1 || { cat $O/configs.log; exit 1; }
cat $O/configs.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" --output-format csv -o run -- python3 "$R/bench.py" --steps 100 --warmup 10 > "$R/$O/prof.log" 2>&1 || { tail -30 "$R/$O/prof.log"; exit 1; }
find "$R/$O/prof" -name "*kernel_stats.csv"
