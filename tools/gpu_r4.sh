#!/bin/bash
# Round-4 iteration session: smoke, driver-shaped bench, phase clocks of the
# headline kernel, then the BINARY GPU tests (bit-exact vs the CPU backend).
# Each GPU step has its own time limit; the chain stops at the first failure.
#   TAG=r4a tools/gpu_r4.sh            (TESTS="tests/x.py ..." to pick tests)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4}; mkdir -p $O
if [ -x build/variants/gen_base ]; then  # the headline kernel alone first (no torch import): a hang shows in 60 s
  timeout -k 10 60 build/variants/gen_base --gens 20 --warmup 2 || exit 1
fi
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 50 > $O/bench500.log 2>&1 || { cat $O/bench500.log; exit 1; }
tail -1 $O/bench500.log
if [ -x build/variants/gen_timing ]; then
  timeout -k 10 120 build/variants/gen_timing --gens 100 > $O/timing.json 2>&1 || { cat $O/timing.json; exit 1; }
  cat $O/timing.json
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > $O/extra.log 2>&1 || { tail -30 $O/extra.log; exit 1; }
  tail -30 $O/extra.log
fi
T=${TESTS:-tests/test_gpu_binary.py tests/test_jit.py tests/test_local_islands.py tests/test_graph.py}
[ "$T" = none ] && exit 0
timeout -k 10 1000 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; exit $rc
