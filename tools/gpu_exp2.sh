#!/bin/bash
# Round-3 batch 2: GPU tests of the REAL / roulette changes, the configs they
# touch, then the headline variants (tools/variants.sh) with phase clocks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-exp2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_real.py tests/test_gpu_binary.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot onemax1024 onemax1024_roulette_2pt onemax1024_rank knapsack1024 > $O/configs.log 2>&1 || { cat $O/configs.log; exit 1; }
cat $O/configs.log
V=build/variants
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_base" "$V/gen_w4" > $O/headline_ab.txt 2>&1
rc=$?; cat $O/headline_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 $V/gen_timing --gens 100 > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
cat $O/timing.txt
