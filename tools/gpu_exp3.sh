#!/bin/bash
# Round-3 batch 3: GPU tests of the dynamic work units and the native radix
# sort, the configs they touch, then unit-size / static A/B (tools/variants.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-exp3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_real.py tests/test_gpu_binary.py tests/test_local_islands.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python bench/bench_configs.py --only onemax1024 rastrigin30 rastrigin30_rot onemax1024_roulette_2pt onemax1024_rank knapsack1024 > $O/configs.log 2>&1 || { cat $O/configs.log; exit 1; }
cat $O/configs.log
V=build/variants
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_base" "PGA_TP_STATIC=1 $V/gen_base" "$V/gen_u64" "$V/gen_u256" "$V/gen_w4" "$V/gen_u64w4" > $O/headline_ab.txt 2>&1
rc=$?; cat $O/headline_ab.txt; [ $rc -ne 0 ] && exit $rc
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_rbase --encoding real --pop 1048576 --length 30" "PGA_TP_STATIC=1 $V/gen_rbase --encoding real --pop 1048576 --length 30" "$V/gen_ru64 --encoding real --pop 1048576 --length 30" "$V/gen_ru256 --encoding real --pop 1048576 --length 30" > $O/real_ab.txt 2>&1
rc=$?; cat $O/real_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 $V/gen_timing --gens 100 > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
tail -40 $O/timing.txt
