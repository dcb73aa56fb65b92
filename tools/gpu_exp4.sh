#!/bin/bash
# Round-3 batch 4: age-skewed static shares (tp.hpp tp_cut), PGA_TP_SKEW A/B
# on the headline and Rastrigin configs, phase clocks at the default skew.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-exp4}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_real.py tests/test_gpu_binary.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -gt 1 ] && exit $rc
V=build/variants
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_s0" "$V/gen_s10" "$V/gen_s15" "$V/gen_s20" "$V/gen_s30" > $O/headline_ab.txt 2>&1
rc=$?; cat $O/headline_ab.txt; [ $rc -ne 0 ] && exit $rc
RA="--encoding real --pop 1048576 --length 30"
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_r0 $RA" "$V/gen_r15 $RA" "$V/gen_r25 $RA" > $O/real_ab.txt 2>&1
rc=$?; cat $O/real_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 $V/gen_timing --gens 100 > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
tail -3 $O/timing.txt
timeout -k 10 400 python bench/bench_configs.py --only onemax1024 rastrigin30 rastrigin30_rot onemax1024_roulette_2pt onemax1024_rank > $O/configs.log 2>&1 || { cat $O/configs.log; exit 1; }
cat $O/configs.log
