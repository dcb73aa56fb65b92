#!/bin/bash
# Round-3 headline / REAL experiment batch: interleaved A/B of kernel variants
# built by tools/variants.sh (gen_bench against -D variants of one source).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/exp1; mkdir -p $O
V=build/variants
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_base" "$V/gen_timing" "$V/gen_xohash" "$V/gen_nokeys" "$V/gen_w4" "$V/gen_w6" > $O/headline_ab.txt 2>&1
rc=$?; cat $O/headline_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 $V/gen_timing --gens 200 > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
cat $O/timing.txt
RA="--encoding real --length 30 --gens 200"
AB_TIMEOUT=120 bash tools/ab.sh 2 "$V/gen_rbase $RA" "$V/gen_rnoscores $RA" "$V/gen_rblxhash $RA" "$V/gen_rw5 $RA" "$V/gen_rseg2 $RA" > $O/real_ab.txt 2>&1
rc=$?; cat $O/real_ab.txt; exit $rc
