#!/bin/bash
# Round-4 A/B of headline-kernel variants (build/variants/gen_*, tools/variants.sh
# on binary_gs.hip): interleaved rounds (tools/ab.sh) of $ARMS (";"-separated
# commands), then the phase clocks of $TIMING (";"-separated commands).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
V=build/variants
IFS=';' read -ra arms <<< "${ARMS:-$V/gen_base --gens 300;PGA_TP_POOL=0 $V/gen_base --gens 300;PGA_TP_POOL=4 $V/gen_base --gens 300;$V/gen_pd1 --gens 300}"
AB_TIMEOUT=60 tools/ab.sh ${ROUNDS:-3} "${arms[@]}" || exit 1
IFS=';' read -ra tims <<< "${TIMING:-$V/gen_t --gens 100;PGA_TP_POOL=0 $V/gen_t --gens 100;PGA_TP_POOL=0 $V/gen_swapt --gens 100}"
for t in "${tims[@]}"; do
  echo "== $t"
  timeout -k 10 60 bash -c "$t" || exit 1
done
