#!/bin/bash
# Round-4 A/B of headline-kernel variants (build/variants/gen_*, tools/variants.sh):
# interleaved rounds (tools/ab.sh), then the phase clocks of the timing builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
V=build/variants
args=()
for v in ${VARIANTS:-pd1 flags pd3}; do args+=("$V/gen_$v --gens 300"); done
AB_TIMEOUT=60 tools/ab.sh ${ROUNDS:-3} "${args[@]}" || exit 1
for t in ${TIMING:-timing flagst}; do
  timeout -k 10 60 $V/gen_$t --gens 100 || exit 1
done
