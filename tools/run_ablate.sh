#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2; do
  for n in ${ABL:-0 1 2 4 8 7 15}; do
    echo "abl=$n round=$r $(timeout -k 5 60 ./build/micro/gen_abl$n --gens ${GENS:-300} ${ARGS:-})" || exit 1
  done
done
