#!/bin/bash
# A/B the gen_bench variant binaries build/micro/gen_v* (alternating, 3 rounds)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2 3; do
  for b in ${VARIANTS:-build/micro/gen_v0 build/micro/gen_v1}; do
    echo "$(basename $b) round=$r $(timeout -k 5 60 $b --gens ${GENS:-400} ${ARGS:-})" || exit 1
  done
done
