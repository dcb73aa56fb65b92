#!/bin/bash
# run build/micro/<prefix>* variants interleaved, 2 rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2; do
  for b in build/micro/${PREFIX:-gen_cache}*; do
    echo "$(basename $b) r$r $(timeout -k 5 60 $b --gens ${GENS:-300} ${ARGS:-})" || exit 1
  done
done
