#!/bin/bash
# Interleaved A/B runner: tools/ab.sh ROUNDS "cmd A" "cmd B" [...]
# Runs every command once per round, round-robin (so clock/thermal drift hits
# every arm alike), each under its own time limit; stops at the first failure.
# Example (generic vs fast kernels):
#   tools/ab.sh 3 "python bench.py --steps 300" "PGA_FORCE_GENERIC=1 python bench.py --steps 300"
set -o pipefail
rounds=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "$rounds"); do
  i=0
  for c in "$@"; do
    i=$((i + 1))
    out=$(timeout -k 10 ${AB_TIMEOUT:-300} bash -c "$c" 2>/dev/null | tail -1) || { echo "arm $i failed: $c"; exit 1; }
    echo "round $r arm $i: $out"
  done
done
