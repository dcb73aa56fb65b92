#!/bin/bash
# Batched vs streamed islands on one device (bench/bench_islands.py), OneMax-1024 and Rastrigin-30.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 120 python bench/bench_islands.py --problem onemax || exit 1
timeout -k 10 120 python bench/bench_islands.py --problem rastrigin30 || exit 1
timeout -k 10 120 python bench/bench_islands.py --problem tsp128 --gens 100 || exit 1
