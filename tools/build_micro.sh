#!/bin/bash
# Standalone roofline microbenchmarks (bench/micro/*.hip -> build/micro/<name>):
# gather (random-row gather floor), tourn_t (transposed-tournament floor),
# alu_rate (integer op issue rates), lds_occupancy.  No library code involved.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/micro
for f in bench/micro/*.hip; do
  hipcc -O3 --offload-arch=gfx950 "$f" -o "build/micro/$(basename "$f" .hip)" &
done
wait
ls build/micro
