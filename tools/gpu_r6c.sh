#!/bin/bash
# migration epoch kernel traces: onemax / rastrigin30 / tsp256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
for p in onemax rastrigin30 tsp256; do
  PGA_MIG_PROBLEM=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$p -o mig -- python bench/migration_cost.py > $O/prof_$p.log 2>&1 || { tail -20 $O/prof_$p.log; exit 1; }
  grep '^{' $O/prof_$p.log | tail -1
  f=$(find $O/prof_$p -name "*kernel_stats.csv" | head -1); cp "$f" $O/mig_${p}_kernel_stats.csv
done
