#!/bin/bash
# kernel timeline of the RCCL self-exchange bench (overlap of the epoch's kernels with the generation)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
for m in transport compute; do
  if [ $m = compute ]; then export PGA_MIG_ON_COMPUTE=1; fi
  MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$m -o tl -- python bench.py --rccl-self --problem onemax --steps 60 --warmup 20 > $O/tl_$m.log 2>&1 || { tail -20 $O/tl_$m.log; exit 1; }
  f=$(find $O/tl_$m -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace_$m.csv
  grep '^{' $O/tl_$m.log | tail -1 | cut -c1-200
done
