#!/bin/bash
# A/B: generic vs pipelined GEN kernel, interleaved rounds in separate processes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for r in 1 2; do
  for p in 0 1; do
    PGA_PIPELINE=$p timeout -k 10 120 python bench.py --steps ${STEPS:-300} --warmup 30 > gpurun_out/ab_${p}_${r}.json 2>/dev/null || exit 1
    echo "pipe=$p round=$r $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${p}_${r}.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,1),'us/gen', round(d['gens_per_sec']),'gens/s')")"
  done
done
