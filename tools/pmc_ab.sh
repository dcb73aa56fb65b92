#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
for v in pd1 seg4w5; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/pmc_$v" -o run -- "$R/build/variants/gen_$v" --gens 20 --warmup 2 > "$R/gpurun_out/pmc_$v.log" 2>&1 || exit 1
done
