#!/bin/bash
# L2 hit/miss of the GEN kernel: tournament vs rank vs roulette selection (OneMax-1024, pop 1M)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/r6w; mkdir -p $O
for c in onemax1024 onemax1024_rank onemax1024_roulette_2pt; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex binary_gen_tp --output-format csv -d "$O/$c" -o run -- \
    python3 "$R/bench/bench_configs.py" --only $c --scale 0.2 > "$O/$c.log" 2>&1) || { tail -20 "$O/$c.log"; exit 1; }
  echo "$c done"
done
