#!/bin/bash
# PMC passes (kernel-trace only) of the TSP-256 OX / PMX configs, one counter set per run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
O="$R/gpurun_out/pmc_tsp"
mkdir -p "$O"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
S2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for c in tsp256_ox tsp256_pmx; do
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/${c}_set$i" -o run -- \
      python3 "$R/bench/bench_configs.py" --only $c > "$O/${c}_set$i.log" 2>&1 || { tail -20 "$O/${c}_set$i.log"; exit 1; }
  done
done
echo done
