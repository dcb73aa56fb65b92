#!/bin/bash
# TSP-256 PMC passes (OX / PMX, FULL variants), then every BASELINE config on one device
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/r6p; mkdir -p $O
for xo in ox pmx; do
  i=0
  for set in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
             "TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex perm_gen_fast --output-format csv -d "$O/pmc_$xo/set$i" -o run -- \
      python3 "$R/bench.py" --problem tsp256 --crossover $xo --steps 20 --warmup 3 > "$O/pmc_${xo}_set$i.log" 2>&1) || { tail -20 "$O/pmc_${xo}_set$i.log"; exit 1; }
  done
  python3 tools/prof_summary.py pmc "$O/pmc_$xo" > "$O/pmc_$xo.md" && tail -3 "$O/pmc_$xo.md"
done
timeout -k 10 900 python bench/bench_configs.py --out $O/configs.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
python -c "import json; [print(r['config'], round(r['ms_per_gen']*1e3,2), 'us/gen', round(r['gens_per_sec'])) for r in json.load(open('$O/configs.json'))]"
