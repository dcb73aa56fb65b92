#!/bin/bash
# Profile every GPU BASELINE config: kernel stats, then PMC counter sets
# (each set in its own --kernel-trace run; never combined with sys/runtime
# traces).  Outputs under gpurun_out/prof_all/; summarise with
# tools/prof_summary.py and copy into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
O="$R/gpurun_out/prof_all"
mkdir -p "$O"
CFG=${CFG:-"onemax1024 rastrigin30 rastrigin30_rot tsp256_ox tsp256_pmx e1_sum100_refops maxcut512_qubo qubo1024 onemax1024_rank"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/bench/bench_configs.py" --only $CFG --scale 0.2 > "$O/stats.log" 2>&1 || { tail -20 "$O/stats.log"; exit 1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_I8" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/pmc/set$i" -o run -- \
    python3 "$R/bench/bench_configs.py" --only $CFG --scale 0.05 > "$O/pmc_set$i.log" 2>&1 || { tail -20 "$O/pmc_set$i.log"; exit 1; }
done
echo prof_all done
