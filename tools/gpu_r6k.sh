#!/bin/bash
# headline PMC passes (one counter set per run): the L2 -> fabric read / write request sizes, to settle the bytes per generation
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/r6k; mkdir -p $O
i=0
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum SQ_WAVES" \
           "TCC_MISS_sum TCC_REQ_sum SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex binary_gen_tp --output-format csv -d "$O/pmc/set$i" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 > "$O/pmc_set$i.log" 2>&1) || { tail -20 "$O/pmc_set$i.log"; exit 1; }
done
python3 tools/prof_summary.py pmc "$O/pmc" > "$O/pmc_summary.md" && cat "$O/pmc_summary.md"
