#!/bin/bash
# rocprofv3 kernel stats of each named BASELINE config in its own run
# (bench/bench_configs.py --only NAME), plus the headline phase clocks
# (build/variants/gen_timing from tools/variants.sh "timing:-DPGA_TP_TIMING").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-profcfg}"; mkdir -p "$O"
if [ -x "$R/build/variants/gen_timing" ]; then
  timeout -k 10 120 "$R/build/variants/gen_timing" --gens 100 > "$O/timing.txt" 2>&1 || { cat "$O/timing.txt"; exit 1; }
  tail -12 "$O/timing.txt"
fi
for c in ${CFG:-onemax1024_rank onemax1024_roulette_2pt rastrigin30 rastrigin30_rot tsp256_ox tsp256_pmx onemax1024_jit}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$c" -o run -- \
    python3 "$R/bench/bench_configs.py" --only $c --scale ${SCALE:-0.3} > "$O/$c.log" 2>&1 || { tail -20 "$O/$c.log"; exit 1; }
  tail -1 "$O/$c.log"
  python3 "$R/tools/prof_summary.py" stats "$O/$c/run_kernel_stats.csv" 2>/dev/null | head -12 || true
done
