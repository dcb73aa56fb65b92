#!/bin/bash
# TSP on the select-then-breed fast kernel: GPU tests, TSP configs, kernel traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r5q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench/bench_configs.py --only tsp256_ox tsp256_pmx tsp256_int_ox tsp256_int_pmx tsp256_euc_ox \
  tsp256_euc_pmx tsp256_asym_ox tsp256_asym_pmx --out $O/configs_tsp.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
cat $O/configs_tsp.json
timeout -k 10 200 python bench/bench_islands.py > $O/islands.log 2>&1 || { tail -20 $O/islands.log; exit 1; }
tail -6 $O/islands.log
cd /tmp
for c in tsp256_ox tsp256_pmx; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$c --output-format csv -o run -- \
    python3 $R/bench/bench_configs.py --only "$c" > $R/$O/prof_$c.log 2>&1 || { tail -20 $R/$O/prof_$c.log; exit 1; }
done
echo done
