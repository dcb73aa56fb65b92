#!/bin/bash
# islands after the block-size rule of the TSP table path; perm tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py tests/test_local_islands.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
rm -f $O/islands.jsonl
timeout -k 10 200 python bench/bench_islands.py --problem tsp128 > $O/islands_tsp128.log 2>&1 || { tail -20 $O/islands_tsp128.log; exit 1; }
grep '^{' $O/islands_tsp128.log
timeout -k 10 200 python bench/bench_configs.py --only tsp256_ox tsp256_pmx --out $O/cfg.json > $O/cfg.log 2>&1 || { tail -20 $O/cfg.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$O/cfg.json')): print(r['config'], round(r['gens_per_sec']))"
