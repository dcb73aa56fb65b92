#!/bin/bash
# TSP FULL variants: bit-exact tests, A/B vs the general variants; counter list for the headline PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py tests/test_local_islands.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in full general full; do
  extra=""; [ $v = general ] && extra="PGA_PERM_NO_FULL=1"
  env $extra timeout -k 10 300 python bench/bench_configs.py --only tsp256_ox tsp256_pmx tsp256_int_ox tsp256_int_pmx --out $O/configs_$v.json > $O/configs_$v.log 2>&1 || { tail -20 $O/configs_$v.log; exit 1; }
  python -c "import json; [print('$v', r['config'], round(r['ms_per_gen']*1e3,1), 'us/gen', round(r['gens_per_sec'])) for r in json.load(open('$O/configs_$v.json'))]"
done
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -oE "TCC_EA0_[A-Z_0-9]+|TCC_BUBBLE[A-Z_0-9]*|TCC_EA_[A-Z_0-9]+" $O/counters.txt | sort -u | head -40
