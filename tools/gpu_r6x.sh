#!/bin/bash
# rank scatter / fused roulette with their global loads issued first: correctness + timing + kernel split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r6x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ -k "roulette or rank or headline_geometry or graph or sort or topk" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 150 python bench/bench_configs.py --only onemax1024_rank onemax1024_roulette_2pt --out $O/c$i.json > $O/c$i.log 2>&1 || { tail -20 $O/c$i.log; exit 1; }
done
python -c "import json; [print(r['config'], round(r['ms_per_gen']*1e3,2)) for i in (1,2,3) for r in json.load(open('$O/c%d.json' % i))]"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o rr -- python3 $GRAFT_REPO_ROOT/bench/bench_configs.py --only onemax1024_rank onemax1024_roulette_2pt --scale 0.3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
