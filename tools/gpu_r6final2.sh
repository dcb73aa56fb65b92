#!/bin/bash
# round-6 closing checkpoint: the whole GPU suite, smoke(), the driver-shape bench, every config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r6final2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 900 python bench/bench_configs.py --out $O/configs.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
python -c "import json; [print(r['config'], round(r['ms_per_gen']*1e3,2), 'us/gen', round(r['gens_per_sec'])) for r in json.load(open('$O/configs.json'))]"
