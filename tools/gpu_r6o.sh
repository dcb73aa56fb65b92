#!/bin/bash
# rotation through MFMA with the matrix as A: REAL tests, rastrigin30 / rastrigin30_rot configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_real.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
timeout -k 10 200 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot > $O/cfg_$r.log 2>&1 || { tail -20 $O/cfg_$r.log; exit 1; }
grep '^{' $O/cfg_$r.log | python -c "import json,sys; [print(d['config'], round(d['ms_per_gen']*1e3,2)) for d in map(json.loads, sys.stdin)]"
done
