#!/bin/bash
# persistent multi-generation headline launch: bit-exact tests, then an interleaved A/B of the driver's bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_binary.py -k "persistent or headline_geometry" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AB_TIMEOUT=120 tools/ab.sh 3 "python bench.py --steps 20 --warmup 5 | python -c 'import json,sys; print(\"multi 20\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" \
  "PGA_TP_MULTI=0 python bench.py --steps 20 --warmup 5 | python -c 'import json,sys; print(\"plain 20\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" \
  "python bench.py --steps 500 --warmup 50 | python -c 'import json,sys; print(\"multi 500\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" \
  "PGA_TP_MULTI=0 python bench.py --steps 500 --warmup 50 | python -c 'import json,sys; print(\"plain 500\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" | tee $O/ab.txt || exit 1
for v in 1 0; do
  PGA_TP_MULTI=$v MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --steps 300 --warmup 20 > $O/self_$v.log 2>&1 || { tail -20 $O/self_$v.log; exit 1; }
  grep '^{' $O/self_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('self multi=$v', round(d['ms_per_step']*1e3,2), d['migrations_timed'], d['migrations_expected'])"
done
