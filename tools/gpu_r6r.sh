#!/bin/bash
# early re-scoring of the migrants on the transport stream (PGA_MIG_EVAL_EARLY=1): island tests under it, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
PGA_MIG_EVAL_EARLY=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parallel.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
j() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step']*1e3,2), d['migrations_timed'], d['migrations_expected'])"; }
export -f j
AB_TIMEOUT=120 tools/ab.sh 3 "MASTER_PORT=29711 python bench.py --rccl-self --steps 300 --warmup 20 | j base" \
  "MASTER_PORT=29712 PGA_MIG_EVAL_EARLY=1 python bench.py --rccl-self --steps 300 --warmup 20 | j early" \
  "python bench.py --steps 300 --warmup 20 | python -c 'import json,sys; print(\"nomig\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" | tee $O/ab.txt
for p in rastrigin30 tsp256; do
AB_TIMEOUT=120 tools/ab.sh 1 "MASTER_PORT=29713 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 | j ${p}_base" \
  "MASTER_PORT=29714 PGA_MIG_EVAL_EARLY=1 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 | j ${p}_early" | tee -a $O/ab.txt
done
