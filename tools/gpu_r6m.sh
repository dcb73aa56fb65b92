#!/bin/bash
# headline A/B: non-temporal child stores, persistent launch; plus the persistent bit-exact test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_binary.py -k "persistent or headline_geometry" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
j() { python -c "import json,sys; print('$1', json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step']*1e3)"; }
export -f j
AB_TIMEOUT=120 tools/ab.sh 3 "python bench.py --steps 500 --warmup 50 | j base" \
  "PGA_TP_NT_STORE=1 python bench.py --steps 500 --warmup 50 | j ntstore" \
  "PGA_TP_MULTI=1 PGA_TP_NT_STORE=1 python bench.py --steps 500 --warmup 50 | j multi_nt" | tee $O/ab.txt || exit 1
