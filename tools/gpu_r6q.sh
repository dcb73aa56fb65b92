#!/bin/bash
# two-pass (count + select) vs look-back top-k on the fused histogram: tests under both, migration A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp
PGA_TOPK_2PASS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused_hist.py tests/test_gpu_binary.py -k "fused or topk or migration" > $O/pytest_2pass.log 2>&1 || { tail -40 $O/pytest_2pass.log; exit 1; }
tail -1 $O/pytest_2pass.log
for v in 0 1; do PGA_TOPK_2PASS=$v timeout -k 10 120 python bench/migration_cost.py > $O/mig_$v.log 2>&1 || { tail -20 $O/mig_$v.log; exit 1; }
  grep '^{' $O/mig_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('2pass=$v epoch_device_fused', round(d['epoch_device_fused_us'],1), 'epoch', round(d['epoch_us'],1))"; done
j() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step']*1e3,2), d['migrations_timed'], d['migrations_expected'])"; }
export -f j
AB_TIMEOUT=120 tools/ab.sh 2 "MASTER_PORT=29701 python bench.py --rccl-self --steps 300 --warmup 20 | j lookback" \
  "MASTER_PORT=29702 PGA_TOPK_2PASS=1 python bench.py --rccl-self --steps 300 --warmup 20 | j twopass" \
  "python bench.py --steps 300 --warmup 20 | python -c 'import json,sys; print(\"nomig\", json.loads(sys.stdin.read().strip().splitlines()[-1])[\"ms_per_step\"]*1e3)'" | tee $O/ab.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_perm.py > $O/pytest_perm.log 2>&1 || { tail -40 $O/pytest_perm.log; exit 1; }
tail -1 $O/pytest_perm.log
for r in 1 2; do
timeout -k 10 200 python bench/bench_configs.py --only tsp256_ox tsp256_pmx > $O/tsp_$r.log 2>&1 || { tail -20 $O/tsp_$r.log; exit 1; }
grep '^{' $O/tsp_$r.log | python -c "import json,sys; [print(d['config'], round(d['ms_per_gen']*1e3,2)) for d in map(json.loads, sys.stdin)]"
done
