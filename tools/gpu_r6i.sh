#!/bin/bash
# migration A/B after the fence fix: lag 2/3 x transport/compute, every problem (RCCL self-exchange)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, problem, env...
  local name=$1 p=$2; shift 2
  env "$@" MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step']*1e3,2), 'us/gen', d['migrations_timed'], d['migrations_expected'])"
}
for p in onemax rastrigin30 tsp256; do
  timeout -k 10 120 python bench.py --problem $p --steps 300 --warmup 20 > $O/nomig_$p.log 2>&1 && grep '^{' $O/nomig_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p nomig', round(d['ms_per_step']*1e3,2))"
  for lag in 2 3; do
    run ${p}_l${lag}_transport $p PGA_MIG_LAG=$lag || exit 1
    run ${p}_l${lag}_compute $p PGA_MIG_LAG=$lag PGA_MIG_ON_COMPUTE=1 || exit 1
  done
done
