#!/bin/bash
# migration A/B on one GPU (RCCL self-exchange through bench.py): lag, where the epoch's
# selection runs (transport / compute stream), top-k keys per thread
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, problem, env...
  local name=$1 p=$2; shift 2
  env "$@" MASTER_PORT=$((20000 + RANDOM % 20000)) timeout -k 10 120 python bench.py --rccl-self --problem $p --steps 300 --warmup 20 > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step']*1e3,2), 'us/gen', d['migrations_timed'], d['migrations_expected'])"
}
timeout -k 10 120 python bench.py --steps 300 --warmup 20 > $O/nomig.log 2>&1 && grep '^{' $O/nomig.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('onemax nomig', round(d['ms_per_step']*1e3,2))"
for lag in 2 3; do for where in transport compute; do for kpt in 16 64; do
  extra=""; [ $where = compute ] && extra="PGA_MIG_ON_COMPUTE=1"
  run om_l${lag}_${where}_k$kpt onemax PGA_MIG_LAG=$lag PGA_TOPK_KPT=$kpt $extra || exit 1
done; done; done
for p in rastrigin30 tsp256; do
  timeout -k 10 120 python bench.py --problem $p --steps 300 --warmup 20 > $O/nomig_$p.log 2>&1 && grep '^{' $O/nomig_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p nomig', round(d['ms_per_step']*1e3,2))"
  for kpt in 16 64; do run ${p}_l3_transport_k$kpt $p PGA_MIG_LAG=3 PGA_TOPK_KPT=$kpt || exit 1; run ${p}_l3_compute_k$kpt $p PGA_MIG_LAG=3 PGA_TOPK_KPT=$kpt PGA_MIG_ON_COMPUTE=1 || exit 1; done
done
