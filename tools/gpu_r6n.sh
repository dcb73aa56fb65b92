#!/bin/bash
# small REAL populations: two-phase vs generic kernel by population threshold (reference E1 and its fn-ptr build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for th in default 65536; do
  extra=""; [ $th != default ] && extra="PGA_TP_MIN_S=$th"
  env $extra timeout -k 10 120 python bench/bench_configs.py --only e1_sum100_refops rastrigin30 > $O/cfg_$th.log 2>&1 || { tail -20 $O/cfg_$th.log; exit 1; }
  grep '^{' $O/cfg_$th.log | python -c "import json,sys; [print('$th', d['config'], d['pop'], round(d['ms_per_gen']*1e3,2)) for d in map(json.loads, sys.stdin)]"
  env $extra timeout -k 5 60 build/examples/e1_onemax_float 200 > $O/e1_fnptr_$th.log 2>&1 || { cat $O/e1_fnptr_$th.log; exit 1; }
  echo "$th fnptr: $(head -1 $O/e1_fnptr_$th.log)"
done
done
