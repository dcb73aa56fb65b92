#!/bin/bash
# REAL two-phase kernel fixed-cost probes (tools/variants.sh real.hip builds):
# gen_rbase (as shipped), gen_rp0 (prologue only), gen_rp1 (+ first round's
# tournaments), gen_rp2 (no epilogue), E1-shaped populations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/rprobe; mkdir -p $O
for v in rbase rp0 rp1 rp2; do
  for S in 512 4096 40000; do
    echo -n "{\"variant\": \"$v\", " >> $O/probe.jsonl
    timeout -k 10 60 build/variants/gen_$v --encoding real --length 100 --objective 22 --xo uniform --mutation reset_one \
      --lo 0 --hi 1 --elitism 0 --pop $S --gens 300 --warmup 30 | tail -1 | cut -c2- >> $O/probe.jsonl || exit 1
  done
done
cat $O/probe.jsonl
