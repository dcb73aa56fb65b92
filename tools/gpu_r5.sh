#!/bin/bash
# Round-5 iteration session: headline kernel alone (no torch), its phase
# clocks, PMC passes of the headline geometry (one counter set per run),
# driver-shape bench, then GPU tests.  Each GPU step has its own time limit;
# the chain stops at the first failure.
#   TAG=r5a tools/gpu_r5.sh      PMC=0 skips the counter passes,
#   TESTS="tests/x.py ..." picks tests (none: skip), EXTRA="cmd" runs before the tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r5}; mkdir -p $O
for v in ${VARIANTS:-base}; do
  if [ -x build/variants/gen_$v ]; then
    timeout -k 10 60 build/variants/gen_$v --gens ${GENS:-300} --warmup 20 > $O/gen_$v.json 2>&1 || { cat $O/gen_$v.json; exit 1; }
    echo "gen_$v: $(head -1 $O/gen_$v.json)"
  fi
done
if [ -x build/variants/gen_timing ]; then
  timeout -k 10 120 build/variants/gen_timing --gens 100 > $O/timing.json 2>&1 || { cat $O/timing.json; exit 1; }
  cat $O/timing.json
fi
if [ "${PMC:-1}" = 1 ] && [ -x build/variants/gen_base ]; then
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "TCC_REQ_sum TCC_READ_sum TCC_WRITE_sum TCC_EA0_RDREQ_32B_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
             "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/pmc/set$i" -o run -- \
      "$R/build/variants/gen_base" --gens 20 --warmup 2 > "$O/pmc_set$i.log" 2>&1) || { tail -20 "$O/pmc_set$i.log"; exit 1; }
  done
  python3 tools/prof_summary.py pmc "$O/pmc" > "$O/pmc_summary.md" && echo pmc done
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
  tail -1 $O/bench20.log
  timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 50 > $O/bench500.log 2>&1 || { cat $O/bench500.log; exit 1; }
  tail -1 $O/bench500.log
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 900 bash -c "$EXTRA" > $O/extra.log 2>&1 || { tail -30 $O/extra.log; exit 1; }
  tail -30 $O/extra.log
fi
T=${TESTS:-tests}
[ "$T" = none ] && exit 0
timeout -k 10 1000 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; exit $rc
