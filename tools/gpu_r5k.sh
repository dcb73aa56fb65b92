#!/bin/bash
# Round-5 check: smoke, fused-histogram + RCCL engine-transport tests, the
# whole GPU suite, driver-shape bench, migration cost (device epoch and RCCL
# self-exchange overhead per transport), the migration host probe, E1 fn-ptr.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5k}; mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest ${FIRST:-tests/test_fused_hist.py tests/test_parallel.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_first.log 2>&1 || { tail -30 $O/pytest_first.log; exit 1; }
tail -2 $O/pytest_first.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { cat $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
PGA_OUT=$O/mig_epoch.json timeout -k 10 200 python bench/migration_cost.py > $O/mig_epoch.log 2>&1 || { tail -20 $O/mig_epoch.log; exit 1; }
cat $O/mig_epoch.json
PGA_RCCL_SELF=1 PGA_OUT=$O/mig_rccl_self.json timeout -k 10 400 python bench/migration_cost.py > $O/mig_rccl.log 2>&1 || { tail -20 $O/mig_rccl.log; exit 1; }
cat $O/mig_rccl_self.json
timeout -k 10 200 python bench/mig_host_probe.py > $O/mig_host_probe.json 2> $O/mig_host_probe.err || { tail -20 $O/mig_host_probe.err; exit 1; }
tail -1 $O/mig_host_probe.json
[ "${FULL:-1}" = 1 ] || exit 0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; exit $rc
