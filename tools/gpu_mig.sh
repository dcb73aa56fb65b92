#!/bin/bash
# Island-migration cost on one GPU: migration tests, device work per epoch,
# the real RCCL self-exchange overhead, and its
# kernel trace.  Every GPU step has its own limit; the chain stops at the
# first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_binary.py tests/test_parallel.py tests/test_local_islands.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
timeout -k 10 120 python bench/migration_cost.py > gpurun_out/mig_fused.json 2> gpurun_out/mig_fused.err || { tail -20 gpurun_out/mig_fused.err; exit 1; }
cat gpurun_out/mig_fused.json
cd /tmp
PGA_RCCL_SELF=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/migprof2" --output-format csv -o run -- python3 "$R/bench/migration_cost.py" > "$R/gpurun_out/migprof2.log" 2>&1 || { tail -20 "$R/gpurun_out/migprof2.log"; exit 1; }
grep overhead "$R/gpurun_out/migprof2.log"
