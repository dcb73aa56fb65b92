#!/bin/bash
# Round-5: rotated-MFMA / roulette checks and kernel traces of the migration
# epoch, the rotated Rastrigin and the roulette config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r5m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_real.py tests/test_gpu_binary.py tests/test_local_islands.py tests/test_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python bench/bench_configs.py --only rastrigin30 rastrigin30_rot onemax1024_roulette_2pt onemax1024_rank e1_sum100_refops > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mig --output-format csv -o run -- python3 $R/bench/migration_cost.py > $O/prof_mig.log 2>&1 || { tail -20 $O/prof_mig.log; exit 1; }
for c in rastrigin30_rot onemax1024_roulette_2pt; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c --output-format csv -o run -- python3 $R/bench/bench_configs.py --only $c > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 1; }
done
echo done
