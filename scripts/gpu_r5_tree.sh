#!/bin/bash
# r5: tree-engine GPU tests + driver-window headline bench (+ optional rocprof tree sequence)
set -o pipefail
O=gpurun_out/r5/${TAG:-tree}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/bench$i.log 2>&1 || { cat $O/bench$i.log; exit 1; }; tail -1 $O/bench$i.log | cut -c1-400; done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/bench1375k.log 2>&1 || { cat $O/bench1375k.log; exit 1; }
tail -1 $O/bench1375k.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
rm -rf $O/db
cat $O/tree_sequence.md
