#!/bin/bash
# r5: AUTO root pass from 16-bit fine planes (k_hist_root16) — decision tests, AUTO bench, tree sequence
set -o pipefail
O=gpurun_out/r5/c24
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py -m gpu > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -40; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job --histogram-type AUTO > $O/auto$i.log 2>&1 || { cat $O/auto$i.log; exit 1; }; tail -1 $O/auto$i.log | cut -c1-200; done
H2O_HIST_ROOT16=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job --histogram-type AUTO > $O/auto_off.log 2>&1 || { cat $O/auto_off.log; exit 1; }; tail -1 $O/auto_off.log | cut -c1-200
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/qg.log 2>&1 || { cat $O/qg.log; exit 1; }; tail -1 $O/qg.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --histogram-type AUTO > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/auto_tree_sequence.md || exit 1
rm -rf $O/db
cat $O/auto_tree_sequence.md
