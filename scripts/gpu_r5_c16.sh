#!/bin/bash
# r5: tree snapshot by kernel into mapped pinned memory vs the runtime D2H copy
set -o pipefail
O=gpurun_out/r5/c16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/k_$i.log 2>&1 || { cat $O/k_$i.log; exit 1; }; tail -1 $O/k_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
  H2O_SNAP_KERNEL=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/c_$i.log 2>&1 || { cat $O/c_$i.log; exit 1; }; tail -1 $O/c_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/kb_$i.log 2>&1 || { cat $O/kb_$i.log; exit 1; }; tail -1 $O/kb_$i.log | grep -o '"ms_per_step[^,]*'
  H2O_SNAP_KERNEL=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/cb_$i.log 2>&1 || { cat $O/cb_$i.log; exit 1; }; tail -1 $O/cb_$i.log | grep -o '"ms_per_step[^,]*'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
rm -rf $O/db
head -3 $O/tree_sequence.md; tail -4 $O/tree_sequence.md
