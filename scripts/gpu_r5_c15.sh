#!/bin/bash
# r5: split search + plan in one launch, leaf-sum finish in the leaf-assign launch: tests, A/B, sequences
set -o pipefail
O=gpurun_out/r5/c15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_kernels_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/fused_$i.log 2>&1 || { cat $O/fused_$i.log; exit 1; }; tail -1 $O/fused_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
  H2O_PLAN_FUSED=0 H2O_LEAF_FUSED=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/sep_$i.log 2>&1 || { cat $O/sep_$i.log; exit 1; }; tail -1 $O/sep_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
done
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/b1375_$i.log 2>&1 || { cat $O/b1375_$i.log; exit 1; }; tail -1 $O/b1375_$i.log | grep -o '"ms_per_step[^,]*'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
rm -rf $O/db
cat $O/tree_sequence.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db2 -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --rows 1375000 > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db2/run_results.db --sequence k_gbm_step > $O/tree_sequence_1375k.md || exit 1
rm -rf $O/db2
head -3 $O/tree_sequence_1375k.md
