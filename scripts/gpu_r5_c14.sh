#!/bin/bash
# r5: k_ranges folded into the route's last block + fp32 partials from 1M rows: tests, A/B, sequences
set -o pipefail
O=gpurun_out/r5/c14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/fused_$i.log 2>&1 || { cat $O/fused_$i.log; exit 1; }; tail -1 $O/fused_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
  H2O_ROUTE_RANGES=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/sep_$i.log 2>&1 || { cat $O/sep_$i.log; exit 1; }; tail -1 $O/sep_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
done
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/b1375_$i.log 2>&1 || { cat $O/b1375_$i.log; exit 1; }; tail -1 $O/b1375_$i.log | grep -o '"ms_per_step[^,]*'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
rm -rf $O/db
head -3 $O/tree_sequence.md; grep -E "route|ranges" $O/tree_sequence.md
timeout -k 10 300 python3 scripts/fit_profile.py --which gbm > $O/gbm_profile.log 2>&1 || { tail -30 $O/gbm_profile.log; exit 1; }; head -4 $O/gbm_profile.log
