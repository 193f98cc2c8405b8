#!/bin/bash
# r5: fp32 partial slots at 11M (H2O_PARTIAL_F32=1) A/B after the vectorized flush
set -o pipefail
O=gpurun_out/r5/c13
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/f64_$i.log 2>&1 || { cat $O/f64_$i.log; exit 1; }; tail -1 $O/f64_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
  H2O_PARTIAL_F32=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/f32_$i.log 2>&1 || { cat $O/f32_$i.log; exit 1; }; tail -1 $O/f32_$i.log | grep -o '"ms_per_step[^,]*\|"train_auc[^,]*'
done
for i in 1 2; do H2O_HOST_PROF=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/b1375_$i.log 2>&1 || { cat $O/b1375_$i.log; exit 1; }; grep -E "host-prof" $O/b1375_$i.log; tail -1 $O/b1375_$i.log | grep -o '"ms_per_step[^,]*'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --rows 1375000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence_1375k.md || exit 1
rm -rf $O/db
head -3 $O/tree_sequence_1375k.md; tail -3 $O/tree_sequence_1375k.md
