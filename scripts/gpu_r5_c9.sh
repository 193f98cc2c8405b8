#!/bin/bash
# r5: AUTO (H2O default histogram) headline shape, tree sequence (leaf-assign prefetch), DL calibration matrix
set -o pipefail
O=gpurun_out/r5/c9
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job --histogram-type AUTO > $O/auto$i.log 2>&1 || { cat $O/auto$i.log; exit 1; }; tail -1 $O/auto$i.log | cut -c1-200; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
rm -rf $O/db
head -3 $O/tree_sequence.md; grep -E "leaf_assign|route" $O/tree_sequence.md
timeout -k 10 600 python3 scripts/dl_calib.py > $O/dl_calib.log 2>&1 || { tail -30 $O/dl_calib.log; exit 1; }
cat $O/dl_calib.log | cut -c1-400
