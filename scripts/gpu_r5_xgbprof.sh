#!/bin/bash
# r5: XGBoost 100M x 50 kernel table (FPACK) + per-tree sequence
set -o pipefail
O=gpurun_out/r5/xgbprof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which xgb --trees 20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
rm -rf $O/db
head -20 $O/kernel_stats.md; head -45 $O/tree_sequence.md
