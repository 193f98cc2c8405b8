#!/bin/bash
# XGBoost 100M x 50 kernel profile (30 trees) and per-tree sequence.
set -o pipefail
O=gpurun_out/r4_xgbprof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_suite.py --which xgb --trees 30 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-300
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 20 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || true
rm -rf $O/prof
head -24 $O/kernel_stats.md
head -45 $O/tree_sequence.md
