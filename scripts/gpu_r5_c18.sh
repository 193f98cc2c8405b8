#!/bin/bash
# r5: AUTO (UniformAdaptive, nbins_top_level 1024) tree sequence + XGBoost with fp32 partials
set -o pipefail
O=gpurun_out/r5/c18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --histogram-type AUTO > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/auto_sequence.md || exit 1
rm -rf $O/db
cat $O/auto_sequence.md
timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { tail -30 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log | cut -c1-300
