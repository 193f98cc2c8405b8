#!/bin/bash
# r6: per-kernel sequence of one AUTO (UniformAdaptive) tree at 11M rows on the final code
set -o pipefail
O=gpurun_out/r6/${TAG:-autoseq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --no-auto --histogram-type AUTO > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/seq_auto.md || exit 1
rm -rf $O/db
cat $O/seq_auto.md
