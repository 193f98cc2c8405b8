#!/bin/bash
# r6: kernel table of DeepLearning at H2O's default mini_batch_size (GPU steps of N // 16384 = 610 rows at 10M)
set -o pipefail
O=gpurun_out/r6/${TAG:-dldef}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which dl --batch 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 20 > $O/kernels.md || exit 1
rm -rf $O/db
head -24 $O/kernels.md
