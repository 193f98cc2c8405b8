#!/bin/bash
# Kernel profile of the bf16 and fp32 DL bench loops (2M rows).
set -o pipefail
O=gpurun_out/r4_dlprof
mkdir -p $O
export TMPDIR=/tmp
for dt in bf16 float32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$dt -o run -- python scripts/bench_suite.py --which dl --rows 2000000 --dtype $dt > $O/run_$dt.log 2>&1 || exit $?
  python3 scripts/rocpd_stats.py $O/p_$dt/run_results.db --top 12 --md > $O/kernel_stats_$dt.md && rm -rf $O/p_$dt
  head -9 $O/kernel_stats_$dt.md
done
