#!/bin/bash
# r6: GLM 10M x 50 timed fit only (window from its k_num_stats): per-kernel table + dispatch order with gaps
set -o pipefail
O=gpurun_out/r6/${TAG:-glmwin}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --window k_num_stats --top 40 > $O/window.md || exit 1
rm -rf $O/db
head -45 $O/window.md
