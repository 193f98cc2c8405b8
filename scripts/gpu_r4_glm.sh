#!/bin/bash
# GLM kernels after the load-batching changes: GPU tests (gram / zbeta / xtv / glm) + glm_big profile.
set -o pipefail
O=gpurun_out/r4_glm
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "gram or zbeta or xtv or glm or GLM" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python scripts/bench_suite.py --which glm_big > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --top 12 --md > $O/kernel_stats.md || exit 1
rm -rf $O/p
grep -h '"metric"' $O/run.log | cut -c1-200
head -14 $O/kernel_stats.md
