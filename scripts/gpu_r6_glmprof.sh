#!/bin/bash
# r6: kernel table of the GLM 10M x 50 fit (binomial IRLSM, 5 iterations) — HIP kernels vs torch glue
set -o pipefail
O=gpurun_out/r6/${TAG:-glmprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 40 > $O/kernels.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --gaps k_num_stats --min-gap 20 > $O/gaps.md || exit 1
rm -rf $O/db
head -45 $O/kernels.md
head -3 $O/gaps.md
