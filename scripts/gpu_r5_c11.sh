#!/bin/bash
# r5: KMeans per-block slabs / no per-step assignments; GLM training predictions from the training design
set -o pipefail
O=gpurun_out/r5/c11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_glm_irls_gpu.py -m gpu -k "kmeans or glm or irls" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which glm_big > $O/glm.log 2>&1 || { tail -30 $O/glm.log; exit 1; }; tail -1 $O/glm.log
$S --which kmeans > $O/kmeans.log 2>&1 || { tail -30 $O/kmeans.log; exit 1; }; tail -1 $O/kmeans.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 20 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -12 $O/kmeans_kernel_stats.md
