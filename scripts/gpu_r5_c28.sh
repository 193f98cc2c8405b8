#!/bin/bash
# KMeans: 4-waves/SIMD Lloyd variant as the default for K <= 16, P <= 24 (tests + bench + stats, A/B vs H2O_KM_OCC4=0)
set -o pipefail
O=gpurun_out/r5/c28
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_rccl_trainers_gpu.py -m gpu -k "kmeans" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which kmeans > $O/km1.log 2>&1 || { tail -30 $O/km1.log; exit 1; }; tail -1 $O/km1.log | cut -c1-260
$S --which kmeans > $O/km2.log 2>&1 || { tail -30 $O/km2.log; exit 1; }; tail -1 $O/km2.log | cut -c1-260
H2O_KM_OCC4=0 $S --which kmeans > $O/km_off.log 2>&1 || { tail -30 $O/km_off.log; exit 1; }; tail -1 $O/km_off.log | cut -c1-260
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 12 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -8 $O/kmeans_kernel_stats.md
