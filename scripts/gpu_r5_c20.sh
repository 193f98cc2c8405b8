#!/bin/bash
# r5: KMeans Lloyd kernel with two tiles in flight per wave (A/B against H2O_KM_DB=0) + kernel stats
set -o pipefail
O=gpurun_out/r5/c20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "kmeans" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
H2O_KM_DB=0 $S --which kmeans > $O/kmeans_sb.log 2>&1 || { tail -30 $O/kmeans_sb.log; exit 1; }; tail -1 $O/kmeans_sb.log | cut -c1-400
$S --which kmeans > $O/kmeans_db.log 2>&1 || { tail -30 $O/kmeans_db.log; exit 1; }; tail -1 $O/kmeans_db.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 20 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -8 $O/kmeans_kernel_stats.md
