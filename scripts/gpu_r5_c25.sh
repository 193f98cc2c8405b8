#!/bin/bash
# r5: KMeans unit weights (no per-iteration weight cast) + KM_VEC (16-byte LDS staging) A/B
set -o pipefail
O=gpurun_out/r5/c25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_rccl_trainers_gpu.py -m gpu -k "kmeans" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which kmeans > $O/km1.log 2>&1 || { tail -30 $O/km1.log; exit 1; }; tail -1 $O/km1.log | cut -c1-260
$S --which kmeans > $O/km2.log 2>&1 || { tail -30 $O/km2.log; exit 1; }; tail -1 $O/km2.log | cut -c1-260
H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/kmvec.so $S --which kmeans > $O/km_vec.log 2>&1 || { tail -30 $O/km_vec.log; exit 1; }; tail -1 $O/km_vec.log | cut -c1-260
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 12 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -10 $O/kmeans_kernel_stats.md
H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/kmvec.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbv -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_vec.log 2>&1 || { tail -20 $O/prof_vec.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbv/run_results.db --top 4 --md > $O/kmeans_vec_kernel_stats.md || exit 1
rm -rf $O/dbv
head -6 $O/kmeans_vec_kernel_stats.md
