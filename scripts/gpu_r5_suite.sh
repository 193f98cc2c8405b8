#!/bin/bash
# r5: the secondary benchmarks (GLM / KMeans / DL) normal and through a 1-rank RCCL group, GLM host profile,
# rocprofv3 kernel tables of GLM and KMeans
set -o pipefail
O=gpurun_out/r5/${TAG:-suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_glm_irls_gpu.py tests/test_kernels_gpu.py -k "irls or glm" -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which glm_big > $O/glm.log 2>&1 || { tail -30 $O/glm.log; exit 1; }; tail -1 $O/glm.log
H2O_FORCE_SHARDED=1 $S --which glm_big > $O/glm_rccl.log 2>&1 || { tail -30 $O/glm_rccl.log; exit 1; }; tail -1 $O/glm_rccl.log
$S --which kmeans > $O/kmeans.log 2>&1 || { tail -30 $O/kmeans.log; exit 1; }; tail -1 $O/kmeans.log
H2O_FORCE_SHARDED=1 $S --which kmeans > $O/kmeans_rccl.log 2>&1 || { tail -30 $O/kmeans_rccl.log; exit 1; }; tail -1 $O/kmeans_rccl.log
$S --which dl > $O/dl4096.log 2>&1 || { tail -30 $O/dl4096.log; exit 1; }; tail -1 $O/dl4096.log | cut -c1-900
$S --which dl --batch 256 > $O/dl256_bf16.log 2>&1 || { tail -30 $O/dl256_bf16.log; exit 1; }; tail -1 $O/dl256_bf16.log | cut -c1-900
$S --which dl --batch 256 --dtype float32 > $O/dl256_fp32.log 2>&1 || { tail -30 $O/dl256_fp32.log; exit 1; }; tail -1 $O/dl256_fp32.log | cut -c1-900
$S --which dl --dtype float32 > $O/dl4096_fp32.log 2>&1 || { tail -30 $O/dl4096_fp32.log; exit 1; }; tail -1 $O/dl4096_fp32.log | cut -c1-900
H2O_FORCE_SHARDED=1 $S --which dl > $O/dl_rccl.log 2>&1 || { tail -30 $O/dl_rccl.log; exit 1; }; tail -1 $O/dl_rccl.log | cut -c1-900
timeout -k 10 300 python3 scripts/fit_profile.py --which glm > $O/glm_profile.log 2>&1 || { tail -30 $O/glm_profile.log; exit 1; }; head -3 $O/glm_profile.log
timeout -k 10 300 python3 scripts/fit_profile.py --which dl > $O/dl_profile.log 2>&1 || { tail -30 $O/dl_profile.log; exit 1; }; head -3 $O/dl_profile.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbg -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof_glm.log 2>&1 || { tail -20 $O/prof_glm.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbg/run_results.db --top 30 --md > $O/glm_kernel_stats.md || exit 1
rm -rf $O/dbg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 30 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -8 $O/glm_kernel_stats.md $O/kmeans_kernel_stats.md
