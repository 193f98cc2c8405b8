#!/bin/bash
# r5: pipelined numeric transform + phased KMeans Lloyd tile (weights in the one-hot operand) + idle gaps of a DL fit
set -o pipefail
O=gpurun_out/r5/c22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dl_calibration_gpu.py -m gpu -k "kmeans or transform or expander or num_ or calib or dl" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which kmeans > $O/kmeans.log 2>&1 || { tail -30 $O/kmeans.log; exit 1; }; tail -1 $O/kmeans.log | cut -c1-300
$S --which dl > $O/dl.log 2>&1 || { tail -30 $O/dl.log; exit 1; }; tail -1 $O/dl.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dbk -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_km.log 2>&1 || { tail -20 $O/prof_km.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbk/run_results.db --top 20 --md > $O/kmeans_kernel_stats.md || exit 1
rm -rf $O/dbk
head -6 $O/kmeans_kernel_stats.md
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/dbd -o run -- python3 scripts/fit_profile.py --which dl --no-cprofile > $O/prof_dl.log 2>&1 || { tail -20 $O/prof_dl.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbd/run_results.db --gaps k_num_stats --min-gap 20 > $O/dl_gaps.md || exit 1
python3 scripts/rocpd_stats.py $O/dbd/run_results.db --top 12 --md > $O/dl_kernel_stats.md || exit 1
rm -rf $O/dbd
grep fit $O/prof_dl.log
head -40 $O/dl_gaps.md; head -10 $O/dl_kernel_stats.md
