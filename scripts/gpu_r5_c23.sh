#!/bin/bash
# r5: DL fused step — the layer-1 input transpose (hT0) written by the waves without a layer-1 tile, overlapped
set -o pipefail
O=gpurun_out/r5/c23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dl_calibration_gpu.py -m gpu -k "dl or mlp or deep or calib" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which dl > $O/dl1.log 2>&1 || { tail -30 $O/dl1.log; exit 1; }; tail -1 $O/dl1.log | cut -c1-400
$S --which dl > $O/dl2.log 2>&1 || { tail -30 $O/dl2.log; exit 1; }; tail -1 $O/dl2.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dbd -o run -- python3 scripts/bench_suite.py --which dl > $O/prof_dl.log 2>&1 || { tail -20 $O/prof_dl.log; exit 1; }
python3 scripts/rocpd_stats.py $O/dbd/run_results.db --top 12 --md > $O/dl_kernel_stats.md || exit 1
rm -rf $O/dbd
head -8 $O/dl_kernel_stats.md
