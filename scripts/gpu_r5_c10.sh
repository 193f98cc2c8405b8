#!/bin/bash
# r5: metrics HIP lattice + GLM single-lambda path + DL bench at H2O's default standardization
set -o pipefail
O=gpurun_out/r5/c10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_metrics_gpu.py tests/test_glm_irls_gpu.py tests/test_dl_calibration_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -15
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which glm_big > $O/glm.log 2>&1 || { tail -30 $O/glm.log; exit 1; }; tail -1 $O/glm.log
$S --which dl > $O/dl_bf16.log 2>&1 || { tail -30 $O/dl_bf16.log; exit 1; }; tail -1 $O/dl_bf16.log | cut -c1-900
$S --which dl --dtype float32 > $O/dl_fp32.log 2>&1 || { tail -30 $O/dl_fp32.log; exit 1; }; tail -1 $O/dl_fp32.log | cut -c1-900
$S --which dl --batch 256 > $O/dl256_bf16.log 2>&1 || { tail -30 $O/dl256_bf16.log; exit 1; }; tail -1 $O/dl256_bf16.log | cut -c1-900
timeout -k 10 300 python3 scripts/fit_profile.py --which glm > $O/glm_profile.log 2>&1 || { tail -30 $O/glm_profile.log; exit 1; }; head -3 $O/glm_profile.log
