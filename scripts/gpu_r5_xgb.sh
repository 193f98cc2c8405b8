#!/bin/bash
# r5: XGBoost FPACK (one 32/32 fixed-point LDS atomic per row and feature) — tests + 100M x 50 A/B
set -o pipefail
O=gpurun_out/r5/${TAG:-xgb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "xgboost or tree_family" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees ${TREES:-100} > $O/xgb_fpack.log 2>&1 || { tail -30 $O/xgb_fpack.log; exit 1; }
tail -1 $O/xgb_fpack.log
H2O_XGB_FPACK=0 timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees ${TREES:-100} > $O/xgb_u64.log 2>&1 || { tail -30 $O/xgb_u64.log; exit 1; }
tail -1 $O/xgb_u64.log
