#!/bin/bash
# round 3, call 1: gpu tests (incl. the >2^31-byte bins test), headline bench, histogram primitive
# microbenchmark, XGBoost 100M x 50 (100 trees) under rocprofv3 kernel trace (the former 0x1016 fault)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 60 ./scripts/mb_hist2.bin > $O/mb_hist2.log 2>&1 || { echo "mb failed"; cat $O/mb_hist2.log; exit 1; }
cat $O/mb_hist2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_xgb -o run -- python3 scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -30 $O/xgb.log; exit 1; }
tail -2 $O/xgb.log
