#!/bin/bash
# 4-GiB buffer addressing: big-plane GPU tests, then the XGBoost 100M x 50 bench (500 trees).
set -o pipefail
O=gpurun_out/r4_xgbbuf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py -x -v --timeout 300 --timeout-method thread -m gpu -k "2pow31" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python scripts/bench_suite.py --which xgb > $O/xgb.log 2>&1 || { tail -5 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log | cut -c1-300
H2O_HIST_BUF=0 timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb_nobuf.log 2>&1 || { tail -5 $O/xgb_nobuf.log; exit 1; }
tail -1 $O/xgb_nobuf.log | cut -c1-300
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb_buf100.log 2>&1 || { tail -5 $O/xgb_buf100.log; exit 1; }
tail -1 $O/xgb_buf100.log | cut -c1-300
