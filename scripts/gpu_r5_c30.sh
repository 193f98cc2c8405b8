#!/bin/bash
# Wide planar runs: root-split direction bytes for level 1 (XGBoost 100M x 50 A/B) + planar decision tests
set -o pipefail
O=gpurun_out/r5/c30
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_engine.py -m gpu -k "planar or row_widths or many_features or wide_bins or root16" > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error" $O/tests.log | tail -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees 100"
$S > $O/xgb_on.log 2>&1 || { tail -30 $O/xgb_on.log; exit 1; }; tail -1 $O/xgb_on.log | cut -c1-300
H2O_ROW_DIR_PLANAR=0 $S > $O/xgb_off.log 2>&1 || { tail -30 $O/xgb_off.log; exit 1; }; tail -1 $O/xgb_off.log | cut -c1-300
$S > $O/xgb_on2.log 2>&1 || { tail -30 $O/xgb_on2.log; exit 1; }; tail -1 $O/xgb_on2.log | cut -c1-300
