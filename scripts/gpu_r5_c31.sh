#!/bin/bash
# Route row moves with non-temporal loads / stores (H2O_ROUTE_NT A/B): tests under NT=3, headline + XGBoost benches
set -o pipefail
O=gpurun_out/r5/c31
mkdir -p $O
export TMPDIR=/tmp
H2O_ROUTE_NT=3 timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_engine.py -m gpu -k "route or planar or matches_reference" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for nt in 0 1 2 3 0 3; do
  H2O_ROUTE_NT=$nt timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_nt$nt.log 2>&1 || { tail -30 $O/bench_nt$nt.log; exit 1; }
  echo "nt=$nt $(tail -1 $O/bench_nt$nt.log | cut -c1-200)"
done
S="timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees 100"
for nt in 0 3; do
  H2O_ROUTE_NT=$nt $S > $O/xgb_nt$nt.log 2>&1 || { tail -30 $O/xgb_nt$nt.log; exit 1; }
  echo "xgb nt=$nt $(tail -1 $O/xgb_nt$nt.log | cut -c1-300)"
done
