#!/bin/bash
# Backwards tile walks (last-level-cache reuse between consecutive passes over the same rows): H2O_HIST_DBG bit 2 =
# FILT histogram blocks walk their ranges backwards, bit 3 = routes take tiles in descending order
set -o pipefail
O=gpurun_out/r5/c32
mkdir -p $O
export TMPDIR=/tmp
H2O_HIST_DBG=12 timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_engine.py -m gpu -k "route or planar or matches_reference or filt" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for d in 0 4 8 12 0 4 12; do
  H2O_HIST_DBG=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_d$d.log 2>&1 || { tail -30 $O/bench_d$d.log; exit 1; }
  echo "dbg=$d $(tail -1 $O/bench_d$d.log | cut -c150-230)"
done
S="timeout -k 10 400 python3 scripts/bench_suite.py --which xgb --trees 100"
for d in 0 4 12; do
  H2O_HIST_DBG=$d $S > $O/xgb_d$d.log 2>&1 || { tail -30 $O/xgb_d$d.log; exit 1; }
  echo "xgb dbg=$d $(tail -1 $O/xgb_d$d.log | cut -c150-260)"
done
