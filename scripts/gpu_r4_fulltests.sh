#!/bin/bash
# The driver's round-end GPU tier: every gpu test, smoke(), and the default bench.
set -o pipefail
O=gpurun_out/r4_full
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
# the other BASELINE configurations (one line each)
timeout -k 10 400 python scripts/bench_suite.py --which dl > $O/dl10m.log 2>&1 || { tail -5 $O/dl10m.log; exit 1; }
tail -1 $O/dl10m.log | cut -c1-400
timeout -k 10 400 python scripts/bench_suite.py --which xgb > $O/xgb.log 2>&1 || { tail -5 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log | cut -c1-400
