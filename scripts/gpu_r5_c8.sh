#!/bin/bash
set -o pipefail
O=gpurun_out/r5/c8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tree_engine.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/bench$i.log 2>&1 || { cat $O/bench$i.log; exit 1; }; tail -1 $O/bench$i.log | cut -c1-200; done
bash scripts/gpu_r5_xgbprof.sh && bash scripts/gpu_r5_pmc3.sh && bash scripts/gpu_r5_suite.sh
