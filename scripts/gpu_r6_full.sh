#!/bin/bash
# r6: the whole GPU tier (pytest -m gpu, one process), smoke, the driver-window headline bench (+ AUTO side run)
set -o pipefail
O=gpurun_out/r6/${TAG:-full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-900
