#!/bin/bash
# r6: tree-engine + native-comm GPU tests, then the driver-window headline bench (+ AUTO side run)
set -o pipefail
O=gpurun_out/r6/${TAG:-tree}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1200
