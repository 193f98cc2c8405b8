#!/bin/bash
# r6: graph cache per launch-plan signature — the multinomial graph test, tree GPU tests, headline bench
set -o pipefail
O=gpurun_out/r6/${TAG:-graphk}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_distributed_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
