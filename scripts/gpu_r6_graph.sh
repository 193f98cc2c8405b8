#!/bin/bash
# r6: per-tree hipGraph replay — tree GPU tests, headline bench, 1.375M-row shard with host-loop timings (graph on/off)
set -o pipefail
O=gpurun_out/r6/${TAG:-graph}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_kernels_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-job --no-auto"
for g in 1 0; do
  H2O_TREE_GRAPH=$g $B > $O/b11m_g$g.log 2>&1 || { tail -20 $O/b11m_g$g.log; exit 1; }
  H2O_TREE_GRAPH=$g H2O_HOST_PROF=1 $B --rows 1375000 > $O/b1375k_g$g.log 2>&1 || { tail -20 $O/b1375k_g$g.log; exit 1; }
  echo "graph=$g 11M $(tail -1 $O/b11m_g$g.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])') 1.375M $(tail -1 $O/b1375k_g$g.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])') $(grep host-prof $O/b1375k_g$g.log | tail -1)"
done
