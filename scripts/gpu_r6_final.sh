#!/bin/bash
# r6 final tree: the whole GPU tier (one process), smoke, the driver-window headline bench (+ AUTO), the 1.375M shard,
# and the suite rows the README quotes (DL at the bench batch and at H2O's default mini_batch_size, GLM, KMeans)
set -o pipefail
O=gpurun_out/r6/${TAG:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-job --no-auto --rows 1375000 > $O/bench_1375k.log 2>&1 || { cat $O/bench_1375k.log; exit 1; }
S="timeout -k 10 300 python3 scripts/bench_suite.py"
$S --which dl > $O/dl.json 2>&1 || { tail -20 $O/dl.json; exit 1; }
$S --which dl --batch 1 > $O/dl_default.json 2>&1 || { tail -20 $O/dl_default.json; exit 1; }
$S --which glm_big > $O/glm.json 2>&1 || { tail -20 $O/glm.json; exit 1; }
$S --which kmeans > $O/kmeans.json 2>&1 || { tail -20 $O/kmeans.json; exit 1; }
for f in bench_1375k.log dl.json dl_default.json glm.json kmeans.json; do echo "$f $(tail -1 $O/$f | cut -c1-300)"; done
