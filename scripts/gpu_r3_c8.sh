#!/bin/bash
# tree engine: LDS-staged leaf walk + feature-sliced row-sharded exchange
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tree_engine.py tests/test_distributed_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_tree.log 2>&1 || { echo "tree tests failed"; grep -E "FAILED|Error|error" $O/pytest_tree.log | head -20; tail -40 $O/pytest_tree.log; exit 1; }
tail -3 $O/pytest_tree.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 180 python bench.py --steps 100 --warmup 5 --no-job > $O/bench100.log 2>&1 || { echo "bench100 failed"; tail -20 $O/bench100.log; exit 1; }
tail -1 $O/bench100.log
bash scripts/gpu_prof_summary.sh gbm bench.py --steps 20 --warmup 5 --no-job || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -k "dl_" --timeout 120 --timeout-method thread > $O/pytest_dl.log 2>&1 || { echo "dl tests failed"; grep -E "FAILED|Error|error" $O/pytest_dl.log | head -20; tail -40 $O/pytest_dl.log; exit 1; }
tail -2 $O/pytest_dl.log
timeout -k 10 300 python scripts/bench_suite.py --which dl > $O/dl.log 2>&1 || { echo "dl bench failed"; tail -20 $O/dl.log; exit 1; }
tail -1 $O/dl.log
bash scripts/gpu_prof_summary.sh dl scripts/bench_suite.py --which dl --rows 2000000 || exit 1
