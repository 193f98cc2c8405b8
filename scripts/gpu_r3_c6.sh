#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 180 python bench.py --steps 100 --warmup 5 --no-job > $O/bench100.log 2>&1 || { echo "bench100 failed"; tail -20 $O/bench100.log; exit 1; }
tail -1 $O/bench100.log
bash scripts/gpu_prof_summary.sh gbm bench.py --steps 20 --warmup 5 --no-job || exit 1
timeout -k 10 300 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log
