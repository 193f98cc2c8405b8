#!/bin/bash
# Tree-engine GPU tests + headline bench + rows sweep (each step time-limited, stops at the first failure).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  ${TESTS:-tests/test_tree_engine.py tests/test_distributed_gpu.py} > gpurun_out/pytest_tree.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_tree.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_rows_sweep.sh
