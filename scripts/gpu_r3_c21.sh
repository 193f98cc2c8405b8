#!/bin/bash
# FILT split-byte prefetch: tree GPU tests, rows sweep (11M / 1.375M), XGBoost 100M x 50 (100 trees), RCCL probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c21
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tree_engine.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROWS="11000000 1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log | cut -c1-300
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_probe.py > $O/rccl.log 2>&1
echo "rccl probe rc=$?"; grep -E "rank|Error|error" $O/rccl.log | head -8
exit 0
