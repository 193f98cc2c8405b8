#!/bin/bash
# split reduce inside the single-block k_plan (levels <= 256 nodes) + leaf values in the leaf-sum pass: tree GPU
# tests, 1.375M rehearsal + dispatch sequence, 11M bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c20
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROWS="1375000 11000000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 bench.py --rows 1375000 --steps 30 --warmup 3 --no-job > $O/run.log 2>&1 || { echo "prof failed"; tail -20 $O/run.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/sequence.md || exit 1
rm -rf $O/db
head -3 $O/sequence.md
