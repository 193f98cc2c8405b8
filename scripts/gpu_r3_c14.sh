#!/bin/bash
# FILT histogram row compaction + wave-level MFMA Gram (augmented, fused Xᵀv) + shuffle zbeta: GPU tests, GBM
# bench + profile, XGBoost 100M x 50 bench + profile, GLM 10M x 50 bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c14
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_tree_engine.py tests/test_distributed_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash scripts/gpu_prof_summary.sh gbm bench.py --steps 20 --warmup 5 || exit 1
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb.log; exit 1; }
tail -1 $O/xgb.log | cut -c1-400
bash scripts/gpu_prof_summary.sh xgb scripts/bench_suite.py --which xgb --trees 30 || exit 1
timeout -k 10 300 python scripts/bench_suite.py --which glm_big > $O/glm_big.log 2>&1 || { echo "glm_big failed"; tail -20 $O/glm_big.log; exit 1; }
tail -1 $O/glm_big.log | cut -c1-300
bash scripts/gpu_prof_summary.sh glm scripts/bench_suite.py --which glm_big || exit 1
