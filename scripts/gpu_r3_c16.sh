#!/bin/bash
# LDS-span zbeta: kernel tests, GLM 10M x 50 bench + profile; strong-scaling rehearsal (per-rank rows of
# 1/2/4/8 GPUs) + kernel profile at 1.375M rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "zbeta or gram" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/bench_suite.py --which glm_big > $O/glm_big.log 2>&1 || { echo "glm_big failed"; tail -20 $O/glm_big.log; exit 1; }
tail -1 $O/glm_big.log | cut -c1-300
bash scripts/gpu_prof_summary.sh glm scripts/bench_suite.py --which glm_big || exit 1
STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
bash scripts/gpu_prof_summary.sh gbm1375k bench.py --rows 1375000 --steps 50 --warmup 5 --no-job || exit 1
