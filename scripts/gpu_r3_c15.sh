#!/bin/bash
# wide numeric bins on the GPU engine (grouped column sampling, xmap bin assign) + R=1 zbeta: full GPU
# suite, GLM 10M x 50 bench + profile, GBM bench (default UniformAdaptive vs QuantilesGlobal headline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c15
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/bench_suite.py --which glm_big > $O/glm_big.log 2>&1 || { echo "glm_big failed"; tail -20 $O/glm_big.log; exit 1; }
tail -1 $O/glm_big.log | cut -c1-300
bash scripts/gpu_prof_summary.sh glm scripts/bench_suite.py --which glm_big || exit 1
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
