#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "dl_fused or dl_trainer" > $O/pytest_dl.log 2>&1 || { echo "dl tests failed"; tail -60 $O/pytest_dl.log; exit 1; }
tail -8 $O/pytest_dl.log
timeout -k 10 300 python scripts/bench_suite.py --which dl > $O/dl.log 2>&1 || { echo "dl bench failed"; tail -30 $O/dl.log; exit 1; }
tail -1 $O/dl.log
bash scripts/gpu_prof_summary.sh dl scripts/bench_suite.py --which dl --rows 2000000 || exit 1
bash scripts/gpu_prof_summary.sh kmeans scripts/bench_suite.py --which kmeans || exit 1
bash scripts/gpu_prof_summary.sh glm scripts/bench_suite.py --which glm_big || exit 1
