#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "kmeans" > gpurun_out/pytest_kmeans.log 2>&1 && \
timeout -k 10 180 python -u scripts/bench_kmeans_step.py > gpurun_out/bench_kmeans.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
KM_N=10000000 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kmeans -o km -- python3 scripts/bench_kmeans_step.py > gpurun_out/prof_kmeans.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_kmeans.log; cat gpurun_out/bench_kmeans.log
exit $rc
