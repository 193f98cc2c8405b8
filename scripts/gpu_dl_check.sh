#!/bin/bash
# DL graph tests + DL bench (2M and 10M rows) + rocprofv3 kernel stats of the 2M bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "deeplearning or zbeta or bias_act" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dl.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_suite.py --which dl --rows 2000000 > gpurun_out/dl_2m.log 2>&1 && \
timeout -k 10 400 python -u scripts/bench_suite.py --which dl > gpurun_out/dl_10m.log 2>&1 && \
bash scripts/gpu_prof_dl.sh
rc=$?
tail -2 gpurun_out/pytest_dl.log; grep -o '{"metric.*' gpurun_out/dl_2m.log gpurun_out/dl_10m.log
exit $rc
