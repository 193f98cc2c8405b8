#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "kmeans or segment" > $O/pytest_km.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_km.log; exit 1; }
tail -3 $O/pytest_km.log
timeout -k 10 200 python scripts/bench_suite.py --which kmeans > $O/km.log 2>&1 || { echo "km bench failed"; tail -20 $O/km.log; exit 1; }
tail -1 $O/km.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_km -o run -- python3 scripts/bench_suite.py --which kmeans > $O/km_prof.log 2>&1 || { echo "km prof failed"; tail -20 $O/km_prof.log; exit 1; }
timeout -k 10 300 python scripts/bench_suite.py --which glm_big > $O/glm.log 2>&1 || { echo "glm bench failed"; tail -20 $O/glm.log; exit 1; }
tail -1 $O/glm.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_glm -o run -- python3 scripts/bench_suite.py --which glm_big > $O/glm_prof.log 2>&1 || { echo "glm prof failed"; tail -20 $O/glm_prof.log; exit 1; }
echo done
