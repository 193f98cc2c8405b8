#!/bin/bash
# rocprofv3 kernel stats of the DeepLearning MLP bench (reduced rows) + a timed python-side breakdown.
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_dl" -o run -- \
  python3 "$R/scripts/bench_suite.py" --which dl --rows ${ROWS:-2000000} > "$R/gpurun_out/prof_dl.log" 2>&1
rc=$?; echo "prof dl rc=$rc"; tail -1 "$R/gpurun_out/prof_dl.log"; exit $rc
