#!/bin/bash
# Secondary benchmarks on one MI355X (each step time-limited, stops at the first failure).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 ${T:-600} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log; return $rc; }
run suite_kmeans python scripts/bench_suite.py --which kmeans && \
run suite_glm python scripts/bench_suite.py --which glm && \
run suite_dl python scripts/bench_suite.py --which dl && \
run suite_xgb python scripts/bench_suite.py --which xgb
