#!/bin/bash
# Round-end verification then secondary benchmarks (each step time-limited; stops at the first failure).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
PROF=0 bash scripts/gpu_r2_check.sh && T=240 bash scripts/gpu_suite.sh
