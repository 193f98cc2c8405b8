#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_prof_summary.sh kmeans scripts/bench_suite.py --which kmeans || exit 1
bash scripts/gpu_prof_summary.sh glm scripts/bench_suite.py --which glm_big || exit 1
