#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_km -o km -- python3 scripts/bench_kmeans_step.py > gpurun_out/prof_km.log 2>&1
rc=$?
find gpurun_out/prof_km -name "*stats*" | head
exit $rc
