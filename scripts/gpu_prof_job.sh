#!/bin/bash
# Whole 100-tree GBM job: phase breakdown + rocprofv3 kernel stats (each step time-limited, chained)
set -o pipefail
mkdir -p gpurun_out/prof_job
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/prof_gbm_job.py > gpurun_out/prof_job/phases.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_job/trace -o job -- python3 -u scripts/prof_gbm_job.py > gpurun_out/prof_job/rocprof.log 2>&1
rc=$?
cat gpurun_out/prof_job/phases.log | tail -3
exit $rc
