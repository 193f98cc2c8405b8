#!/bin/bash
# rocprofv3 kernel statistics of the XGBoost hist benchmark (100M x 50, 100 trees).
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_xgb" -o run -- \
    python3 "$R/scripts/bench_suite.py" --which xgb --trees 100 > "$R/gpurun_out/prof_xgb.log" 2>&1
rc=$?
tail -3 "$R/gpurun_out/prof_xgb.log"
exit $rc
