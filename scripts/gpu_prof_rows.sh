#!/bin/bash
# rocprofv3 kernel trace of bench.py at a given per-rank row count (default: the 8-GPU shard size).
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rows=${ROWS:-1375000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$rows" -o run -- \
  python3 "$R/bench.py" --rows $rows --steps ${STEPS:-10} --warmup 2 > "$R/gpurun_out/prof_$rows.log" 2>&1
rc=$?; echo "prof rows=$rows rc=$rc"; tail -1 "$R/gpurun_out/prof_$rows.log"; exit $rc
