#!/bin/bash
# Strong-scaling rehearsal on one GPU: ms/tree at the per-rank row counts of 1/2/4/8-GPU runs
# (11M / N rows), exposing the fixed per-tree overhead that bounds multi-GPU efficiency.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
for rows in ${ROWS:-1375000 2750000 5500000 11000000}; do
  timeout -k 10 300 python bench.py --rows $rows --steps ${STEPS:-30} --warmup 3 > gpurun_out/sweep_$rows.log 2>&1 || exit $?
  echo "rows=$rows $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$rows.log)"
done
