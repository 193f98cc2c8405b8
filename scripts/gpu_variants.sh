#!/bin/bash
# A/B of tree-engine build variants (env switches) at the per-rank row counts of 8-GPU and 1-GPU runs.
# VARIANTS: space-separated "NAME:ENV=V,ENV=V" items; ROWS: row counts. Each run is time-limited.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
for rows in ${ROWS:-1375000 11000000}; do
  for v in ${VARIANTS:-base:X=0}; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --rows $rows --steps ${STEPS:-40} --warmup 3 \
      > gpurun_out/var_${name}_$rows.log 2>&1 || exit $?
    echo "rows=$rows $name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_${name}_$rows.log)"
  done
done
