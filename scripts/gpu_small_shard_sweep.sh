#!/bin/bash
# Per-rank shard sizes of a strong-scaling run (11M/8, 11M/4 rows) on one GPU: histogram grid and
# fp32 partials knobs. Each run is time-limited; the sweep stops at the first failure.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/small_shard_sweep.log
: > $out
for rows in 1375000 2750000; do
  for grid in 256 128 64; do
    for pf in 0 1; do
      H2O_HIST_GRID=$grid H2O_PARTIAL_F32=$pf timeout -k 10 120 python -u bench.py --rows $rows --steps 30 --warmup 5 --no-job \
        > gpurun_out/ss.json 2>&1 || { echo "FAIL rows=$rows grid=$grid pf=$pf"; tail -5 gpurun_out/ss.json; exit 1; }
      ms=$(python -c "import json;print(json.loads(open('gpurun_out/ss.json').read().strip().splitlines()[-1])['ms_per_step'])")
      echo "rows=$rows grid=$grid pf32=$pf ms_per_tree=$ms" | tee -a $out
    done
  done
done
