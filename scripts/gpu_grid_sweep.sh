#!/bin/bash
# histogram grid / partial precision sweep at the per-rank row counts of a 1/8-GPU strong-scaling run
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/grid_sweep.txt
: > $out
for rows in 1375000 11000000; do
  for g in 64 128 192 256; do
    for pf in 0 1; do
      r=$(H2O_HIST_GRID=$g H2O_PARTIAL_F32=$pf timeout -k 10 120 python -u bench.py --rows $rows --steps 30 --warmup 5 --no-job | tail -1) || exit 1
      ms=$(echo "$r" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
      echo "rows=$rows grid=$g pf32=$pf ms_per_tree=$ms" | tee -a $out
    done
  done
done
