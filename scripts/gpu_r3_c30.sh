#!/bin/bash
# A/B: two packed histogram blocks per CU (H2O_HIST_BPC=2) now that the filtered pass has no block barriers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for bpc in 1 2 1 2; do
  for rows in 11000000 1375000; do
    H2O_HIST_BPC=$bpc timeout -k 10 300 python bench.py --rows $rows --steps 50 --warmup 3 --no-job > gpurun_out/ab_${bpc}_$rows.log 2>&1 || exit 1
    echo "bpc=$bpc rows=$rows $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${bpc}_$rows.log)"
  done
done
