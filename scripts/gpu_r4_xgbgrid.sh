#!/bin/bash
# XGBoost 100M x 50: histogram grid A/B (blocks per histogram launch)
set -o pipefail
O=gpurun_out/r4_xgbgrid
mkdir -p $O
for gr in 256 512 768; do
  H2O_HIST_GRID=$gr timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/g$gr.log 2>&1 || { tail -5 $O/g$gr.log; exit 1; }
  echo "grid=$gr: $(tail -1 $O/g$gr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_tree'],3), d['train_auc'])")"
done
