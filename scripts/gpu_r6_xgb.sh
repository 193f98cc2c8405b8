#!/bin/bash
# r6: XGBoost hist 500 trees, depth 6, 100M x 50 (BASELINE config 3 shape, 1 GPU) on the final tree code
set -o pipefail
O=gpurun_out/r6/${TAG:-xgb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u scripts/bench_suite.py --which xgb --trees 500 > $O/xgb.json 2> $O/xgb.err || { tail -20 $O/xgb.err; exit 1; }
tail -1 $O/xgb.json | cut -c1-400
