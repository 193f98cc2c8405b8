#!/bin/bash
set -o pipefail
O=gpurun_out/r4_dlf32
mkdir -p $O
timeout -k 10 300 python scripts/dl_f32_probe.py 10000000 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep max_err $O/probe.log
for cfg in "2000000 1" "10000000 0" "5000000 1"; do
  set -- $cfg
  H2O_DL_FUSE_WSUM=$2 timeout -k 10 300 python scripts/bench_suite.py --which dl --dtype float32 --rows $1 > $O/dl_$1_$2.log 2>&1 || { tail -5 $O/dl_$1_$2.log; exit 1; }
  echo "rows=$1 fuse_wsum=$2: $(tail -1 $O/dl_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['train_auc'])")"
done
