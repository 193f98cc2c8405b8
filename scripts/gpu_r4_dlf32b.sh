#!/bin/bash
set -o pipefail
O=gpurun_out/r4_dlf32b
mkdir -p $O
run() {  # name rows epochs dtype [env...]
  local name=$1 rows=$2 ep=$3 dt=$4; shift 4
  env "$@" timeout -k 10 300 python scripts/bench_suite.py --which dl --dtype $dt --rows $rows --epochs $ep > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s auc', d['train_auc'])")"
}
run f32_2M_ep2.5 2000000 2.5 float32 H2O_X=1 || exit 1
run f32_5M_libpath 5000000 1 float32 H2O_DL_FUSED_F32=0 || exit 1
run f32_5M_nograph 5000000 1 float32 H2O_DL_GRAPH=0 || exit 1
run bf16_5M 5000000 1 bf16 H2O_X=1 || exit 1
run f32_3M 3000000 1 float32 H2O_X=1 || exit 1
