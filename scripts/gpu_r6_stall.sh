#!/bin/bash
# r6: per-tree GPU-busy timelines at 11M rows: default, a 64-buffer snapshot pool, no GC in the tree loop
set -o pipefail
O=gpurun_out/r6/${TAG:-stall}
mkdir -p $O
export TMPDIR=/tmp
for v in base pool64 nogc; do
  case $v in base) E="";; pool64) E="H2O_TREE_SNAP_POOL=64";; nogc) E="H2O_TREE_GC=0";; esac
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db$v -o run -- python3 bench.py --steps 40 --warmup 2 --no-job --no-auto > $O/prof$v.log 2>&1 || { tail -20 $O/prof$v.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db$v/run_results.db --timeline k_gbm_step > $O/timeline_$v.md || exit 1
  rm -rf $O/db$v
  echo "$v: $(awk -F'|' 'NR>2 && $5+0 < 90 {printf "%s:%s%% ", $2+0, $5+0}' $O/timeline_$v.md)"
done
