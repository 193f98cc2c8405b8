#!/bin/bash
# r6: shard-size tree (1.375M rows: plain and through the 1-rank RCCL driver), per-tree GPU-busy timelines, then the
# secondary BASELINE configs: XGBoost 100M x 50 over 500 trees (config 3 shape), GLM x3, KMeans, DL bf16 4096-row steps
set -o pipefail
O=gpurun_out/r6/${TAG:-suite}
mkdir -p $O
export TMPDIR=/tmp
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-job --no-auto"
$B --rows 1375000 > $O/b1375k.log 2>&1 || { tail -20 $O/b1375k.log; exit 1; }; tail -1 $O/b1375k.log | cut -c1-300
H2O_TREE_COMM_FORCE=ar $B --rows 1375000 > $O/b1375k_ar.log 2>&1 || { tail -20 $O/b1375k_ar.log; exit 1; }; tail -1 $O/b1375k_ar.log | cut -c1-300
for R in 1375000 11000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db$R -o run -- python3 bench.py --steps 30 --warmup 2 --rows $R --no-job --no-auto > $O/prof$R.log 2>&1 || { tail -20 $O/prof$R.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db$R/run_results.db --timeline k_gbm_step > $O/timeline_$R.md || exit 1
  rm -rf $O/db$R
  tail -3 $O/timeline_$R.md
done
S="timeout -k 10 400 python3 scripts/bench_suite.py"
$S --which xgb --trees 500 > $O/xgb500.log 2>&1 || { tail -30 $O/xgb500.log; exit 1; }; tail -1 $O/xgb500.log | cut -c1-600
for i in 1 2 3; do $S --which glm_big > $O/glm$i.log 2>&1 || { tail -30 $O/glm$i.log; exit 1; }; tail -1 $O/glm$i.log | cut -c1-400; done
$S --which kmeans > $O/kmeans.log 2>&1 || { tail -30 $O/kmeans.log; exit 1; }; tail -1 $O/kmeans.log | cut -c1-400
$S --which dl > $O/dl4096.log 2>&1 || { tail -30 $O/dl4096.log; exit 1; }; tail -1 $O/dl4096.log | cut -c1-600
