#!/bin/bash
# r6: per-tree GPU-busy timelines of the final tree code (graph replay + wave plan) at 11M and 1.375M rows
set -o pipefail
O=gpurun_out/r6/${TAG:-timeline}
mkdir -p $O
export TMPDIR=/tmp
for r in 11000000 1375000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db$r -o run -- python3 bench.py --steps 30 --warmup 5 --no-job --no-auto --rows $r > $O/prof$r.log 2>&1 || { tail -20 $O/prof$r.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db$r/run_results.db --timeline k_gbm_step > $O/timeline_$r.md || exit 1
  python3 scripts/rocpd_stats.py $O/db$r/run_results.db --sequence k_gbm_step > $O/seq_$r.md || exit 1
  rm -rf $O/db$r
  echo "$r: $(head -1 $O/seq_$r.md) below-90%: $(awk -F'|' 'NR>2 && $5+0 < 90 {printf "%s:%s%% ", $2+0, $5+0}' $O/timeline_$r.md)"
done
