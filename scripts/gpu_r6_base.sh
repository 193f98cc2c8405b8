#!/bin/bash
# r6: baseline on a fresh box — headline bench, 1.375M-row shard bench + its rocprof tree sequence
set -o pipefail
O=gpurun_out/r6/${TAG:-base}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/bench1375k.log 2>&1 || { cat $O/bench1375k.log; exit 1; }
tail -1 $O/bench1375k.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --rows 1375000 --no-job > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence_1375k.md || exit 1
rm -rf $O/db
head -40 $O/tree_sequence_1375k.md
