#!/bin/bash
# r5: column-wave hist_reduce; headline + job; 1.375M shard host profile and GPU sequence
set -o pipefail
O=gpurun_out/r5/c12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tree_engine.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job > $O/bench$i.log 2>&1 || { cat $O/bench$i.log; exit 1; }; tail -1 $O/bench$i.log | cut -c1-200; done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_job.log 2>&1 || { cat $O/bench_job.log; exit 1; }; tail -1 $O/bench_job.log | grep -o '"ms_per_step[^,]*\|"job_100[^,]*'
H2O_HOST_PROF=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --rows 1375000 --no-job > $O/b1375.log 2>&1 || { cat $O/b1375.log; exit 1; }; grep -E "host-prof" $O/b1375.log; tail -1 $O/b1375.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --rows 1375000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/tree_sequence_1375k.md || exit 1
rm -rf $O/db
head -40 $O/tree_sequence_1375k.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db2 -o run -- python3 bench.py --steps 14 --warmup 2 --no-job > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db2/run_results.db --sequence k_gbm_step > $O/tree_sequence.md || exit 1
rm -rf $O/db2
head -3 $O/tree_sequence.md; grep -E "hist_reduce" $O/tree_sequence.md
