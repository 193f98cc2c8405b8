#!/bin/bash
# H2O-default histogram (AUTO = UniformAdaptive over 1016 wide edges): bench (fine-bin atomics on / off) + profile.
set -o pipefail
O=gpurun_out/r4_auto
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --histogram-type AUTO --steps 10 --warmup 3 > $O/bench_auto.json 2> $O/bench_auto.err || exit $?
H2O_HIST_FINE=0 timeout -k 10 300 python bench.py --histogram-type AUTO --steps 10 --warmup 3 --no-job > $O/bench_auto_nofine.json 2> $O/bench_auto_nofine.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --histogram-type AUTO --steps 5 --warmup 2 --no-job > $O/prof.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || exit 1
rm -rf $O/prof
H2O_HIST_FINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof0 -o run -- python bench.py --histogram-type AUTO --steps 5 --warmup 2 --no-job > $O/prof0.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/prof0/run_results.db --top 30 --md > $O/kernel_stats_nofine.md || exit 1
rm -rf $O/prof0
cat $O/bench_auto.json $O/bench_auto_nofine.json
