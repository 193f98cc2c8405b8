#!/bin/bash
# Three-tier narrow levels: tree-engine GPU tests, AUTO / QG bench, AUTO profile + tree sequence; DL phase clocks.
set -o pipefail
O=gpurun_out/r4_narrow4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --histogram-type AUTO --steps 30 --warmup 3 > $O/bench_auto.json 2> $O/bench_auto.err || { tail -20 $O/bench_auto.err; exit 1; }
cat $O/bench_auto.json
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > $O/bench_qg.json 2> $O/bench_qg.err || exit 1
cat $O/bench_qg.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --histogram-type AUTO --steps 12 --warmup 2 --no-job > $O/prof.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || true
rm -rf $O/prof
head -14 $O/kernel_stats.md
