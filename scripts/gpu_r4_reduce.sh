#!/bin/bash
set -o pipefail
O=gpurun_out/r4_reduce
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py tests/test_native_comm_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > $O/bench_qg.json 2> $O/bench_qg.err || exit 1
cat $O/bench_qg.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 12 --warmup 2 --no-job > $O/prof.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 20 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || true
rm -rf $O/prof
grep k_hist_reduce $O/kernel_stats.md | cut -c1-140
