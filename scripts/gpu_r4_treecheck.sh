#!/bin/bash
# Tree-kernel change check: tree GPU tests, then the headline bench and the 1.375M-row shard.
set -o pipefail
O=gpurun_out/r4_treecheck
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_distributed_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench11m.json 2> $O/bench11m.err || exit $?
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/bench1375k.json 2> $O/bench1375k.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-job > $O/prof.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || exit 1
rm -rf $O/prof
cat $O/bench11m.json $O/bench1375k.json
