#!/bin/bash
# Expander transform / stats: GPU tests, DL 10M bench, kernel stats of the DL setup.
set -o pipefail
O=gpurun_out/r4_expander
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "expander or dl or deep or fused" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python scripts/bench_suite.py --which dl > $O/dl10m.log 2>&1 || { tail -5 $O/dl10m.log; exit 1; }
tail -1 $O/dl10m.log | cut -c1-420
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_suite.py --which dl > $O/prof.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 16 --md > $O/kernel_stats.md || exit 1
rm -rf $O/prof
head -20 $O/kernel_stats.md
