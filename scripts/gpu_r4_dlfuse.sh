#!/bin/bash
# DL: split-sum fused into ADADELTA — GPU tests, A/B bench lines (H2O_DL_FUSE_WSUM=0/1), bf16 kernel profile.
set -o pipefail
O=gpurun_out/r4_dlfuse
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "fused or deep or dl or adadelta" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for fz in 1 0; do
  for dt in bf16 float32; do
    H2O_DL_FUSE_WSUM=$fz timeout -k 10 200 python scripts/bench_suite.py --which dl --rows 2000000 --dtype $dt > $O/bench_${dt}_$fz.log 2>&1 || exit $?
    echo "fuse=$fz $dt: $(tail -1 $O/bench_${dt}_$fz.log)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python scripts/bench_suite.py --which dl --rows 2000000 --dtype bf16 > $O/prof.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/p/run_results.db --top 12 --md > $O/kernel_stats_bf16.md && rm -rf $O/p
head -9 $O/kernel_stats_bf16.md
