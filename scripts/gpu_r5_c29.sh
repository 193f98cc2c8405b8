#!/bin/bash
# KMeans: PS=5 shape for P=20 (default 4-wave variant) and a 5-wave A/B (w5g1)
set -o pipefail
O=gpurun_out/r5/c29
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "kmeans" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=$PWD/llama_github_io_amd/lib_alt
for v in default w5g1; do
  if [ $v = default ]; then E=""; else E="H2O_HIP_LIB=$L/$v.so"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db_$v -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db_$v/run_results.db --top 3 --md > $O/stats_$v.md || exit 1
  rm -rf $O/db_$v
  echo "$v: $(grep lloyd $O/stats_$v.md | cut -c1-160)"
done
