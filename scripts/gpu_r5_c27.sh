#!/bin/bash
# KMeans Lloyd kernel occupancy A/B: default (3 waves/SIMD, stride 49) vs 4 waves/SIMD (stride 21) with G=4 / G=2
set -o pipefail
O=gpurun_out/r5/c27
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/llama_github_io_amd/lib_alt
for v in default km4 km4g2 kmg2; do
  if [ $v = default ]; then E=""; else E="H2O_HIP_LIB=$L/$v.so"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db_$v -o run -- python3 scripts/bench_suite.py --which kmeans > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db_$v/run_results.db --top 3 --md > $O/stats_$v.md || exit 1
  rm -rf $O/db_$v
  echo "$v: $(grep lloyd $O/stats_$v.md | cut -c1-160)"
done
