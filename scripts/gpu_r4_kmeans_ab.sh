#!/bin/bash
# KMeans Lloyd step A/B: default build vs KM_VEC=1 (aligned LDS staging), same box; then a kernel profile of each.
set -o pipefail
O=gpurun_out/r4_km
mkdir -p $O
export TMPDIR=/tmp
for v in default kmvec default kmvec; do
  if [ $v = default ]; then unset H2O_HIP_LIB; else export H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/$v.so; fi
  timeout -k 10 200 python scripts/bench_kmeans_step.py > $O/step_$v.json 2> $O/step_$v.err || exit $?
  echo "$v $(head -1 $O/step_$v.json)"
done
unset H2O_HIP_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_kmeans_step.py > $O/prof.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 12 --md > $O/kernel_stats.md && rm -rf $O/prof
head -6 $O/kernel_stats.md
