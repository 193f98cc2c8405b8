#!/bin/bash
# k_zbeta LDS span A/B: 48 KiB (default) vs 24 KiB per block (more blocks per CU)
set -o pipefail
O=gpurun_out/r4_zbeta
mkdir -p $O
export TMPDIR=/tmp
[ -f llama_github_io_amd/lib_alt/zb6k.so ] || bash scripts/build_alt.sh zb6k -DZB_LDS_FLOATS=6144 > /dev/null || exit 1
for lib in main zb6k; do
  e=""; [ $lib != main ] && e="H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/$lib.so"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$lib -o run -- python scripts/bench_suite.py --which glm_big > $O/run_$lib.log 2>&1 || { tail -5 $O/run_$lib.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/p_$lib/run_results.db --top 10 --md > $O/ks_$lib.md || exit 1
  rm -rf $O/p_$lib
  echo "== $lib: $(grep -h '"metric"' $O/run_$lib.log | cut -c1-110)"
  grep -E "k_zbeta" $O/ks_$lib.md | cut -c1-130
done
