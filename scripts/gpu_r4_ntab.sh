#!/bin/bash
# expander transform tile A/B: 32 rows x 256 features (default) vs 128 rows x 64 features
set -o pipefail
O=gpurun_out/r4_ntab
mkdir -p $O
export TMPDIR=/tmp
[ -f llama_github_io_amd/lib_alt/nt128.so ] || bash scripts/build_alt.sh nt128 -DNT_ROWS=128 -DNT_FC=64 > /dev/null || exit 1
H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/nt128.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k expander > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in main nt128; do
  e=""; [ $lib != main ] && e="H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/$lib.so"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$lib -o run -- python scripts/bench_suite.py --which dl > $O/run_$lib.log 2>&1 || { tail -5 $O/run_$lib.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/p_$lib/run_results.db --top 8 --md > $O/ks_$lib.md || exit 1
  rm -rf $O/p_$lib
  echo "== $lib: $(grep -h k_num_transform $O/ks_$lib.md | cut -c1-130)"
done
