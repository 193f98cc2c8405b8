#!/bin/bash
# GLM Gram A/B: waves per launch (4096 / 8192 / 16384) and 16 row pairs in flight (alt build).
set -o pipefail
[ -f llama_github_io_amd/lib_alt/unrg16.so ] || bash scripts/build_alt.sh unrg16 -DGRAM_UNRG=16 > /dev/null || exit 1
O=gpurun_out/r4_gram
mkdir -p $O
export TMPDIR=/tmp
CFGS=${GRAM_CFGS:-"4096,main 8192,main 16384,main 4096,unrg16"}
for cfg in $CFGS; do
  cfg=${cfg/,/ }
  set -- $cfg
  lib=""; [ "$2" != main ] && lib="H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/$2.so"
  env H2O_GRAM_WAVES=$1 $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$1_$2 -o run -- python scripts/bench_suite.py --which glm_big > $O/run_$1_$2.log 2>&1 || { tail -5 $O/run_$1_$2.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/p_$1_$2/run_results.db --top 8 --md > $O/ks_$1_$2.md || exit 1
  rm -rf $O/p_$1_$2
  echo "== waves=$1 lib=$2: $(tail -1 $O/run_$1_$2.log | cut -c1-160)"
  grep -E "k_gram|k_zbeta|k_xtv" $O/ks_$1_$2.md | cut -c1-120
done
