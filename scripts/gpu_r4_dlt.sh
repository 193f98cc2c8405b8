#!/bin/bash
# k_dl_rows phase clocks (diagnostic DL_TIMING build) for bf16 and fp32
set -o pipefail
[ -f llama_github_io_amd/lib_alt/dlt.so ] || bash scripts/build_alt.sh dlt -DDL_TIMING > /dev/null || exit 1
O=gpurun_out/r4_dlt
mkdir -p $O
for dt in bf16 float32; do
  H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/dlt.so timeout -k 10 240 python scripts/dl_phase_timing.py $dt > $O/$dt.log 2>&1 || { tail -20 $O/$dt.log; exit 1; }
  cat $O/$dt.log
done
