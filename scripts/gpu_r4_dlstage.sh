#!/bin/bash
# DL: weights of the small layers staged in LDS — GPU tests, A/B bench (H2O_DL_STAGE=0/1), phase clocks.
set -o pipefail
[ -f llama_github_io_amd/lib_alt/dlt.so ] || bash scripts/build_alt.sh dlt -DDL_TIMING > /dev/null || exit 1
O=gpurun_out/r4_dlstage
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "fused or deep or dl or adadelta" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for st in 1 0; do
  for dt in bf16 float32; do
    H2O_DL_STAGE=$st timeout -k 10 200 python scripts/bench_suite.py --which dl --rows 2000000 --dtype $dt > $O/bench_${dt}_$st.log 2>&1 || exit 1
    echo "stage=$st $dt: $(tail -1 $O/bench_${dt}_$st.log | cut -c1-260)"
  done
done
for ws in 4 6 16; do
  H2O_DL_WSPLIT=$ws timeout -k 10 200 python scripts/bench_suite.py --which dl --rows 2000000 --dtype bf16 > $O/bench_ws$ws.log 2>&1 || exit 1
  echo "wsplit=$ws bf16: $(tail -1 $O/bench_ws$ws.log | cut -c1-200)"
done
for dt in bf16 float32; do
  H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/dlt.so timeout -k 10 240 python scripts/dl_phase_timing.py $dt > $O/phase_$dt.log 2>&1 || { tail -20 $O/phase_$dt.log; exit 1; }
  grep -v amdgpu.ids $O/phase_$dt.log
done
