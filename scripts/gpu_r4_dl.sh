#!/bin/bash
# DeepLearning fused MFMA step: bf16 + fp32 GPU tests, benches (2M rows and the 1.25M-row per-rank shard of 8 GPUs),
# and a kernel trace of the default fp32 loop (no library GEMM kernels expected).
set -o pipefail
O=gpurun_out/r4_dl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "dl_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python scripts/bench_suite.py --which dl --rows 2000000 --dtype bf16 > $O/bench_bf16.json 2> $O/bench_bf16.err || exit $?
timeout -k 10 300 python scripts/bench_suite.py --which dl --rows 2000000 --dtype float32 > $O/bench_f32.json 2> $O/bench_f32.err || exit $?
timeout -k 10 300 python scripts/bench_suite.py --which dl --rows 1250000 --dtype bf16 > $O/bench_bf16_shard.json 2> $O/bench_bf16_shard.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o run -- python scripts/bench_suite.py --which dl --rows 1000000 --dtype float32 > $O/prof_f32.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/prof_f32/run_results.db --top 30 --md > $O/kernel_stats_f32.md || exit 1
rm -rf $O/prof_f32
cat $O/bench_bf16.json $O/bench_f32.json $O/bench_bf16_shard.json
