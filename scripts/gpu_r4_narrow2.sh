#!/bin/bash
# Three-tier narrow levels: tree-engine GPU tests, AUTO / QG bench, AUTO profile + tree sequence; DL phase clocks.
set -o pipefail
[ -f llama_github_io_amd/lib_alt/dlt.so ] || bash scripts/build_alt.sh dlt -DDL_TIMING > /dev/null || exit 1
O=gpurun_out/r4_narrow2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --histogram-type AUTO --steps 30 --warmup 3 > $O/bench_auto.json 2> $O/bench_auto.err || { tail -20 $O/bench_auto.err; exit 1; }
cat $O/bench_auto.json
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > $O/bench_qg.json 2> $O/bench_qg.err || exit 1
cat $O/bench_qg.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --histogram-type AUTO --steps 12 --warmup 2 --no-job > $O/prof.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
python3 scripts/rocpd_stats.py $O/prof/run_results.db --sequence k_gbm_step --md > $O/tree_sequence.md || true
rm -rf $O/prof
head -14 $O/kernel_stats.md
for dt in bf16; do
  H2O_HIP_LIB=$PWD/llama_github_io_amd/lib_alt/dlt.so timeout -k 10 240 python scripts/dl_phase_timing.py $dt > $O/phase_$dt.log 2>&1 || { tail -20 $O/phase_$dt.log; exit 1; }
  grep -v amdgpu.ids $O/phase_$dt.log
done
timeout -k 10 200 python scripts/bench_suite.py --which dl --rows 2000000 --dtype bf16 > $O/dl_bf16.log 2>&1 || exit 1
tail -1 $O/dl_bf16.log | cut -c1-300
