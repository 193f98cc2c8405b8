#!/bin/bash
# DL bench loops: bf16 / fp32, serial vs Hogwild two-stream steps (H2O_DL_HOGWILD=1), plus a bf16 kernel profile.
set -o pipefail
O=gpurun_out/r4_dlprof
mkdir -p $O
export TMPDIR=/tmp
for dt in bf16 float32; do
  for hw in 0 1; do
    H2O_DL_HOGWILD=$hw timeout -k 10 200 python scripts/bench_suite.py --which dl --rows 2000000 --dtype $dt > $O/b_${dt}_$hw.json 2> $O/b_${dt}_$hw.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${dt}_$hw.json')); print('$dt hogwild=$hw', round(d['value']/1e6,2), 'M/s loop', round(d['phases']['train_loop'],4), 'auc', round(d['train_auc'],4))"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_bf16 -o run -- python scripts/bench_suite.py --which dl --rows 2000000 --dtype bf16 > $O/run_bf16.log 2>&1 || exit $?
python3 scripts/rocpd_stats.py $O/p_bf16/run_results.db --top 12 --md > $O/kernel_stats_bf16.md && rm -rf $O/p_bf16
head -9 $O/kernel_stats_bf16.md
