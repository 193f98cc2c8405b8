#!/bin/bash
# r6: GLM 10M x 50 after the metrics changes (masked lattice rows, numpy threshold table): tests, 3 records, window
set -o pipefail
O=gpurun_out/r6/${TAG:-glm3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_metrics_gpu.py \
  tests/test_glm_irls_gpu.py tests/test_kernels_gpu.py -k "metric or glm or gram or auc or expander" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/glm.jsonl 2>> $O/glm.err || exit 1
done
cut -c1-140 $O/glm.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --window k_num_stats --top 40 > $O/window.md || exit 1
rm -rf $O/db
head -12 $O/window.md
