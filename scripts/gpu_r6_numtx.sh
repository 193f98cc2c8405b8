#!/bin/bash
# r6: k_num_transform whole-row span store + in-kernel intercept column — tests, GLM 10M x 50 bench, kernel table
set -o pipefail
O=gpurun_out/r6/${TAG:-numtx}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_glm_irls_gpu.py -k "expander or glm or gram" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/glm.jsonl 2>> $O/glm.err || exit 1
done
cut -c1-140 $O/glm.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 30 > $O/kernels.md || exit 1
rm -rf $O/db
head -14 $O/kernels.md
