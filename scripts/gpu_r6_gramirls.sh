#!/bin/bash
# r6: fused IRLS + Gram pass (k_gram_irls) — numerics tests, then GLM 10M x 50 A/B (two-pass vs fused), kernel table
set -o pipefail
O=gpurun_out/r6/${TAG:-gramirls}
mkdir -p $O
export TMPDIR=/tmp
H2O_GLM_GRAM_IRLS=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_glm_irls_gpu.py \
  tests/test_kernels_gpu.py -k "glm or gram" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  H2O_GLM_GRAM_IRLS=0 timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/ab_twopass.jsonl 2>> $O/ab.err || exit 1
  H2O_GLM_GRAM_IRLS=1 timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/ab_fused.jsonl 2>> $O/ab.err || exit 1
done
cat $O/ab_twopass.jsonl $O/ab_fused.jsonl
H2O_GLM_GRAM_IRLS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 30 > $O/kernels.md || exit 1
rm -rf $O/db
head -12 $O/kernels.md
