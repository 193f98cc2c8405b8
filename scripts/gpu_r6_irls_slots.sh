#!/bin/bash
# NOTE: ran against a templated k_gram_irls<LG> (H2O_GRAM_IRLS_SLOTS) that was measured and reverted; see profiles/r6_gram_irls_slots_ab.md
# r6: k_gram_irls row slots per batch A/B (8 = default, 4 = 4 waves / SIMD) — numerics at 4, GLM 10M x 50 records, kernel time
set -o pipefail
O=gpurun_out/r6/${TAG:-irls_slots}
mkdir -p $O
export TMPDIR=/tmp
H2O_GRAM_IRLS_SLOTS=4 timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_glm_irls_gpu.py > $O/tests4.log 2>&1 || { tail -30 $O/tests4.log; exit 1; }
tail -1 $O/tests4.log
for i in 1 2; do
  H2O_GRAM_IRLS_SLOTS=8 timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/s8.jsonl 2>> $O/err.log || exit 1
  H2O_GRAM_IRLS_SLOTS=4 timeout -k 10 200 python3 scripts/bench_suite.py --which glm_big >> $O/s4.jsonl 2>> $O/err.log || exit 1
done
cut -c1-100 $O/s8.jsonl $O/s4.jsonl
for s in 8 4; do
  H2O_GRAM_IRLS_SLOTS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db$s -o run -- python3 scripts/bench_suite.py --which glm_big > $O/prof$s.log 2>&1 || { tail -20 $O/prof$s.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/db$s/run_results.db --md --top 4 > $O/kernels$s.md || exit 1
  rm -rf $O/db$s
  grep k_gram_irls $O/kernels$s.md
done
