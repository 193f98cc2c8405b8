#!/bin/bash
# Leaf-assign LDS leaf sums striped over 8 lane copies (H2O_LEAF_COPIES A/B) + tree tests + leaf-assign counters
set -o pipefail
O=gpurun_out/r5/c34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_engine.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 1 8 1 8 4; do
  H2O_LEAF_COPIES=$c timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_c$c.log 2>&1 || { tail -30 $O/bench_c$c.log; exit 1; }
  echo "copies=$c $(tail -1 $O/bench_c$c.log | cut -c150-230)"
done
B="python3 bench.py --steps 3 --warmup 1"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- $B > $O/ks.log 2>&1 || exit $?
grep -h "leaf_assign" $O/ks/*kernel_stats.csv | cut -c1-200
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/p2 > $O/p2.md && grep -E "kernel|leaf_assign" $O/p2.md
