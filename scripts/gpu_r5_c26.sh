#!/bin/bash
# KMeans phased Lloyd kernel PMC (issue / wait breakdown, instruction mix, MFMA busy)
set -o pipefail
O=gpurun_out/r5/c26
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*" $O/avail.txt | sort -u > $O/mfma_counters.txt || true
cat $O/mfma_counters.txt
B="python3 scripts/bench_suite.py --which kmeans --rows 2000000"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/p1 > $O/p1.md && python3 scripts/pmc_summary.py $O/p2 > $O/p2.md || exit 1
rm -rf $O/p1 $O/p2
if grep -q "SQ_VALU_MFMA_BUSY_CYCLES" $O/mfma_counters.txt; then
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p3 -o p3 -- $B > $O/p3.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py $O/p3 > $O/p3.md || exit 1
  rm -rf $O/p3
fi
grep -h -E "kernel|lloyd" $O/p*.md | cut -c1-400
