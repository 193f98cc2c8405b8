#!/bin/bash
# PMC passes over the headline bench (3 trees): where the histogram kernels' wave cycles go.
set -o pipefail
O=gpurun_out/r5/pmc1
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 2 --no-job"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/p1 > $O/p1.md && python3 scripts/pmc_summary.py $O/p2 > $O/p2.md || exit 1
rm -rf $O/p1 $O/p2
head -8 $O/p1.md; head -8 $O/p2.md
M=./scripts/mb_hist4.bin
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/m1 -o m1 -- $M > $O/m1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $O/m2 -o m2 -- $M > $O/m2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/m1 > $O/m1.md && python3 scripts/pmc_summary.py $O/m2 > $O/m2.md || exit 1
rm -rf $O/m1 $O/m2
cat $O/m1.md $O/m2.md
