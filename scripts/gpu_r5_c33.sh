#!/bin/bash
# Issue / LDS counters of the headline tree kernels (what bounds the histogram passes and routes)
set -o pipefail
O=gpurun_out/r5/c33
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d $O/p1 -o p1 -- $B > $O/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $O/p2 -o p2 -- $B > $O/p2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/p1 > $O/p1.md && python3 scripts/pmc_summary.py $O/p2 > $O/p2.md || exit 1
head -12 $O/p1.md; head -12 $O/p2.md
