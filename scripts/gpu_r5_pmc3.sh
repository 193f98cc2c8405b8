#!/bin/bash
# HBM bytes per tree kernel (TCC FETCH_SIZE / WRITE_SIZE, KB) on the headline bench: does the filtered pass read
# the selected rows twice (direction bytes, then the gathered words)?
set -o pipefail
O=gpurun_out/r5/pmc3
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 2 --no-job"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- $B > $O/f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- $B > $O/w.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/f > $O/fetch.md && python3 scripts/pmc_summary.py $O/w > $O/write.md || exit 1
rm -rf $O/f $O/w
head -14 $O/fetch.md; head -14 $O/write.md
