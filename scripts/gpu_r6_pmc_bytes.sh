#!/bin/bash
# r6: HBM bytes per tree kernel (FETCH_SIZE, WRITE_SIZE: one counter group per pass) on the final tree code, 11M rows
set -o pipefail
O=gpurun_out/r6/${TAG:-pmc}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 8 --warmup 2 --no-job --no-auto"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- $B > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- $B > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
python3 scripts/pmc_summary.py $O/f > $O/fetch.md && python3 scripts/pmc_summary.py $O/w > $O/write.md || exit 1
rm -rf $O/f $O/w
head -16 $O/fetch.md; head -16 $O/write.md
