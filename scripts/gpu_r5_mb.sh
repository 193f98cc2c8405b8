#!/bin/bash
# r5: LDS histogram primitive rates + driver-window headline bench on the current tree
set -o pipefail
O=gpurun_out/r5/mb
mkdir -p $O
timeout -k 10 120 ./scripts/mb_hist2.bin > $O/mb_hist2.log 2>&1 || { echo "mb failed"; cat $O/mb_hist2.log; exit 1; }
cat $O/mb_hist2.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log
