#!/bin/bash
set -o pipefail
O=gpurun_out/r5/mb3
mkdir -p $O
timeout -k 10 120 ./scripts/mb_hist3.bin > $O/mb_hist3.log 2>&1 || { echo "mb failed"; cat $O/mb_hist3.log; exit 1; }
cat $O/mb_hist3.log
