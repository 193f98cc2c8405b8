#!/bin/bash
set -o pipefail
O=gpurun_out/r5/mb4
mkdir -p $O
timeout -k 10 200 ./scripts/mb_hist4.bin > $O/mb_hist4.log 2>&1 || { echo "mb failed"; cat $O/mb_hist4.log; exit 1; }
cat $O/mb_hist4.log
