#!/bin/bash
set -o pipefail
O=gpurun_out/r5/mbld
mkdir -p $O
timeout -k 10 200 ./scripts/mb_ld.bin > $O/mb_ld.log 2>&1 || { echo "mb failed"; cat $O/mb_ld.log; exit 1; }
cat $O/mb_ld.log
