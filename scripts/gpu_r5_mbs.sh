#!/bin/bash
set -o pipefail
O=gpurun_out/r5/mbs
mkdir -p $O
timeout -k 10 200 ./scripts/mb_stream.bin > $O/mb_stream.log 2>&1 || { echo "mb failed"; cat $O/mb_stream.log; exit 1; }
cat $O/mb_stream.log
