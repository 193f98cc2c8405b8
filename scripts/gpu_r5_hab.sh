#!/bin/bash
set -o pipefail
O=gpurun_out/r5/hab
mkdir -p $O
timeout -k 10 300 python3 scripts/hist_ab.py > $O/hist_ab.log 2>&1 || { tail -30 $O/hist_ab.log; exit 1; }
tail -2 $O/hist_ab.log
