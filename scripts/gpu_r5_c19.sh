#!/bin/bash
set -o pipefail
O=gpurun_out/r5/c19
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/fit_profile.py --which dl > $O/dl_profile.log 2>&1 || { tail -30 $O/dl_profile.log; exit 1; }
head -60 $O/dl_profile.log | cut -c1-200
