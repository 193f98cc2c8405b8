#!/bin/bash
set -o pipefail
O=gpurun_out/r4_dlf32c
mkdir -p $O
timeout -k 10 400 python scripts/dl_f32_owb_probe.py 5000000 > $O/probe.log 2>&1 || { tail -8 $O/probe.log; exit 1; }
grep owb $O/probe.log
H2O_DL_CHUNK=1 timeout -k 10 400 python scripts/dl_f32_owb_probe.py 5000000 > $O/probe_ch1.log 2>&1 || { tail -8 $O/probe_ch1.log; exit 1; }
grep owb $O/probe_ch1.log
