#!/bin/bash
set -o pipefail
O=gpurun_out/r4_dlf32d
mkdir -p $O
H2O_DL_GRAPH=0 timeout -k 10 400 python scripts/dl_f32_owb_probe.py 5000000 float32 > $O/a.log 2>&1 || { tail -8 $O/a.log; exit 1; }
grep owb $O/a.log
H2O_DL_FUSED_F32=0 timeout -k 10 400 python scripts/dl_f32_owb_probe.py 5000000 float32 > $O/b.log 2>&1 || { tail -8 $O/b.log; exit 1; }
grep owb $O/b.log
timeout -k 10 400 python scripts/dl_f32_owb_probe.py 5000000 bf16 > $O/c.log 2>&1 || { tail -8 $O/c.log; exit 1; }
grep owb $O/c.log
timeout -k 10 400 python scripts/dl_f32_owb_probe.py 3000000 float32 > $O/d.log 2>&1 || { tail -8 $O/d.log; exit 1; }
grep owb $O/d.log
