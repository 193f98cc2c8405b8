#!/bin/bash
set -o pipefail
O=gpurun_out/r4_commnarrow
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_comm_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python scripts/bench_suite.py --which dl --dtype float32 > $O/dl10m_f32.log 2>&1 || { tail -5 $O/dl10m_f32.log; exit 1; }
tail -1 $O/dl10m_f32.log | cut -c1-300
