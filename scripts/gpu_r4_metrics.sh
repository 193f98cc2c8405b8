#!/bin/bash
set -o pipefail
O=gpurun_out/r4_metrics
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "metric or auc or gains or dl or deep" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python scripts/bench_suite.py --which dl > $O/dl10m.log 2>&1 || { tail -5 $O/dl10m.log; exit 1; }
tail -1 $O/dl10m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases'])"
