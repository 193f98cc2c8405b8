#!/bin/bash
# r6: single-wave plan for levels of <= 64 nodes (H2O_PLAN_WAVE=1 default / 0 block plan) + DL ADADELTA strips
set -o pipefail
O=gpurun_out/r6/${TAG:-wave}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_kernels_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-job --no-auto"
ms() { tail -1 $1 | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])'; }
for w in 1 0 1 0; do
  H2O_PLAN_WAVE=$w $B --rows 1375000 > $O/b1375k_w$w.log 2>&1 || { tail -20 $O/b1375k_w$w.log; exit 1; }
  H2O_PLAN_WAVE=$w $B > $O/b11m_w$w.log 2>&1 || { tail -20 $O/b11m_w$w.log; exit 1; }
  echo "wave=$w 1.375M $(ms $O/b1375k_w$w.log) 11M $(ms $O/b11m_w$w.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --no-auto --rows 1375000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/seq_1375k.md || exit 1
rm -rf $O/db
S="timeout -k 10 300 python3 scripts/bench_suite.py --which dl"
for v in "FLAT=1" "STRIP=8" "STRIP=16" "FLAT=1" "STRIP=8" "STRIP=16"; do
  env H2O_ADADELTA_$v $S > $O/dl_$v.log 2>&1 || { tail -20 $O/dl_$v.log; exit 1; }
  echo "$v $(tail -1 $O/dl_$v.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s loop", round(d["phases"]["train_loop"],4))')"
done
cat $O/seq_1375k.md | head -40
