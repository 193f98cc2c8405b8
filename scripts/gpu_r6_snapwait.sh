#!/bin/bash
# r6: bounded lookahead of the tree snapshots (wait for the oldest tree instead of a pinned allocation):
# tree GPU tests, A/B of H2O_TREE_SNAP_WAIT at 1.375M and 11M, a 1.375M timeline with the default
set -o pipefail
O=gpurun_out/r6/${TAG:-snapwait}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py tests/test_native_comm_gpu.py tests/test_kernels_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-job --no-auto"
ms() { tail -1 $1 | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])'; }
for w in 1 0 1 0; do
  H2O_TREE_SNAP_WAIT=$w $B --rows 1375000 > $O/b1375k_w$w.log 2>&1 || { tail -20 $O/b1375k_w$w.log; exit 1; }
  H2O_TREE_SNAP_WAIT=$w $B > $O/b11m_w$w.log 2>&1 || { tail -20 $O/b11m_w$w.log; exit 1; }
  echo "wait=$w 1.375M $(ms $O/b1375k_w$w.log) 11M $(ms $O/b11m_w$w.log)"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "driver window $(ms $O/bench.log) job $(tail -1 $O/bench.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["config"]["job_100_trees_ms_incl_binning_and_metrics"])')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 bench.py --steps 30 --warmup 5 --no-job --no-auto --rows 1375000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --timeline k_gbm_step > $O/timeline_1375000.md || exit 1
rm -rf $O/db
echo "below-90%: $(awk -F'|' 'NR>2 && $5+0 < 90 {printf "%s:%s%% ", $2+0, $5+0}' $O/timeline_1375000.md)"
