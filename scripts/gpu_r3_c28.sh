#!/bin/bash
# hist atomics addressed by v_bfe + v_lshl_add, UNIT (unit-weight packed) hist variant: tree tests, sweep, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c28
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tree_engine.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROWS="11000000 1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/gprof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-job > "$GRAFT_REPO_ROOT/$O/gprof.log" 2>&1 || { echo "gprof failed"; tail -20 "$GRAFT_REPO_ROOT/$O/gprof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c28/gprof/run_kernel_stats.csv")))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb.log; exit 1; }
grep -o '"ms_per_tree": [0-9.]*' $O/xgb.log
