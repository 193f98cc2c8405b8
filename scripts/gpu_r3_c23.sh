#!/bin/bash
# wave-local FILT queues: tree GPU tests, rows sweep, XGBoost 100M x 50 host phases + kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c23
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tree_engine.py tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROWS="11000000 1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
H2O_HOST_PROF=1 timeout -k 10 300 python scripts/bench_suite.py --which xgb --trees 30 > $O/xgb_host.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb_host.log; exit 1; }
grep -E "host-prof|metric" $O/xgb_host.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_suite.py" --which xgb --trees 30 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || { echo "prof failed"; tail -20 "$GRAFT_REPO_ROOT/$O/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/c23/prof/**/*kernel_stats.csv", recursive=True))
rows = list(csv.DictReader(open(f[0])))
for r in rows[:25]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
