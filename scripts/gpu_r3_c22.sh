#!/bin/bash
# XGBoost 100M x 50 slowdown hunt: host phase profile + rocprofv3 kernel stats (30 trees)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c22
mkdir -p $O
H2O_HOST_PROF=1 timeout -k 10 300 python scripts/bench_suite.py --which xgb --trees 30 > $O/xgb_host.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb_host.log; exit 1; }
grep -E "host-prof|metric" $O/xgb_host.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_suite.py" --which xgb --trees 30 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || { echo "prof failed"; tail -20 "$GRAFT_REPO_ROOT/$O/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c22/prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/c22/prof/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
for r in rows[:25]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
