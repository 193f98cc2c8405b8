#!/bin/bash
# KMeans Lloyd step: timing, kernel stats, PMC (VALU / LDS / bank conflicts) of k_lloyd_mfma
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c31
mkdir -p $O
timeout -k 10 200 python scripts/bench_kmeans_step.py > $O/step.log 2>&1 || { tail $O/step.log; exit 1; }
cat $O/step.log | grep kernel
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o km -- python3 "$GRAFT_REPO_ROOT/scripts/bench_kmeans_step.py" > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/$O/prof.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc" -o p1 -- python3 "$GRAFT_REPO_ROOT/scripts/bench_kmeans_step.py" > "$GRAFT_REPO_ROOT/$O/pmc.log" 2>&1
echo "pmc rc=$?"
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c31/prof/km_kernel_stats.csv")))
for r in rows[:6]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
python3 scripts/pmc_summary.py gpurun_out/c31/pmc | head -6
