#!/bin/bash
# KMeans: bank-friendly LDS stride, PS=6 variant for P <= 24, one resident round of blocks: GPU kernel tests,
# step timing, end-to-end suite line, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c32
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "kmeans or lloyd" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/bench_kmeans_step.py > $O/step.log 2>&1 || { tail $O/step.log; exit 1; }
grep kernel $O/step.log
timeout -k 10 300 python scripts/bench_suite.py --which kmeans > $O/suite.log 2>&1 || { tail $O/suite.log; exit 1; }
grep metric $O/suite.log | cut -c1-300
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o km -- python3 "$GRAFT_REPO_ROOT/scripts/bench_kmeans_step.py" > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/$O/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c32/prof/km_kernel_stats.csv")))
for r in rows[:3]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
