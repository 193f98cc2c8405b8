#!/bin/bash
# GBM bench: fixed overhead of the 20-step window (warmup vs steady state), per-tree timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c9
mkdir -p $O
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-job > $O/b20w5.log 2>&1 || { echo "bench failed"; tail -20 $O/b20w5.log; exit 1; }
tail -1 $O/b20w5.log | cut -c1-300
timeout -k 10 180 python bench.py --steps 20 --warmup 40 --no-job > $O/b20w40.log 2>&1 || { echo "bench failed"; tail -20 $O/b20w40.log; exit 1; }
tail -1 $O/b20w40.log | cut -c1-300
H2O_HOST_PROF=1 timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-job > $O/hostprof.log 2>&1 || { echo "bench failed"; tail -20 $O/hostprof.log; exit 1; }
grep host-prof $O/hostprof.log | tail -2
mkdir -p $O/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl/db -o run -- python3 bench.py --steps 20 --warmup 5 --no-job > $O/tl/run.log 2>&1 || { echo "prof failed"; tail -20 $O/tl/run.log; exit 1; }
python3 scripts/rocpd_stats.py $O/tl/db/run_results.db --timeline k_gbm_step > $O/timeline.md || exit 1
rm -rf $O/tl/db
cat $O/timeline.md
