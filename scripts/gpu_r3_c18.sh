#!/bin/bash
# dispatch sequence of one GBM tree at 1.375M rows (which small kernels / fills / copies a tree issues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c18
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 bench.py --rows 1375000 --steps 30 --warmup 3 --no-job > $O/run.log 2>&1 || { echo "prof failed"; tail -20 $O/run.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --sequence k_gbm_step > $O/sequence.md || exit 1
rm -rf $O/db
cat $O/sequence.md
