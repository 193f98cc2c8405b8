#!/bin/bash
# final check of the session: every GPU test, smoke, headline bench (driver shape), rows sweep, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PROF=1 bash scripts/gpu_r2_check.sh || exit 1
ROWS="11000000 5500000 2750000 1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
