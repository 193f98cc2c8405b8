#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_r3_c6.sh || exit 1
bash scripts/gpu_r3_c5.sh || exit 1
