#!/bin/bash
# full GPU tests + smoke + headline bench, then the secondary suite and the H2O-default (UniformAdaptive) GBM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PROF=0 bash scripts/gpu_r2_check.sh || exit 1
T=300 bash scripts/gpu_suite.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-job --histogram-type AUTO > gpurun_out/bench_ua.log 2>&1 || { tail gpurun_out/bench_ua.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ua.log
bash scripts/gpu_pmc_tree.sh > gpurun_out/pmc_run.log 2>&1; echo "pmc rc=$?"
