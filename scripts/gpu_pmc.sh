#!/bin/bash
# One PMC pass (LDS bank conflicts / LDS activity per kernel) over a short bench run.
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc ${PMC:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES} --output-format csv \
  -d "$R/gpurun_out/pmc" -o run -- python3 "$R/bench.py" --steps ${STEPS:-3} --warmup 1 > "$R/gpurun_out/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 "$R/gpurun_out/pmc.log"; exit $rc
