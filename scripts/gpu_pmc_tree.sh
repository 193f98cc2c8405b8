#!/bin/bash
# PMC counters of the tree kernels on a short bench run (counters only with --kernel-trace; one pass per group)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 bench.py --steps 3 --warmup 2 --rows 11000000 --no-job > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 bench.py --steps 3 --warmup 2 --rows 11000000 --no-job > gpurun_out/pmc/p2.log 2>&1
rc=$?
ls -R gpurun_out/pmc | head -20
exit $rc
