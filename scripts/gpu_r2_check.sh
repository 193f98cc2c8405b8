#!/bin/bash
# Round-2 GPU check: GPU tests + smoke + 1-GPU headline bench + rocprofv3 kernel stats of the bench
# (each step time-limited, chained with &&; stops at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
{ [ "${PROF:-1}" != "1" ] || { cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1; }; }
rc=$?
cd "$R"
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -2 gpurun_out/bench.log
exit $rc
