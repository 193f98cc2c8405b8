#!/bin/bash
# One gpurun call: GPU tests, smoke, short bench, rocprofv3 kernel stats. Stops at the first crash.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
ok() { [ "$1" -eq 0 ]; }   # any failure stops the call: a wrong kernel can fault the next step
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1; rc=$?
  echo "prof rc=$rc"; tail -3 "$R/gpurun_out/prof.log"
  find "$R/gpurun_out/prof" -name "*stats*" | head
fi
