#!/bin/bash
# striped leaf-sum atomics + column compression: full GPU suite, GBM bench (11M) and 1.375M rehearsal + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c17
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
ROWS="1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
bash scripts/gpu_prof_summary.sh gbm1375k bench.py --rows 1375000 --steps 50 --warmup 5 --no-job || exit 1
