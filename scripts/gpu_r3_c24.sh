#!/bin/bash
# after the XGBoost binning fix + wave-local FILT: XGBoost 100M x 50 (100 trees) + kernel stats; GBM 11M kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c24
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tree_engine.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROWS="11000000 1375000" STEPS=50 bash scripts/gpu_rows_sweep.sh || exit 1
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb.log; exit 1; }
grep metric $O/xgb.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/xprof" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_suite.py" --which xgb --trees 30 > "$GRAFT_REPO_ROOT/$O/xprof.log" 2>&1 || { echo "xprof failed"; tail -20 "$GRAFT_REPO_ROOT/$O/xprof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/gprof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-job > "$GRAFT_REPO_ROOT/$O/gprof.log" 2>&1 || { echo "gprof failed"; tail -20 "$GRAFT_REPO_ROOT/$O/gprof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > $O/bench100.log 2>&1 || { echo "bench failed"; tail $O/bench100.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench100.log
exit 0
