#!/bin/bash
# full GPU suite (after the sharded CoxPH/PSVM/Aggregator/Isotonic work + packed bin-assign kernel),
# XGBoost 100M x 50 planar vs row-major A/B on the same box, GBM bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c13
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb_planar.log 2>&1 || { echo "xgb failed"; tail -20 $O/xgb_planar.log; exit 1; }
tail -1 $O/xgb_planar.log | cut -c1-400
H2O_BINS_ROWMAJOR=1 timeout -k 10 400 python scripts/bench_suite.py --which xgb --trees 100 > $O/xgb_rowmajor.log 2>&1 || { echo "xgb rowmajor failed"; tail -20 $O/xgb_rowmajor.log; exit 1; }
tail -1 $O/xgb_rowmajor.log | cut -c1-400
bash scripts/gpu_prof_summary.sh xgb scripts/bench_suite.py --which xgb --trees 30 || exit 1
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
