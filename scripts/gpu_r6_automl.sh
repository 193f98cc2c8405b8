#!/bin/bash
# BASELINE config 5 shape: AutoML (GBM + DRF + GLM + DL + XGBoost + StackedEnsembles) on 1M x 100 with a 900 s budget
# (a gpurun call is capped at 1200 s, so the 1 h budget of the BASELINE cannot run in one call), leader MOJO round trip.
set -o pipefail
O=gpurun_out/r6/automl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1140 python3 -u scripts/bench_suite.py --which automl --budget ${BUDGET:-900} > $O/automl.json 2> $O/automl.err || { tail -20 $O/automl.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/automl.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ('value','seconds','leader','leader_auc','mojo_max_abs_diff','algos')})"
