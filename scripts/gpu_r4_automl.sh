#!/bin/bash
# AutoML on 1M x 100 (GBM + DRF + GLM + DL + StackedEnsemble) with a 600 s budget, leader MOJO round trip.
set -o pipefail
O=gpurun_out/r4_automl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/bench_suite.py --which automl --budget 600 > $O/automl.json 2> $O/automl.err || { tail -20 $O/automl.err; exit 1; }
cat $O/automl.json
