#!/bin/bash
# r5: RCCL trainer tier + GBM/XGB step tests, then the tree check (hist A/B, tests, bench, sequence)
set -o pipefail
O=gpurun_out/r5/${TAG:-c7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rccl_trainers_gpu.py -m gpu > $O/rccl.log 2>&1 || { tail -60 $O/rccl.log; exit 1; }
tail -2 $O/rccl.log
./scripts/gpu_r5_hab.sh || exit 1
TAG=${TAG:-c7} ./scripts/gpu_r5_tree.sh
