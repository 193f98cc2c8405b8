#!/bin/bash
# r6: DeepLearning 10M x 784 bf16 — the tiled ADADELTA update (64 x 64 tiles, transposed copy through LDS) against
# the per-element kernel, a batch-size row, and a kernel table / idle-gap list of the fit
set -o pipefail
O=gpurun_out/r6/${TAG:-dl}
mkdir -p $O
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "adadelta or dl or deeplearning" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py --which dl"
for v in 0 1 0; do
  H2O_ADADELTA_FLAT=$v $S > $O/dl_flat$v.log 2>&1 || { tail -20 $O/dl_flat$v.log; exit 1; }
  echo "flat=$v $(tail -1 $O/dl_flat$v.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s", d["phases"])')"
done
$S --batch 8192 > $O/dl_b8192.log 2>&1 || { tail -20 $O/dl_b8192.log; exit 1; }
echo "batch 8192 $(tail -1 $O/dl_b8192.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s logloss", d["train_logloss"])')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which dl > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 25 > $O/kernels.md || exit 1
python3 scripts/rocpd_stats.py $O/db/run_results.db --gaps k_num_stats --min-gap 20 > $O/gaps.md || exit 1
rm -rf $O/db
head -20 $O/kernels.md
head -3 $O/gaps.md
