#!/bin/bash
# r6: tiled ADADELTA strips (8 / 16 rows per workgroup) vs the flat per-element kernel, 10M x 784 bf16
set -o pipefail
O=gpurun_out/r6/${TAG:-dl2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "adadelta or dl_fused or dl_trainer" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
S="timeout -k 10 300 python3 scripts/bench_suite.py --which dl"
for v in "FLAT=1" "STRIP=8" "STRIP=16" "FLAT=1" "STRIP=8" "STRIP=16"; do
  env H2O_ADADELTA_$v $S > $O/dl_$v.log 2>&1 || { tail -20 $O/dl_$v.log; exit 1; }
  echo "$v $(tail -1 $O/dl_$v.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s loop", round(d["phases"]["train_loop"],4))')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 scripts/bench_suite.py --which dl > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --md --top 12 > $O/kernels.md || exit 1
rm -rf $O/db
head -8 $O/kernels.md
