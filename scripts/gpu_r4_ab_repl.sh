#!/bin/bash
# Same-box A/B of histogram settings: low-cardinality bin replicas (H2O_HIST_REPL=0 turns them off) and the
# histogram grid (H2O_HIST_GRID: blocks per launch; 256 = one 16-wave block per CU, 512 = two).
set -o pipefail
O=gpurun_out/r4_ab_repl
mkdir -p $O
export TMPDIR=/tmp
run() {  # name rows steps env...
  local n=$1 r=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --rows $r --steps $st --warmup 5 --no-job > $O/$n.json 2> $O/$n.err || return $?
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['ms_per_step'])"
}
for i in 1 2; do
  run on_$i 11000000 20 H2O_HIST_REPL=1 || exit $?
  run off_$i 11000000 20 H2O_HIST_REPL=0 || exit $?
  run g512_$i 11000000 20 H2O_HIST_GRID=512 || exit $?
done
run g384 11000000 20 H2O_HIST_GRID=384 || exit $?
run on_1375k 1375000 50 H2O_HIST_REPL=1 || exit $?
run off_1375k 1375000 50 H2O_HIST_REPL=0 || exit $?
run g512_1375k 1375000 50 H2O_HIST_GRID=512 || exit $?
