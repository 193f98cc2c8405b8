#!/bin/bash
# Same-box A/B of the histogram's low-cardinality bin replicas (H2O_HIST_REPL=0 turns them off), alternated twice.
set -o pipefail
O=gpurun_out/r4_ab_repl
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-job > $O/on_$i.json 2> $O/on_$i.err || exit $?
  H2O_HIST_REPL=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-job > $O/off_$i.json 2> $O/off_$i.err || exit $?
done
timeout -k 10 200 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/on_1375k.json 2> $O/on_1375k.err || exit $?
H2O_HIST_REPL=0 timeout -k 10 200 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/off_1375k.json 2> $O/off_1375k.err || exit $?
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'])"; done
