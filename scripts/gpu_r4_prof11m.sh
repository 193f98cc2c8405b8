#!/bin/bash
# Headline shape (11M x 28, depth 6): bench line + kernel trace of 20 trees (no 100-tree job), per-tree
# sequence / timeline. Output under gpurun_out/r4_prof11m/.
set -o pipefail
O=gpurun_out/r4_prof11m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-job > $O/prof.log 2>&1 || exit $?
cat $O/bench.json
