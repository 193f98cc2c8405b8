#!/bin/bash
# H2O-default histogram (AUTO = UniformAdaptive over 1016 wide edges): bench + per-kernel profile.
set -o pipefail
O=gpurun_out/r4_auto
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --histogram-type AUTO --steps 10 --warmup 3 > $O/bench_auto.json 2> $O/bench_auto.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --histogram-type AUTO --steps 5 --warmup 2 --no-job > $O/prof.log 2>&1 || exit $?
cat $O/bench_auto.json
