#!/bin/bash
# 1-GPU rehearsal of the 8-GPU per-rank shard (1.375M rows = 11M / 8): the single-process tree vs the
# row-sharded native driver on a 1-rank RCCL communicator (H2O_TREE_COMM_FORCE), plus a kernel trace of the
# latter. Output under gpurun_out/r4_rehearsal/.
set -o pipefail
O=gpurun_out/r4_rehearsal
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/single.json 2> $O/single.err || exit $?
H2O_TREE_COMM_FORCE=ar timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/force_ar.json 2> $O/force_ar.err || exit $?
H2O_TREE_COMM_FORCE=rs timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --no-job > $O/force_rs.json 2> $O/force_rs.err || exit $?
H2O_TREE_COMM_FORCE=ar timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ar -o run -- python bench.py --rows 1375000 --steps 30 --warmup 5 --no-job > $O/prof_ar.log 2>&1 || exit $?
cat $O/single.json $O/force_ar.json $O/force_rs.json
