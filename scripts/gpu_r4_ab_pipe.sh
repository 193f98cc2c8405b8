#!/bin/bash
# A/B of the plain-pass software pipeline and of a 64-VGPR (two blocks per CU) histogram build, same box.
set -o pipefail
O=gpurun_out/r4_ab_pipe
mkdir -p $O
export TMPDIR=/tmp
L=llama_github_io_amd/lib_alt
run() {  # name lib rows steps env...
  local n=$1 lib=$2 r=$3 st=$4; shift 4
  if [ "$lib" = default ]; then unset H2O_HIP_LIB; else export H2O_HIP_LIB=$PWD/$L/$lib.so; fi
  env "$@" timeout -k 10 200 python bench.py --rows $r --steps $st --warmup 5 --no-job > $O/$n.json 2> $O/$n.err || return $?
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['ms_per_step'])"
}
for i in 1 2; do
  run pipe_$i default 11000000 20 || exit $?
  run nopipe_$i nopipe 11000000 20 || exit $?
done
run minw8_g512 minw8 11000000 20 H2O_HIST_GRID=512 || exit $?
run minw8u4_g512 minw8u4 11000000 20 H2O_HIST_GRID=512 || exit $?
run pipe_1375k default 1375000 50 || exit $?
run nopipe_1375k nopipe 1375000 50 || exit $?
unset H2O_HIP_LIB
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_engine.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
