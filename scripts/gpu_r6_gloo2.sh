#!/bin/bash
# r6: rehearsal of the multi-rank bench on ONE GPU — two ranks on cuda:0 over gloo (RCCL refuses two ranks on one
# device): the row-sharded native driver with host-staged collectives, the bench's barrier / max-over-ranks timing
set -o pipefail
O=gpurun_out/r6/${TAG:-gloo2}
mkdir -p $O
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29617 WORLD_SIZE=2 LOCAL_RANK=0
B="python3 bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-job --no-auto --rows 2750000"
RANK=1 timeout -k 10 400 $B > $O/rank1.log 2>&1 &
p1=$!
RANK=0 timeout -k 10 400 $B > $O/rank0.log 2>&1
rc0=$?
wait $p1
rc1=$?
echo "rc0=$rc0 rc1=$rc1"
tail -1 $O/rank0.log | cut -c1-600
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ]
