#!/bin/bash
# r6: same-box A/B of the headline bench: the previous commit's tree (_ab_old, own build) vs this tree, alternating
set -o pipefail
O=gpurun_out/r6/${TAG:-ab}
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
for i in 1 2 3; do
  (cd $R/_ab_old && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job --no-auto) > $O/old$i.log 2>&1 || { cat $O/old$i.log; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-job --no-auto > $O/new$i.log 2>&1 || { cat $O/new$i.log; exit 1; }
  echo "old $(python3 -c "import json;print(json.loads(open('$O/old$i.log').read().strip().splitlines()[-1])['ms_per_step'])") new $(python3 -c "import json;print(json.loads(open('$O/new$i.log').read().strip().splitlines()[-1])['ms_per_step'])")"
done
