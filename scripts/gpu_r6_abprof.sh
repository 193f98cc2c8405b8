#!/bin/bash
# r6: per-kernel tree sequences of the previous commit's tree (_ab_old) and this tree on the same box
set -o pipefail
O=gpurun_out/r6/${TAG:-abprof}
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
(cd $R/_ab_old && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/db_old -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --no-auto) > $O/prof_old.log 2>&1 || { tail -20 $O/prof_old.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db_new -o run -- python3 bench.py --steps 14 --warmup 2 --no-job --no-auto > $O/prof_new.log 2>&1 || { tail -20 $O/prof_new.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db_old/run_results.db --sequence k_gbm_step > $O/seq_old.md || exit 1
python3 scripts/rocpd_stats.py $O/db_new/run_results.db --sequence k_gbm_step > $O/seq_new.md || exit 1
rm -rf $O/db_old $O/db_new
paste -d'|' <(cut -d'|' -f2-4 $O/seq_old.md) <(cut -d'|' -f4 $O/seq_new.md) | head -40
