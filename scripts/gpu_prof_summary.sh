#!/bin/bash
# usage: gpu_prof_summary.sh <name> <python args...>: rocprofv3 kernel trace of one script run, summarised
# on the box (the rocpd database itself is deleted: gpurun copies back at most 64 MiB)
set -o pipefail
name=$1; shift
O=gpurun_out/prof_$name
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/db -o run -- python3 "$@" > $O/run.log 2>&1 || { echo "prof $name failed"; tail -20 $O/run.log; exit 1; }
python3 scripts/rocpd_stats.py $O/db/run_results.db --top 30 --md > $O/kernel_stats.md || exit 1
rm -rf $O/db
tail -2 $O/run.log
head -8 $O/kernel_stats.md
