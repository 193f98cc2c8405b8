#!/bin/bash
# A/B of compile-time kernel variants (llama_github_io_amd/lib_alt/*.so via H2O_HIP_LIB) on the headline bench.
set -o pipefail
O=gpurun_out/r4_ab
mkdir -p $O
export TMPDIR=/tmp
for lib in default $(ls llama_github_io_amd/lib_alt/*.so 2>/dev/null); do
  tag=$(basename $lib .so)
  if [ "$lib" = default ]; then unset H2O_HIP_LIB; else export H2O_HIP_LIB=$PWD/$lib; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-job > $O/$tag.json 2> $O/$tag.err || exit $?
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['ms_per_step'])")"
done
