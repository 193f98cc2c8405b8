#!/bin/bash
# Alternative builds of the HIP library with compile-time kernel variants: llama_github_io_amd/lib_alt/<tag>.so
# usage: scripts/build_alt.sh <tag> <-Dflags...>   (A/B on the box through H2O_HIP_LIB)
set -e
tag=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/llama_github_io_amd/csrc
O=$R/llama_github_io_amd/lib_alt
mkdir -p $O/obj_$tag
objs=()
for f in $C/*.hip; do
  o=$O/obj_$tag/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $f -o $o -I $C -Wno-unused-result
  objs+=($o)
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/$tag.so "${objs[@]}" -ldl
rm -rf $O/obj_$tag
echo built $O/$tag.so
