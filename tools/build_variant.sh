#!/bin/bash
# Build a variant library (one source recompiled with extra -D flags) into fastconsensus_amd/lib/<name>/
# (CPU host; run `python -m fastconsensus_amd.build` first for the other objects).
#   tools/build_variant.sh <name> <source: cd.hip | cd_rl.hip | ...> -DFLAG ...
set -eu
name=$1; src=$2; shift 2
L=fastconsensus_amd/lib
mkdir -p $L/$name
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude "$@" -x hip -c fastconsensus_amd/csrc/$src -o $L/$name/$src.o
objs=""
for s in graph.hip consensus.hip cd.hip cd_rl.hip leiden.hip capi.cpp gen.cpp; do
    if [ "$s" = "$src" ]; then objs="$objs $L/$name/$src.o"; else objs="$objs $L/obj/$s.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/$name/libfastconsensus_amd.so $objs
echo "built $L/$name"
