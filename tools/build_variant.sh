#!/bin/bash
# Build a variant library (cd.hip with extra -D flags) into fastconsensus_amd/lib/<name>/ (CPU host).
#   tools/build_variant.sh <name> -DFLAG ...
set -eu
name=$1; shift
L=fastconsensus_amd/lib
mkdir -p $L/$name
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude "$@" -x hip -c fastconsensus_amd/csrc/cd.hip -o $L/$name/cd.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/$name/libfastconsensus_amd.so \
    $L/obj/graph.hip.o $L/obj/consensus.hip.o $L/$name/cd.o $L/obj/leiden.hip.o $L/obj/capi.cpp.o $L/obj/gen.cpp.o
echo "built $L/$name"
