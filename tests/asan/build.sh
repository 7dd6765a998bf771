#!/bin/bash
# ASan/UBSan host build of the C-ABI (capi.cpp, gen.cpp instrumented on the host side only,
# -Xarch_host; device code untouched) linked with the regular graph/consensus/cd objects of
# fastconsensus_amd/build.py, plus tests/asan/asan_driver.c.  Output: tests/asan/_build/.
set -eu
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/tests/asan/_build
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -fPIC -std=c++17 --offload-arch=gfx950 -I$ROOT/include"
for s in capi.cpp gen.cpp; do
    $HIPCC $FLAGS $SAN -c "$ROOT/fastconsensus_amd/csrc/$s" -o "$OUT/$s.o"
done
OBJ=$ROOT/fastconsensus_amd/lib/obj
$HIPCC --offload-arch=gfx950 $SAN -g -o "$OUT/asan_driver" \
    -x c "$ROOT/tests/asan/asan_driver.c" -x none "$OUT/capi.cpp.o" "$OUT/gen.cpp.o" \
    "$OBJ/graph.hip.o" "$OBJ/consensus.hip.o" "$OBJ/cd.hip.o" "$OBJ/cd_rl.hip.o" "$OBJ/leiden.hip.o"
echo "built $OUT/asan_driver"
