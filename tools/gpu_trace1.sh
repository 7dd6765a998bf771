#!/bin/bash
set -u
mkdir -p gpurun_out
for v in "" "FC_PUSH_DIV=2" "FC_PUSH_DIV=1"; do
  echo "== $v"
  env FC_TRACE=1 $v timeout -k 10 200 python tools/cd_ab.py --child fastconsensus_amd/lib/libfastconsensus_amd.so lfr1m 0 1 > gpurun_out/tr_$v.out 2> gpurun_out/tr_$v.err || exit 1
  grep "cd it=0 sweep\|tail" gpurun_out/tr_$v.err | head -30
  cat gpurun_out/tr_$v.out | cut -c1-200
done
