#!/bin/bash
# A/B of the decide block size (variant libraries from tools/build_variant.sh).
set -u
mkdir -p gpurun_out/dtb
for v in ${VARIANTS:-base dtb512 dtb1024 base}; do
  if [ $v = base ]; then L=fastconsensus_amd/lib/libfastconsensus_amd.so; else L=fastconsensus_amd/lib/$v/libfastconsensus_amd.so; fi
  FC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dtb/$v.json 2> gpurun_out/dtb/$v.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/dtb/$v.json'))
print('$v', round(d['ms_per_step'],1),'ms', {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
