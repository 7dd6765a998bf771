#!/bin/bash
# A/B runs of bench.py: each argument is "name" (lib variant under fastconsensus_amd/lib/<name>/, or
# "base") optionally followed by ":ENV=VAL" settings, e.g. base:FC_APPLY_BLOCKS=64.
set -u
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*:}
  if [ $name = base ]; then L=fastconsensus_amd/lib/libfastconsensus_amd.so; else L=fastconsensus_amd/lib/$name/libfastconsensus_amd.so; fi
  tag=$(echo "$spec" | tr ':=,' '___')
  env $envs FC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/ab/$tag.json'))
print('$spec', round(d['ms_per_step'],1),'ms', {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
