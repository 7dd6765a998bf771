#!/bin/bash
# Bench each variant library (LIBS="name1 name2"; "base" = the in-tree build), after the GPU tests.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/expl
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
fi
for rep in ${REPS:-1}; do
for l in ${LIBS:-base}; do
  if [ $l = base ]; then lp=fastconsensus_amd/lib/libfastconsensus_amd.so; else lp=fastconsensus_amd/lib/$l/libfastconsensus_amd.so; fi
  FC_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/expl/$l.json 2> gpurun_out/expl/$l.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/expl/$l.json'))
print('$l', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done; done
