#!/bin/bash
# parity tests, then bench for every (env setting x argument set): ENVS="A=1 A=2", ARGS="--x 1;--x 2"
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/expm
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra RUNS <<< "${ARGS:- }"
for e in ${ENVS:-FC_X=0}; do
for a in "${RUNS[@]}"; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline $a > gpurun_out/expm/$i.json 2> gpurun_out/expm/$i.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/expm/$i.json'))
print('$e [$a]', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done; done
