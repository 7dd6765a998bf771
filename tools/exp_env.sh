#!/bin/bash
# parity tests, then bench under several environment settings: ENVS="A=1,B=2 C=3" (space-separated runs)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/expenv
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
i=0
for e in ${ENVS:-FC_X=0}; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/expenv/$i.json 2> gpurun_out/expenv/$i.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/expenv/$i.json'))
print('$e', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
