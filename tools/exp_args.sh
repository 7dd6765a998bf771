#!/bin/bash
# parity tests, then bench under several argument sets: ARGS="--a 1;--b 2" (';'-separated runs)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/expargs
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra RUNS <<< "${ARGS:- }"
for a in "${RUNS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline $a > gpurun_out/expargs/$i.json 2> gpurun_out/expargs/$i.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/expargs/$i.json'))
print('[$a]', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
