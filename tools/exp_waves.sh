#!/bin/bash
# decide grid size sweep (FC_DECIDE_WAVES), after the parity tests
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
for wv in ${WAVES:-8192 16384 4096 100000000}; do
  FC_DECIDE_WAVES=$wv timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/w_$wv.json 2> gpurun_out/w_$wv.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/w_$wv.json'))
print('$wv', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
