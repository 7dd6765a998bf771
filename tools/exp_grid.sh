#!/bin/bash
# parity tests, then decide-grid variants (FC_DECIDE_BLOCKS: 0 = one item per block)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
for db in ${DBS:-0 2048}; do
  FC_DECIDE_BLOCKS=$db timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g_$db.json 2> gpurun_out/g_$db.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/g_$db.json'))
print('$db', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
