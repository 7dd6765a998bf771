#!/bin/bash
# Development loop on the GPU box: parity tests, then one traced LFR-1M bench step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 15 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
FC_TRACE=1 timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
rc=$?; tail -n 4 gpurun_out/iter_bench.err; [ $rc -eq 0 ] || exit $rc
python -c "
import json;d=json.load(open('gpurun_out/iter_bench.json'))
print(round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()}, 'frac', round(d['roofline']['frac'],4))"
