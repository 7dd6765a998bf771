#!/bin/bash
# parity tests, then sweep-0 decide time (kernel trace) and the bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/iter_pytest.out 2>&1
rc=$?; tail -n 3 gpurun_out/iter_pytest.out; [ $rc -eq 0 ] || exit $rc
DBGS="${DBGS:-0}" bash tools/exp_ablate.sh || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || exit $?
python -c "
import json;d=json.load(open('gpurun_out/iter_bench.json'))
print(round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()}, 'frac', round(d['roofline']['frac'],4))"
