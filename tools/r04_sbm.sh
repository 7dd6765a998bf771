#!/bin/bash
set -u
OUT=gpurun_out/r04sbm
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config sbm4m --steps 3 --warmup 1 --no-cpu-baseline > $OUT/sbm4m.json 2> $OUT/sbm4m.err || { echo "bench failed"; tail -5 $OUT/sbm4m.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/sbm4m.json')); print('sbm4m', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cd_parity.py -k "c5 or C5 or sbm" -m gpu > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
