#!/bin/bash
# Storage-order pass sweeps (FC_ORDER_SWEEPS) A/B on the default LFR-1M line.
set -u
OUT=gpurun_out/ord
mkdir -p $OUT
export TMPDIR=/tmp
for s in 4 2 3 1; do
  FC_ORDER_SWEEPS=$s timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/s$s.json 2> $OUT/s$s.err || { echo "bench $s failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s$s.json')); print('order sweeps $s', round(d['ms_per_step'],2), 'ms load', round(d['load_ms_per_step'],2), 'cd', round(d['phase_ms_per_step_rank0']['cd_ms'],1))"
done
