#!/bin/bash
# A/B: output array page-locked at allocation (default) vs pageable, C4 and C3.
set -u
mkdir -p gpurun_out/pin
for cfg in lfr1m lfr100k; do
  for mode in pin nopin; do
    extra=""; [ $mode = nopin ] && extra="--no-pin-out"
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline $extra > gpurun_out/pin/${cfg}_$mode.json 2> gpurun_out/pin/${cfg}_$mode.err || { tail gpurun_out/pin/${cfg}_$mode.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pin/${cfg}_$mode.json')); print('$cfg $mode', round(d['ms_per_step'],2), round(d['loop_ms_per_step'],2), round(d['load_ms_per_step'],2), d['output_array'])"
  done
done
