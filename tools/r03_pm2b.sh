#!/bin/bash
# A/B: Leiden-style marks on every graph (prune_mark=2) vs the default, C4 and C3.
set -u
mkdir -p gpurun_out/pm
for cfg in lfr1m lfr100k; do
  for pm in 1 2; do
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --opt prune_mark=$pm > gpurun_out/pm/${cfg}_$pm.json 2> gpurun_out/pm/${cfg}_$pm.err || { tail gpurun_out/pm/${cfg}_$pm.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pm/${cfg}_$pm.json')); print('$cfg pm=$pm', round(d['ms_per_step'],2), d['config']['iterations'], d['phase_ms_per_step_rank0']['cd_ms'])"
  done
done
