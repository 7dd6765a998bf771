#!/bin/bash
# A/B: buckets of the load-time storage-order pass (FC_ORDER_BUCKETS; it only permutes storage,
# results are identical), C4.
set -u
mkdir -p gpurun_out/ob
for b in 32 8 16 4; do
  FC_ORDER_BUCKETS=$b timeout -k 10 300 python3 -u bench.py --config lfr1m --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ob/b$b.json 2> gpurun_out/ob/b$b.err || { tail gpurun_out/ob/b$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ob/b$b.json')); print('buckets $b', round(d['ms_per_step'],2), 'load', round(d['load_ms_per_step'],2), 'cd', round(d['phase_ms_per_step_rank0']['cd_ms'],2), d['config']['m_final'])"
done
