#!/bin/bash
# Per-GPU share of the C4 run at N=8/4/2 GPUs: one GPU running n_p=8/16/32 replicas (phase breakdown).
set -u
mkdir -p gpurun_out/np
export TMPDIR=/tmp
for np in ${NPS:-8 16 32}; do
  FC_TRACE=${TRACE:-0} timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --n-p $np ${BENCH_ARGS:-} \
      > gpurun_out/np/np$np.json 2> gpurun_out/np/np$np.err || exit $?
  python -c "
import json;d=json.load(open('gpurun_out/np/np$np.json'))
print('n_p=$np', round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
done
