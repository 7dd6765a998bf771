#!/bin/bash
# Rehearsal of the N>1 bench path on one GPU: 2 ranks share cuda:0, collectives over gloo
# (RCCL needs one GPU per rank).  Exercises run_sharded end to end on the HIP engine.
set -u
mkdir -p gpurun_out/multi
for c in ${CFGS:-lfr100k lfr1m}; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
     --master-port 29517 bench.py --gpus 2 --config $c --steps 2 --warmup 1 --dist-backend gloo \
     > gpurun_out/multi/gloo2_$c.json 2> gpurun_out/multi/gloo2_$c.err || exit $?
  python -c "
import json;d=json.loads([l for l in open('gpurun_out/multi/gloo2_$c.json') if l.startswith('{')][-1])
print('$c', 'n_gpus', d['n_gpus'], round(d['ms_per_step'],1),'ms', d['config']['iterations'], d['config']['parallelism'])"
done
