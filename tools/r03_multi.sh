#!/bin/bash
# N>1 rehearsal on one GPU (2 ranks share cuda:0 over gloo): shared-memory label output vs the
# all-gather to rank 0; then the n_p=8 share under rocprofv3 --kernel-trace --stats.
set -u
mkdir -p gpurun_out/mu
export TMPDIR=/tmp
for mode in shared gather; do
  extra=""; [ $mode = gather ] && extra="--gather-out"
  timeout -k 10 600 python3 -u bench.py --gpus 2 --config lfr1m --steps 3 --warmup 1 --dist-backend gloo $extra \
     > gpurun_out/mu/gloo2_$mode.json 2> gpurun_out/mu/gloo2_$mode.err || { tail -20 gpurun_out/mu/gloo2_$mode.err; exit 1; }
  python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/mu/gloo2_$mode.json') if l.startswith('{')][-1])
print('$mode', round(d['ms_per_step'],1), d['config']['iterations'], d['config']['m_final'], d['dist'])"
done
ls /dev/shm | grep -c psm_ || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/mu/np8 -o np8 --output-format csv -- \
    python3 bench.py --config lfr1m --n-p 8 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/mu/np8.json 2> gpurun_out/mu/np8.err || { tail -20 gpurun_out/mu/np8.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/mu/np8.json'));print('np8', round(d['ms_per_step'],2), d['phase_ms_per_step_rank0'])"
find gpurun_out/mu/np8 -name "*kernel_stats.csv" -exec cp {} gpurun_out/mu/np8_kernel_stats.csv \;
find gpurun_out/mu/np8 -name "*kernel_trace.csv" -exec cp {} gpurun_out/mu/np8_kernel_trace.csv \;
rm -rf gpurun_out/mu/np8
echo done
