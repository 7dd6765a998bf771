#!/bin/bash
# One Leiden LFR-1M fast_consensus call with FC_TRACE=1 (per-level / per-sweep lines on stderr).
set -u
mkdir -p gpurun_out/ltrace
FC_TRACE=1 timeout -k 10 300 python3 bench.py --config lfr1m_leiden --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ltrace/bench.json 2> gpurun_out/ltrace/trace.err || exit 1
echo done
