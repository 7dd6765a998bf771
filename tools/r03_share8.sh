#!/bin/bash
# n_p=8 per-GPU share of the LFR-1M run (one GPU's work at N=8): bench line + kernel trace.
set -u
mkdir -p gpurun_out/share8
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --n-p 8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/share8/bench.json 2> gpurun_out/share8/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/share8/prof -o share8 --output-format csv -- python3 bench.py --n-p 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/share8/prof.log 2>&1 || exit 1
echo done
