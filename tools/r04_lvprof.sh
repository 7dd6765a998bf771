#!/bin/bash
# Leiden LFR-1M / Infomap LFR-100k: kernel stats (rocprofv3 --kernel-trace --stats) and a level trace
set -u
OUT=gpurun_out/r04lvp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/leiden -o leiden --output-format csv -- python3 bench.py --config lfr1m_leiden --steps 1 --warmup 1 --no-cpu-baseline > $OUT/leiden.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/infomap -o infomap --output-format csv -- python3 bench.py --config lfr100k_infomap --steps 1 --warmup 1 --no-cpu-baseline > $OUT/infomap.log 2>&1 && \
FC_TRACE=1 timeout -k 10 300 python3 bench.py --config lfr1m_leiden --steps 1 --warmup 0 --no-cpu-baseline > $OUT/ltrace.json 2> $OUT/ltrace.err
