#!/bin/bash
set -u
OUT=gpurun_out/r04p100k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/e2 -o e2 --output-format csv -- python3 bench.py --config lfr100k --steps 2 --warmup 1 --no-cpu-baseline --opt cd_engine=2 > $OUT/e2.log 2>&1 || { echo fail; tail $OUT/e2.log; exit 1; }
find $OUT -name "*kernel_stats.csv" | head
