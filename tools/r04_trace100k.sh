#!/bin/bash
set -u
OUT=gpurun_out/r04t100k
mkdir -p $OUT
export TMPDIR=/tmp
for eng in 0 2; do
    FC_TRACE=1 timeout -k 10 300 python -u bench.py --config lfr100k --steps 1 --warmup 1 --no-cpu-baseline --opt cd_engine=$eng \
        > $OUT/e$eng.json 2> $OUT/e$eng.err || { echo "bench e$eng failed"; tail -5 $OUT/e$eng.err; exit 1; }
done
