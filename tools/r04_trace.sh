#!/bin/bash
# Per-sweep trace (FC_TRACE=1: host sync per sweep, dt per sweep) of one LFR-1M step, both CD engines.
set -u
OUT=gpurun_out/r04trace
mkdir -p $OUT
export TMPDIR=/tmp
for eng in 0 1; do
    FC_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --opt cd_engine=$eng \
        > $OUT/e$eng.json 2> $OUT/e$eng.err || { echo "bench e$eng failed"; tail -5 $OUT/e$eng.err; exit 1; }
    grep -c "sweep=" $OUT/e$eng.err
done
