#!/bin/bash
set -u
OUT=gpurun_out/r04tsbm
mkdir -p $OUT
export TMPDIR=/tmp
FC_TRACE=1 timeout -k 10 300 python -u bench.py --config sbm4m --steps 1 --warmup 0 --no-cpu-baseline > $OUT/e2.json 2> $OUT/e2.err || { echo "trace failed"; tail -5 $OUT/e2.err; exit 1; }
grep -c "sweep=" $OUT/e2.err
