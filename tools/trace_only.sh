#!/bin/bash
# rocprofv3 kernel trace + stats of one bench step (no PMC)
set -u
CFG=${1:-lfr1m}
OUT=gpurun_out/tr_$CFG${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- \
    python3 bench.py --config $CFG --steps 1 --warmup ${WARMUP:-0} --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/log 2>&1
rc=$?; tail -n 3 $OUT/log; exit $rc
