#!/bin/bash
# Bench line + rocprofv3 kernel stats (+ trace) for one bench config.
#   tools/r03_prof_cfg.sh <config> <tag> [steps]
set -u
CFG=$1; TAG=$2; STEPS=${3:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o $TAG --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
echo done
