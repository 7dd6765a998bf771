#!/bin/bash
# Round-3 bench lines at HEAD for every config (the default line carries its CPU baseline).
set -u
OUT=gpurun_out/lines
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <timeout> <args...>
    local tag=$1 to=$2; shift 2
    timeout -k 10 $to python3 -u bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], d['roofline'] and round(d['roofline']['frac'],4))"
}
run lfr100k 300 --config lfr100k --steps 5 --warmup 2 --no-cpu-baseline
run lfr100k_lpm 300 --config lfr100k_lpm --steps 5 --warmup 2 --no-cpu-baseline
run sbm4m 400 --config sbm4m --steps 3 --warmup 1 --no-cpu-baseline
run np8 300 --n-p 8 --steps 10 --warmup 3 --no-cpu-baseline
run leiden 400 --config lfr1m_leiden --steps 2 --warmup 1 --no-cpu-baseline
run infomap 400 --config lfr100k_infomap --steps 2 --warmup 1 --no-cpu-baseline
