#!/bin/bash
set -u
OUT=$PWD/gpurun_out/r04imab2
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <dir> <args...>
    local tag=$1 dir=$2; shift 2
    (cd $dir && timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err) || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],1), 'ms', d['config']['iterations'])"
}
run r02_1 tools/ablib/r02_tree --config lfr100k_infomap --steps 3 --warmup 1
run head_1 . --config lfr100k_infomap --steps 3 --warmup 1
run r02_2 tools/ablib/r02_tree --config lfr100k_infomap --steps 3 --warmup 1
timeout -k 10 300 python -u tools/timing_ab.py lfr100k_infomap 2
