#!/bin/bash
# Infomap LFR-100k: the tree before the round-3 length-tier commit (348e632^), after the
# heavy-row commit (0b8afcc), and HEAD -- each its own bench.py + library, same box, alternated.
set -u
OUT=$PWD/gpurun_out/r04imab
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <dir> <args...>
    local tag=$1 dir=$2; shift 2
    (cd $dir && timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err) || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],1), 'ms', d['config']['iterations'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
for rep in 1 2; do
    run pre_$rep tools/ablib/pre_tree --config lfr100k_infomap --steps 3 --warmup 1
    run post_$rep tools/ablib/post_tree --config lfr100k_infomap --steps 3 --warmup 1
    run head_$rep . --config lfr100k_infomap --steps 3 --warmup 1
done
