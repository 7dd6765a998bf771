#!/bin/bash
# Default engine = hybrid: bench lines of every config (no --opt), n_p=8/16 shares.
set -u
OUT=gpurun_out/r04def
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
run lfr1m --steps 5 --warmup 2
run lfr100k --config lfr100k --steps 5 --warmup 2
run lfr100k_lpm --config lfr100k_lpm --steps 5 --warmup 2
run np8 --n-p 8 --steps 5 --warmup 2
run np16 --n-p 16 --steps 5 --warmup 2
run sbm4m --config sbm4m --steps 3 --warmup 1
