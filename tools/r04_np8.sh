#!/bin/bash
# n_p = 8 share: storage-order pass and closure rounds
set -u
OUT=gpurun_out/r04np8
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py --n-p 8 --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'load', round(d['load_ms_per_step'],2), {k: round(v,2) for k, v in d['phase_ms_per_step_rank0'].items() if v}, d['config']['m_final'])"
}
run base
run store1 --opt store=1
run clo4 --opt closure_rounds=4
run base2
