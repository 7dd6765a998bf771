#!/bin/bash
set -u
OUT=gpurun_out/r04ab100k
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items()})"
}
run lfr100k_e2cl --config lfr100k --steps 5 --warmup 2 --opt cd_engine=2 --opt rl_min_replicas=1000
run lfr100k_lpm_e2cl --config lfr100k_lpm --steps 5 --warmup 2 --opt cd_engine=2 --opt rl_min_replicas=1000
run lfr100k_e2 --config lfr100k --steps 5 --warmup 2 --opt cd_engine=2
run lfr100k_e0 --config lfr100k --steps 5 --warmup 2 --opt cd_engine=0
