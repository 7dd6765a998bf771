#!/bin/bash
# Replica-lane vs classic CD engine on every bench config (one line each), n_p=8 share included.
set -u
OUT=gpurun_out/rlab
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items()})"
}
for eng in 1 0; do
    st=""; [ $eng -eq 0 ] && st="--store 1"
    run lfr1m_e$eng --steps 5 --warmup 2 --opt cd_engine=$eng $st
    run np8_e$eng --n-p 8 --steps 5 --warmup 2 --opt cd_engine=$eng $st
    run lfr100k_e$eng --config lfr100k --steps 5 --warmup 2 --opt cd_engine=$eng $st
    run lfr100k_lpm_e$eng --config lfr100k_lpm --steps 5 --warmup 2 --opt cd_engine=$eng $st
    run sbm4m_e$eng --config sbm4m --steps 3 --warmup 1 --opt cd_engine=$eng $st
done
