#!/bin/bash
# Hybrid (cd_engine=2) vs classic (0) on the other bench configs and the per-GPU shares.
set -u
OUT=gpurun_out/r04hab
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items()})"
}
for eng in 2 0; do
    run lfr100k_e$eng --config lfr100k --steps 5 --warmup 2 --opt cd_engine=$eng
    run lfr100k_lpm_e$eng --config lfr100k_lpm --steps 5 --warmup 2 --opt cd_engine=$eng
    run np8_e$eng --n-p 8 --steps 5 --warmup 2 --opt cd_engine=$eng
    run np16_e$eng --n-p 16 --steps 5 --warmup 2 --opt cd_engine=$eng
    run sbm4m_e$eng --config sbm4m --steps 3 --warmup 1 --opt cd_engine=$eng
done
run np8_e2rl --n-p 8 --steps 5 --warmup 2 --opt cd_engine=2 --opt rl_min_replicas=1
run np16_e2cl --n-p 16 --steps 5 --warmup 2 --opt cd_engine=2 --opt rl_min_replicas=1000
