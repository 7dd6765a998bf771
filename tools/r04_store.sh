#!/bin/bash
# Label storage order (FC_OPT_STORE) with the hybrid engine: is the ordering pass at load still worth it?
set -u
OUT=gpurun_out/r04store
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms load', round(d['load_ms_per_step'],2), {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
for rep in 1 2; do
run lfr1m_s1_$rep --steps 5 --warmup 2 --store 1
run lfr1m_s0_$rep --steps 5 --warmup 2 --store 0
done
run sbm_s1 --config sbm4m --steps 3 --warmup 1 --store 1
run sbm_s0 --config sbm4m --steps 3 --warmup 1 --store 0
