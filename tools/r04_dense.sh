#!/bin/bash
# dense_div A/B (hybrid semantics switch) on LFR-1M, SBM-4M, n_p=16 share; parity of the switch first.
set -u
OUT=gpurun_out/r04dense
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "dense or twin" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
for dd in 0 2 4; do
    run lfr1m_d$dd --steps 5 --warmup 2 --opt dense_div=$dd
    run sbm4m_d$dd --config sbm4m --steps 3 --warmup 1 --opt dense_div=$dd
done
run np16_d0 --n-p 16 --steps 5 --warmup 2 --opt dense_div=0
run np16_d2 --n-p 16 --steps 5 --warmup 2 --opt dense_div=2
