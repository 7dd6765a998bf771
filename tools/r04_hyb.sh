#!/bin/bash
# Hybrid CD engine (FC_OPT_CD_ENGINE=2): bit-exact twin tests, then LFR-1M bench lines (hybrid vs classic).
set -u
OUT=gpurun_out/r04hyb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "twin or full_run or heavy or storage" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items()})"
}
run lfr1m_e2 --steps 5 --warmup 2 --opt cd_engine=2
run lfr1m_e0 --steps 5 --warmup 2 --opt cd_engine=0
FC_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --opt cd_engine=2 > $OUT/trace_e2.json 2> $OUT/trace_e2.err
