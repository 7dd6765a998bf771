#!/bin/bash
# After the exact-kernel change: CD parity subset, then hybrid vs classic bench lines.
set -u
OUT=gpurun_out/r04exact
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "twin or full_run or heavy or weighted" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # run <tag> <args...>
    local tag=$1; shift
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
run lfr100k_e2 --config lfr100k --steps 5 --warmup 2 --opt cd_engine=2
run lfr100k_lpm_e2 --config lfr100k_lpm --steps 5 --warmup 2 --opt cd_engine=2
run lfr1m_e2 --steps 5 --warmup 2 --opt cd_engine=2
run np16_e2 --n-p 16 --steps 5 --warmup 2 --opt cd_engine=2
run sbm4m_e2 --config sbm4m --steps 3 --warmup 1 --opt cd_engine=2
