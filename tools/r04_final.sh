#!/bin/bash
# Round-4 final verification: whole GPU suite + smoke, then the bench line of every config
# (the headline with its CPU baseline) into gpurun_out/r04final/<config>.json.
set -u
OUT=gpurun_out/r04final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run() {  # run <tag> <timeout> <args...>
    local tag=$1 lim=$2; shift 2
    timeout -k 10 $lim python -u bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); r=d.get('roofline') or {}; print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
run lfr1m 400
run lfr100k 200 --config lfr100k --steps 5 --warmup 2 --no-cpu-baseline
run lfr100k_lpm 200 --config lfr100k_lpm --steps 5 --warmup 2 --no-cpu-baseline
run np8 200 --n-p 8 --steps 5 --warmup 2 --no-cpu-baseline
run np16 200 --n-p 16 --steps 5 --warmup 2 --no-cpu-baseline
run sbm4m 300 --config sbm4m --steps 3 --warmup 1 --no-cpu-baseline
run leiden 300 --config lfr1m_leiden --steps 3 --warmup 1 --no-cpu-baseline
run infomap 300 --config lfr100k_infomap --steps 3 --warmup 1 --no-cpu-baseline
