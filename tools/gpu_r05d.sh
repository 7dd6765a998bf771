#!/bin/bash
# Round 5, call 4: where the replica-lane LPA departs from the twin (n_r >= 33); GPU parity
# suite after the per-sweep bookkeeping change; SBM-4M tail-kernel threshold A/B (LPA's tie
# revisits leave ~30 sweeps of ~27k visits per replica); n_p = 8 share and the headline.
set -u
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug_rl_lpa.py 64 0 > $OUT/debug64.log 2>&1; tail -4 $OUT/debug64.log
timeout -k 10 600 python -u -m pytest -q -rA --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED" $OUT/pytest.log | head -20; }
run() {  # run <tag> <timeout> <args...>
    local tag=$1 lim=$2; shift 2
    timeout -k 10 $lim python -u bench.py --no-cpu-baseline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); r=d.get('roofline') or {}; print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], 'frac', r.get('frac'), {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
run np8 200 --n-p 8 --steps 5 --warmup 2
run lfr1m 300
for t in 4096 16384 32768 65536 262144; do
    run sbm_t$t 300 --config sbm4m --steps 2 --warmup 1 --opt tail_visits=$t
done
exit $rc
