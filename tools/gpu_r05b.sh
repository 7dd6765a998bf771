#!/bin/bash
# Round 5, call 2: GPU suite (LPA tie revisits, scalar-row decide), bench A/B of the scalar rows
# (FC_RL_UNIFORM 0/1) on LFR-1M and SBM-4M, C3 lpm, and a kernel trace of the n_p = 8 share.
set -u
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; }
grep -E "consensus NMI|device mean" $OUT/pytest.log | head -20
run() {  # run <tag> <timeout> <args...>
    local tag=$1 lim=$2; shift 2
    timeout -k 10 $lim python -u bench.py --no-cpu-baseline "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); r=d.get('roofline') or {}; print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], 'frac', r.get('frac'), {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
FC_RL_UNIFORM=1 run lfr1m_u1 300
FC_RL_UNIFORM=0 run lfr1m_u0 300
FC_RL_UNIFORM=1 run lfr1m_u1b 300
FC_RL_UNIFORM=1 run sbm4m 300 --config sbm4m --steps 3 --warmup 1
run lfr100k_lpm 200 --config lfr100k_lpm --steps 5 --warmup 2
run np8 200 --n-p 8 --steps 5 --warmup 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/np8tr -o np8 --output-format csv -- python3 bench.py --n-p 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/np8tr.log 2>&1 || { echo np8 trace failed; tail -5 $OUT/np8tr.log; exit 1; }
echo trace ok
exit $rc
