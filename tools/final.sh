#!/bin/bash
# Final verification of a round: the whole GPU suite + smoke, then the bench line of every config
# (the headline with its CPU baseline) into gpurun_out/<tag>final/<name>.json, and a kernel trace
# of the n_p = 8 share (gpurun_out/<tag>final/np8tr) and of the C4 step (c4tr).  Run tools/pmc_all.sh first and copy its
# summaries into profiles/, so that every line carries traffic from a same-source PMC profile.
# Usage: tools/final.sh <tag> [name...]   (names: suite, the bench lines below, np8trace)
set -u
TAG=$1; shift
NAMES=${*:-"suite lfr1m lfr100k lfr100k_lpm np8 np16 sbm4m leiden infomap np8trace c4trace"}
OUT=gpurun_out/${TAG}final
mkdir -p $OUT
export TMPDIR=/tmp
suite() {
    timeout -k 10 1000 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1
    rc=$?
    tail -3 $OUT/pytest.log
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log
}
run() {  # run <name> <timeout> <args...>
    local tag=$1 lim=$2; shift 2
    timeout -k 10 $lim python -u bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "bench $tag failed"; tail -5 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$tag.json')); r=d.get('roofline') or {}; print('$tag', round(d['ms_per_step'],2), 'ms', '%.3e' % d['value'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), {k: round(v,1) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
}
for n in $NAMES; do
    case $n in
        suite) suite ;;
        lfr1m) run lfr1m 400 ;;
        lfr100k) run lfr100k 200 --config lfr100k --steps 5 --warmup 2 --no-cpu-baseline ;;
        lfr100k_lpm) run lfr100k_lpm 200 --config lfr100k_lpm --steps 5 --warmup 2 --no-cpu-baseline ;;
        np8) run np8 200 --n-p 8 --steps 5 --warmup 2 --no-cpu-baseline ;;
        np16) run np16 200 --n-p 16 --steps 5 --warmup 2 --no-cpu-baseline ;;
        sbm4m) run sbm4m 300 --config sbm4m --steps 3 --warmup 1 --no-cpu-baseline ;;
        leiden) run leiden 300 --config lfr1m_leiden --steps 3 --warmup 1 --no-cpu-baseline ;;
        infomap) run infomap 300 --config lfr100k_infomap --steps 3 --warmup 1 --no-cpu-baseline ;;
        np8trace)
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/np8tr -o np8 --output-format csv -- python3 bench.py --n-p 8 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/np8tr.log 2>&1 || { echo np8 trace failed; tail -5 $OUT/np8tr.log; exit 1; }
            python3 tools/trace_gaps.py $(find $OUT/np8tr -name "*kernel_trace.csv" | head -1) > $OUT/np8_trace_gaps.txt && head -8 $OUT/np8_trace_gaps.txt
            find $OUT/np8tr -name "*kernel_trace.csv" -size +8M -delete
            echo "np8 trace ok" ;;
        c4trace)   # the same kernel trace at n_p = 64 (the headline C4 step)
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4tr -o c4 --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c4tr.log 2>&1 || { echo c4 trace failed; tail -5 $OUT/c4tr.log; exit 1; }
            python3 tools/trace_gaps.py $(find $OUT/c4tr -name "*kernel_trace.csv" | head -1) > $OUT/c4_trace_gaps.txt && head -8 $OUT/c4_trace_gaps.txt
            find $OUT/c4tr -name "*kernel_trace.csv" -size +8M -delete
            echo "c4 trace ok" ;;
        *) echo "unknown $n"; exit 1 ;;
    esac
done
