#!/bin/bash
# Round-3 final A (frozen sources): GPU suite, smoke, PMC passes of the default config summarised
# into profiles/ (so the bench line attaches same-hash traffic), the default bench line with its
# CPU baseline, and the rocprofv3 kernel stats of that bench.  Stops at the first failure.
set -u
OUT=gpurun_out/fin
mkdir -p $OUT/prof
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
tools/pmc_cd.sh r03f_lfr1m fastconsensus_amd/lib/libfastconsensus_amd.so lfr1m 0 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_r03f_lfr1m lfr1m profiles r03 > $OUT/pmc_summary.log 2>&1 || { echo "summary failed"; tail $OUT/pmc_summary.log; exit 1; }
cp profiles/pmc_lfr1m.json profiles/r03_lfr1m_kernel_stats.csv $OUT/prof/
rm -rf gpurun_out/pmc_r03f_lfr1m
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(round(d['ms_per_step'],2), d['roofline']['frac'], d['roofline']['traffic'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rp -o lfr1m --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/rp.log 2>&1 || { echo "rocprof failed"; exit 1; }
cp $(find $OUT/rp -name "*kernel_stats.csv" | head -1) $OUT/prof/r03_bench_lfr1m_kernel_stats.csv
rm -rf $OUT/rp
echo done
