#!/bin/bash
# Round-3 final C (frozen sources, after the closure / shared-output changes): GPU suite, smoke,
# PMC of every bench config summarised into profiles/ (same csrc hash as the timed library),
# the default bench line with its CPU baseline, the other bench lines, kernel stats.
# Stops at the first failure.
set -u
OUT=gpurun_out/fc
mkdir -p $OUT/prof $OUT/lines
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
pass() {  # pass <tag> <config> <algo>
    timeout -k 10 900 tools/pmc_cd.sh $1 fastconsensus_amd/lib/libfastconsensus_amd.so $2 $3 > $OUT/$1.log 2>&1 || { echo "pmc $1 failed"; tail -20 $OUT/$1.log; exit 1; }
    python3 tools/pmc_summary.py gpurun_out/pmc_$1 $2 profiles r03 > $OUT/$1.summary 2>&1 || { echo "summary $1 failed"; tail $OUT/$1.summary; exit 1; }
    cp profiles/pmc_$2.json profiles/r03_$2_kernel_stats.csv $OUT/prof/
    rm -rf gpurun_out/pmc_$1
}
line() {  # line <tag> <args...>
    local tag=$1; shift
    timeout -k 10 400 python3 -u bench.py "$@" > $OUT/lines/$tag.json 2> $OUT/lines/$tag.err || { echo "bench $tag failed"; tail $OUT/lines/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/lines/$tag.json')); r=d['roofline']; print('$tag', round(d['ms_per_step'],2), r['kernel'], round(r['frac'],4), r['traffic'])"
}
pass r03c_lfr1m lfr1m 0
line lfr1m --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rp -o lfr1m --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/rp.log 2>&1 || { echo "rocprof failed"; exit 1; }
cp $(find $OUT/rp -name "*kernel_stats.csv" | head -1) $OUT/prof/r03_bench_lfr1m_kernel_stats.csv
rm -rf $OUT/rp
pass r03c_lfr100k_lpm lfr100k_lpm 1
pass r03c_sbm4m sbm4m 1
export FC_AB_CDONLY=1 FC_PMC_KRE="k_lv_decide|k_lv_heavy"
pass r03c_lfr1m_leiden lfr1m_leiden 3
pass r03c_lfr100k_infomap lfr100k_infomap 4
unset FC_AB_CDONLY FC_PMC_KRE
line lfr100k --config lfr100k --steps 10 --warmup 2 --no-cpu-baseline
line lfr100k_lpm --config lfr100k_lpm --steps 5 --warmup 2 --no-cpu-baseline
line sbm4m --config sbm4m --steps 3 --warmup 1 --no-cpu-baseline
line leiden --config lfr1m_leiden --steps 2 --warmup 1 --no-cpu-baseline
line infomap --config lfr100k_infomap --steps 2 --warmup 1 --no-cpu-baseline
line np8 --config lfr1m --n-p 8 --steps 10 --warmup 2 --no-cpu-baseline
echo done
