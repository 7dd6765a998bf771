#!/bin/bash
# Round-3 final B (frozen sources): PMC of the other bench configs (LPA C3/C5, Leiden and Infomap
# kernels) summarised into profiles/, then their bench lines (same-hash traffic attached).
set -u
mkdir -p gpurun_out/fb gpurun_out/fb_prof gpurun_out/fbl
export TMPDIR=/tmp
pass() {  # pass <tag> <config> <algo>
    timeout -k 10 900 tools/pmc_cd.sh $1 fastconsensus_amd/lib/libfastconsensus_amd.so $2 $3 > gpurun_out/fb/$1.log 2>&1 || { echo "pmc $1 failed"; exit 1; }
    python3 tools/pmc_summary.py gpurun_out/pmc_$1 $2 profiles r03 > gpurun_out/fb/$1.summary 2>&1 || { echo "summary $1 failed"; exit 1; }
    cp profiles/pmc_$2.json profiles/r03_$2_kernel_stats.csv gpurun_out/fb_prof/
    rm -rf gpurun_out/pmc_$1
}
line() {  # line <tag> <args...>
    local tag=$1; shift
    timeout -k 10 400 python3 -u bench.py "$@" --no-cpu-baseline > gpurun_out/fbl/$tag.json 2> gpurun_out/fbl/$tag.err || { echo "bench $tag failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/fbl/$tag.json')); r=d['roofline']; print('$tag', round(d['ms_per_step'],2), r['kernel'], round(r['frac'],4), r['traffic'])"
}
pass r03f_lfr100k_lpm lfr100k_lpm 1
pass r03f_sbm4m sbm4m 1
export FC_AB_CDONLY=1 FC_PMC_KRE="k_lv_decide|k_lv_heavy"
pass r03f_lfr1m_leiden lfr1m_leiden 3
pass r03f_lfr100k_infomap lfr100k_infomap 4
unset FC_AB_CDONLY FC_PMC_KRE
line lfr100k_lpm --config lfr100k_lpm --steps 5 --warmup 2
line sbm4m --config sbm4m --steps 3 --warmup 1
line leiden --config lfr1m_leiden --steps 2 --warmup 1
line infomap --config lfr100k_infomap --steps 2 --warmup 1
echo done
