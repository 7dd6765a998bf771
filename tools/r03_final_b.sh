#!/bin/bash
# Round-3 verification B: PMC for the LPA configs and the Leiden / Infomap kernels, summarised on
# the box (tools/pmc_summary.py -> gpurun_out/fb_prof/) and the raw counter CSVs removed (they
# exceed what gpurun copies back).
set -u
mkdir -p gpurun_out/fb gpurun_out/fb_prof
export TMPDIR=/tmp
pass() {  # pass <tag> <config> <algo>
    timeout -k 10 900 tools/pmc_cd.sh $1 fastconsensus_amd/lib/libfastconsensus_amd.so $2 $3 > gpurun_out/fb/$1.log 2>&1 || { echo "pmc $1 failed"; exit 1; }
    python3 tools/pmc_summary.py gpurun_out/pmc_$1 $2 gpurun_out/fb_prof r03 > gpurun_out/fb/$1.summary 2>&1 || { echo "summary $1 failed"; exit 1; }
    rm -rf gpurun_out/pmc_$1
}
pass r03_lfr100k_lpm lfr100k_lpm 1
pass r03_sbm4m sbm4m 1
export FC_AB_CDONLY=1 FC_PMC_KRE="k_lv_decide|k_lv_heavy"
pass r03_lfr1m_leiden lfr1m_leiden 3
pass r03_lfr100k_infomap lfr100k_infomap 4
echo done
