#!/bin/bash
# Round-3 verification B: PMC for the LPA configs and the Leiden / Infomap kernels.
set -u
mkdir -p gpurun_out/fb
export TMPDIR=/tmp
timeout -k 10 600 tools/pmc_cd.sh r03_lfr100k_lpm fastconsensus_amd/lib/libfastconsensus_amd.so lfr100k_lpm 1 > gpurun_out/fb/pmc_lpm.log 2>&1 || { echo "pmc lpm failed"; exit 1; }
timeout -k 10 900 tools/pmc_cd.sh r03_sbm4m fastconsensus_amd/lib/libfastconsensus_amd.so sbm4m 1 > gpurun_out/fb/pmc_sbm.log 2>&1 || { echo "pmc sbm failed"; exit 1; }
FC_AB_CDONLY=1 FC_PMC_KRE="k_lv_decide|k_lv_heavy" timeout -k 10 900 tools/pmc_cd.sh r03_lfr1m_leiden fastconsensus_amd/lib/libfastconsensus_amd.so lfr1m_leiden 3 > gpurun_out/fb/pmc_leiden.log 2>&1 || { echo "pmc leiden failed"; exit 1; }
FC_AB_CDONLY=1 FC_PMC_KRE="k_lv_decide|k_lv_heavy" timeout -k 10 900 tools/pmc_cd.sh r03_lfr100k_infomap fastconsensus_amd/lib/libfastconsensus_amd.so lfr100k_infomap 4 > gpurun_out/fb/pmc_infomap.log 2>&1 || { echo "pmc infomap failed"; exit 1; }
echo done
