#!/bin/bash
# Same-source PMC for every bench line's traffic (tools/pmc_bench.sh per config), the summaries
# copied into profiles/ on the box and into gpurun_out/pmc_profiles/ (merged back); the raw
# per-launch CSVs are deleted on the box (gpurun merges back at most 64 MiB).
# Usage: tools/pmc_all.sh <tag> [config...]   (default: every config of tools/final.sh)
set -u
TAG=$1; shift
CFGS=${*:-"lfr1m lfr100k lfr100k_lpm sbm4m lfr1m_leiden lfr100k_infomap np8 np16"}
for c in $CFGS; do
    case $c in
        np8|np16) FC_PMC_NP=${c#np} ./tools/pmc_bench.sh lfr1m $TAG > /dev/null || exit 1; d=gpurun_out/pmcb_lfr1m_$c ;;
        *) ./tools/pmc_bench.sh $c $TAG > /dev/null || exit 1; d=gpurun_out/pmcb_$c ;;
    esac
    mkdir -p gpurun_out/pmc_profiles
    cp $d/profiles/* profiles/ && cp $d/profiles/* gpurun_out/pmc_profiles/ && echo "pmc $c ok: $(ls $d/profiles | tr '\n' ' ')"
    find $d -name "*.csv" -size +1M -delete
done
