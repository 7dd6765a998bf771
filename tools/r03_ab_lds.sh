#!/bin/bash
# A/B of decide-kernel LDS variants (tools/build_variant.sh builds) on LFR-1M: timing and label
# hashes (tools/cd_ab.py), then one PMC pass per variant for the LDS counters of k_decide_light.
#   tools/r03_ab_lds.sh <outdir> <variant>...
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m "$@" > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
for v in "$@"; do
    LIB=fastconsensus_amd/lib/$v/libfastconsensus_amd.so
    [ "$v" = base ] && LIB=fastconsensus_amd/lib/libfastconsensus_amd.so
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES \
        --kernel-include-regex "k_decide_light" -d $OUT/$v -o $v --output-format csv \
        -- python3 tools/cd_ab.py --child $LIB lfr1m 0 1 > $OUT/$v.pmc.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
