#!/bin/bash
# Per-variant decide timing + L2 hit/miss PMC pass (k_decide_light) on LFR-1M.
#   tools/r03_ab_l2.sh <outdir> <variant>...
set -u
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m "$@" > $OUT/ab.log 2>&1 || { echo "ab failed"; exit 1; }
for v in "$@"; do
    LIB=fastconsensus_amd/lib/$v/libfastconsensus_amd.so
    [ "$v" = base ] && LIB=fastconsensus_amd/lib/libfastconsensus_amd.so
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum \
        --kernel-include-regex "k_decide_light" -d $OUT/$v -o $v --output-format csv \
        -- python3 tools/cd_ab.py --child $LIB lfr1m 0 1 > $OUT/$v.pmc.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
