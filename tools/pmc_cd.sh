#!/bin/bash
# PMC passes (one counter group per run, --kernel-trace beside --pmc only) over ONE CD batch of
# tools/cd_ab.py's child (no subprocess hop under the profiler).  Usage: tools/pmc_cd.sh <tag> [lib] [config] [algo]
set -u
TAG=$1; LIB=${2:-fastconsensus_amd/lib/libfastconsensus_amd.so}; CFG=${3:-lfr1m}; ALGO=${4:-0}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROG="python3 tools/cd_ab.py --child $LIB $CFG $ALGO 1"
KRE=${FC_PMC_KRE:-"k_decide_light|k_apply|k_cd_tail"}
run() {  # run <name> <rocprof args...>
    local name=$1; shift
    echo "== $name"
    timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $PROG > $OUT/$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 $OUT/$name.log
    case $rc in 0) ;; *) echo "!! stopping"; exit $rc;; esac
}
run trace --kernel-trace --stats
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "$KRE"
run sq2 --kernel-trace --pmc SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --kernel-include-regex "$KRE"
run l2 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE"
run fetch --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$KRE"
run write --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$KRE"
