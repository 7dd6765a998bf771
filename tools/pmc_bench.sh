#!/bin/bash
# rocprofv3 over bench.py itself (the command the bench line comes from): one --kernel-trace
# --stats pass, then one PMC group per run (--kernel-trace beside --pmc only), the decide / apply
# kernels of both CD engines.  Summaries -> profiles/pmc_<config>.json + <tag>_<config>_kernel_stats.csv.
# Usage: tools/pmc_bench.sh <config> <tag> [bench args...]
#   FC_PMC_NP=<n>: bench --n-p <n>, summary profiles/pmc_<config>_np<n>.json (bench.py reads that
#   one for a line run with --n-p <n>)
set -u
CFG=$1; TAG=$2; shift 2
NAME=$CFG
NPARG=""
if [ -n "${FC_PMC_NP:-}" ]; then NAME=${CFG}_np$FC_PMC_NP; NPARG="--n-p $FC_PMC_NP"; fi
OUT=gpurun_out/pmcb_$NAME
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
PROG="python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline $NPARG $*"
KRE=${FC_PMC_KRE:-"k_decide_light|k_rl_decide|k_apply|k_rl_apply|k_cd_tail|k_lv_decide|k_lv_heavy"}
run() {  # run <name> <rocprof args...>
    local name=$1; shift
    echo "== $name"
    timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $PROG > $OUT/$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-300
    case $rc in 0) ;; *) echo "!! stopping"; exit $rc;; esac
}
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$KRE"
run write --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$KRE"
run l2 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE"
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "$KRE"
python3 tools/pmc_summary.py $OUT $NAME $OUT/profiles $TAG > $OUT/summary.json && head -c 1500 $OUT/summary.json
