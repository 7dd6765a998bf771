#!/bin/bash
# GPU-box profiling of bench.py: kernel trace + stats, then separate PMC passes (one
# counter group per pass, --kernel-trace only beside --pmc) on the dominant kernel.
set -u
CFG=${1:-lfr1m}
OUT=gpurun_out/prof_$CFG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
BENCH="python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
run() {  # run <name> <timeout> <rocprof args...>
    local name=$1 t=$2; shift 2
    echo "== $name"
    timeout -k 10 "$t" rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $BENCH \
        > $OUT/$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log
    case $rc in 0) ;; *) echo "!! stopping"; exit $rc;; esac
}
run trace 600 --kernel-trace --stats
run fetch 600 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_decide_light|k_pair_partial|k_apply"
run write 600 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "k_decide_light|k_pair_partial|k_apply"
run l2 600 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_decide_light"
run sq 600 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_decide_light"
find $OUT -name "*.csv" | head -50
