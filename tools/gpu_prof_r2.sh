#!/bin/bash
# Round-2 profiling on the GPU box.  Steps (each under its own timeout, stop at the first failure):
#   micro   : tools/micro/gather (FETCH_SIZE calibration for 4-B random gathers) + its PMC passes
#   list    : rocprofv3 -L (counter names on this box)
#   stats   : rocprofv3 --kernel-trace --stats over bench.py (lfr1m, 3 steps)
#   pmc:<tag>:<config>:<algo> : tools/pmc_cd.sh passes over one CD batch
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "== $name rc=$rc"; case $rc in 0) ;; *) echo "!! stopping at $name"; exit $rc;; esac; }
for s in "$@"; do
    case $s in
        micro)
            O=gpurun_out/micro; mkdir -p $O
            timeout -k 10 120 tools/micro/gather > $O/gather.txt 2>&1; chk $? gather; cat $O/gather.txt
            timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- tools/micro/gather > $O/fetch.log 2>&1; chk $? micro_fetch
            timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o l2 --output-format csv -- tools/micro/gather > $O/l2.log 2>&1; chk $? micro_l2
            timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o rdreq --output-format csv -- tools/micro/gather > $O/rdreq.log 2>&1; echo "== rdreq rc=$? (optional)"
            ;;
        list) timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_L.txt 2>&1; echo "== list rc=$?" ;;
        stats)
            timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_lfr1m -o stats --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/stats_lfr1m.log 2>&1; chk $? stats
            tail -n 3 gpurun_out/stats_lfr1m.log ;;
        pmc:*)
            IFS=: read -r _ tag cfg algo <<< "$s"
            bash tools/pmc_cd.sh $tag fastconsensus_amd/lib/libfastconsensus_amd.so $cfg $algo; chk $? pmc_$tag ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
