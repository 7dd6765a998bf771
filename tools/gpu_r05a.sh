#!/bin/bash
# Round 5, first GPU call: GPU suite at the round-start sources (+ ADVICE fixes), the headline
# bench line, a kernel trace of the n_p = 8 share, and per-launch PMC of SBM-4M's filtered sweeps.
set -u
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/lfr1m.json 2> $OUT/lfr1m.err || { echo bench failed; tail -5 $OUT/lfr1m.err; exit 1; }
head -c 600 $OUT/lfr1m.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/np8 -o np8 --output-format csv -- python3 bench.py --n-p 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/np8.log 2>&1 || { echo np8 trace failed; tail -5 $OUT/np8.log; exit 1; }
tail -1 $OUT/np8.log | cut -c1-400
FC_PMC_KRE="k_decide_light|k_rl_decide|k_apply|k_list" ./tools/pmc_bench.sh sbm4m r05 > $OUT/pmc_sbm.log 2>&1 || { echo pmc failed; tail -5 $OUT/pmc_sbm.log; exit 1; }
python3 tools/pmc_per_launch.py gpurun_out/pmcb_sbm4m "k_decide_light<false" > $OUT/sbm_per_launch.txt 2>&1; tail -30 $OUT/sbm_per_launch.txt
