#!/bin/bash
# Round 5, call 3: GPU suite without the scalar-row decide; SBM-4M per-sweep trace (LPA tie
# revisits) and per-launch PMC of its filtered decide; headline bench line.
set -u
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -rA --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Mismatch" $OUT/pytest.log | head -20; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/lfr1m.json 2> $OUT/lfr1m.err || { echo bench failed; tail -5 $OUT/lfr1m.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/lfr1m.json')); print('lfr1m', round(d['ms_per_step'],2), d['phase_ms_per_step_rank0'])"
FC_TRACE=1 timeout -k 10 300 python -u bench.py --config sbm4m --steps 1 --warmup 1 --no-cpu-baseline > $OUT/sbm_trace.json 2> $OUT/sbm_trace.err || { echo sbm trace failed; tail -5 $OUT/sbm_trace.err; exit 1; }
grep -c "sweep=" $OUT/sbm_trace.err
FC_PMC_KRE="k_decide_light|k_rl_decide|k_apply|k_list" ./tools/pmc_bench.sh sbm4m r05 > $OUT/pmc_sbm.log 2>&1 || { echo pmc failed; tail -5 $OUT/pmc_sbm.log; exit 1; }
python3 tools/pmc_per_launch.py gpurun_out/pmcb_sbm4m "k_decide_light<false" > $OUT/sbm_per_launch.txt 2>&1; tail -40 $OUT/sbm_per_launch.txt
exit $rc
