#!/bin/bash
# Replica-lane engine: parity subset, bench line (trace), kernel stats; classic engine line beside it.
set -u
OUT=gpurun_out/rl2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "replica_lanes or test_cd_bit_exact_vs_twin or heavy_rows or prune_mark or full_run or visit_mode" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('RL', round(d['ms_per_step'],2), {k: round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()}, round(d['roofline']['avg_us'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lfr1m --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
t=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); cp "$t" $OUT/kernel_trace.csv
rm -rf $OUT/prof
head -12 $OUT/kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt cd_engine=0 --store 1 > $OUT/classic.json 2> $OUT/classic.err || { echo "classic failed"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/classic.json')); print('classic', round(d['ms_per_step'],2), {k: round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})"
