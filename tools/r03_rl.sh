#!/bin/bash
# Replica-lane CD engine: twin parity subset, then the LFR-1M bench line (and the classic engine beside it).
set -u
OUT=gpurun_out/rl
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "replica_lanes or test_cd_bit_exact_vs_twin or heavy_rows or prune_mark" > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
FC_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(round(d['ms_per_step'],2), d['phase_ms_per_step_rank0'], d['roofline'])"
grep "rl it=" $OUT/bench.err | head -80
