#!/bin/bash
# A/B of replica-lane decide variants: parity subset on the in-tree library, then
# tools/cd_ab.py on LFR-1M (louvain, lpm) for base and the variants named in $@
set -u
OUT=gpurun_out/r04cmp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "twin or full_run or heavy or weighted or dense or hybrid or handoff or prune" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m --reps 3 base "$@" base "$@" && \
timeout -k 10 300 python3 tools/cd_ab.py --config lfr1m --algo 1 --reps 3 base "$@" && \
timeout -k 10 500 python3 tools/cd_ab.py --config sbm4m --algo 1 --reps 2 base "$@" && \
FC_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err
