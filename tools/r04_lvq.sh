#!/bin/bash
# Leiden adaptive buckets: Leiden GPU tests, then lv_ab default vs FC_LV_QUEUE_DIV=0 (always B) and a level trace
set -u
OUT=gpurun_out/r04lvq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_leiden.py -m gpu -s > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "leiden LFR" $OUT/pytest.log | head; \
timeout -k 10 700 python3 tools/lv_ab.py --config lfr1m_leiden --reps 2 base base@FC_LV_LEVEL_B=16 base@FC_LV_LEVEL_B=8 base@FC_LV_LEVEL_B=4 base@FC_LV_LEVEL_B=8,FC_LV_QUEUE_DIV=0 && \
FC_TRACE=1 FC_LV_LEVEL_B=8 timeout -k 10 300 python3 bench.py --config lfr1m_leiden --steps 1 --warmup 0 --no-cpu-baseline > $OUT/ltrace.json 2> $OUT/ltrace.err &&
for env in "" "FC_LV_LEVEL_B=8" "FC_LV_LEVEL_B=4"; do env $env timeout -k 10 300 python3 tools/lvq_quality.py || exit 1; done
