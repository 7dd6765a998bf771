#!/bin/bash
# Leiden at 4 aggregate-level buckets (default): Leiden GPU tests, lv_ab vs 2 / 32, quality at 2, bench line
set -u
OUT=gpurun_out/r04lvq2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_leiden.py -m gpu -s > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "leiden LFR" $OUT/pytest.log | head
timeout -k 10 500 python3 tools/lv_ab.py --config lfr1m_leiden --reps 2 base base@FC_LV_LEVEL_B=2 base@FC_LV_LEVEL_B=32 && \
FC_LV_LEVEL_B=2 timeout -k 10 300 python3 tools/lvq_quality.py && \
timeout -k 10 300 python -u bench.py --config lfr1m_leiden --steps 3 --warmup 1 --no-cpu-baseline > $OUT/leiden.json 2> $OUT/leiden.err && \
python3 -c "import json; d=json.load(open('$OUT/leiden.json')); print('leiden', d['ms_per_step'], d['value'], d['roofline']['frac'])"
