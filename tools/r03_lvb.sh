#!/bin/bash
# Leiden LFR-1M: buckets at dense aggregate levels (FC_LV_DENSE_DIV) A/B, with the level trace.
set -u
OUT=gpurun_out/lvb
mkdir -p $OUT
export TMPDIR=/tmp
for dv in 0 4 1; do
  FC_TRACE=1 FC_LV_DENSE_DIV=$dv timeout -k 10 300 python3 -u bench.py --config lfr1m_leiden --steps 1 --warmup 1 --no-cpu-baseline > $OUT/d$dv.json 2> $OUT/d$dv.err || { echo "bench $dv failed"; tail -3 $OUT/d$dv.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/d$dv.json')); print('div $dv', round(d['ms_per_step'],1), 'ms')"
  grep "leiden level" $OUT/d$dv.err | grep -v " sweep " | tail -9 | cut -c1-150
done
for dv in 4 1; do
  FC_LV_DENSE_DIV=$dv timeout -k 10 400 python3 -u -m pytest tests/test_leiden.py -x -q -s --timeout 300 -k "quality or modularity or lfr" > $OUT/t$dv.log 2>&1; echo "tests div $dv rc=$?"; grep -iE "modularity|passed|failed|Q " $OUT/t$dv.log | tail -6
done
