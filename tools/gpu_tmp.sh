#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout 600 --timeout-method thread -rf -q -s tests/test_infomap.py tests/test_leiden.py > gpurun_out/im.out 2>&1; rc=$?
grep -E "infomap |leiden LFR|passed|failed" gpurun_out/im.out; [ $rc -eq 0 ] || { tail -30 gpurun_out/im.out; exit $rc; }
timeout -k 10 600 python bench.py --config lfr1m_leiden --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_l1m.out 2> gpurun_out/b_l1m.err || { tail -20 gpurun_out/b_l1m.err; exit 1; }
tail -3 gpurun_out/b_l1m.err
timeout -k 10 600 python bench.py --config lfr100k_infomap --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_i100k.out 2> gpurun_out/b_i100k.err || { tail -20 gpurun_out/b_i100k.err; exit 1; }
tail -3 gpurun_out/b_i100k.err
