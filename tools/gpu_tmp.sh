#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FC_INFOMAP_DEBUG=1 timeout -k 10 120 python tools/im_dbg.py 2>&1 | grep -E "codelength|T " | grep -v "best 1000" | tail -12
timeout -k 10 120 python tools/im_dist.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout 600 --timeout-method thread -rf -s -v tests/test_infomap.py tests/test_leiden.py > gpurun_out/im.out 2>&1; rc=$?
grep -E "infomap |leiden LFR|FAIL|passed|failed" gpurun_out/im.out | tail -20
[ $rc -eq 0 ] || { tail -30 gpurun_out/im.out; exit $rc; }
