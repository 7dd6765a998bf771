#!/bin/bash
# Whole GPU suite + smoke (round-end checks), then an optional extra script.
set -u
OUT=gpurun_out/r04suite
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ $# -gt 0 ]; then "$@"; fi
