#!/bin/bash
# Leiden GPU checks: each step under its own timeout; stop at the first fault/abort/timeout.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -p no:cacheprovider --timeout 600 --timeout-method thread -rf"
timeout -k 10 900 $PYT -s -v -x tests/test_leiden.py > gpurun_out/leiden.out 2> gpurun_out/leiden.err
rc=$?; echo "leiden tests rc=$rc"; tail -40 gpurun_out/leiden.out; tail -20 gpurun_out/leiden.err
exit $rc
