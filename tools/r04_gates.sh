#!/bin/bash
# The reference-distribution gates with their printed margins (C2 / C3, every CD engine setting)
set -u
mkdir -p gpurun_out/gates
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -s --timeout 600 --timeout-method thread tests/test_gpu_cd_parity.py \
    -k "c2_ or c3_consensus" -m gpu > gpurun_out/gates/gates.log 2>&1; rc=$?
grep -E "C2|C3|passed|failed" gpurun_out/gates/gates.log | head -40
exit $rc
