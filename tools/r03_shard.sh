#!/bin/bash
# Sharded closure on the GPU: parity tests, then the per-rank closure time (tools/closure_shard_time.py)
set -u
mkdir -p gpurun_out/sh
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "closure or repair or full_run_bit_exact" > gpurun_out/sh/pytest.log 2>&1 || { tail -30 gpurun_out/sh/pytest.log; exit 1; }
tail -3 gpurun_out/sh/pytest.log
timeout -k 10 300 python3 -u tools/closure_shard_time.py > gpurun_out/sh/time.json 2> gpurun_out/sh/time.err || { tail -20 gpurun_out/sh/time.err; exit 1; }
cat gpurun_out/sh/time.json
