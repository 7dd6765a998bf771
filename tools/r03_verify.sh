#!/bin/bash
# Round-3 re-entry check: the GPU suite, smoke and the default bench line at HEAD.  Stops at the first failure.
set -u
mkdir -p gpurun_out/v
export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/v/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/v/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/v/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/v/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/v/smoke.log; exit 1; }
tail -2 gpurun_out/v/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err || { echo "bench failed"; tail -30 gpurun_out/v/bench.err; exit 1; }
cat gpurun_out/v/bench.json
