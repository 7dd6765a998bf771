#!/bin/bash
# Leiden per-level trace, then the drop-in host path at C3 and C4 sizes.
set -u
mkdir -p gpurun_out/lt gpurun_out/dropin
export TMPDIR=/tmp
FC_TRACE=1 timeout -k 10 300 python3 -u bench.py --config lfr1m_leiden --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/lt/leiden.json 2> gpurun_out/lt/leiden.err || { echo "leiden failed"; exit 1; }
grep "leiden level" gpurun_out/lt/leiden.err | grep -v sweep | head -20
timeout -k 10 300 python3 -u tools/dropin_bench.py 100000 64 > gpurun_out/dropin/c3.json 2> gpurun_out/dropin/c3.err || { echo "dropin c3 failed"; exit 1; }
cat gpurun_out/dropin/c3.json
timeout -k 10 600 python3 -u tools/dropin_bench.py 1000000 64 > gpurun_out/dropin/c4.json 2> gpurun_out/dropin/c4.err || { echo "dropin c4 failed"; exit 1; }
cat gpurun_out/dropin/c4.json
