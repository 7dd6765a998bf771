#!/bin/bash
# The drop-in host path around the engine at C3 (100k) and C4 (1M) sizes.
set -u
mkdir -p gpurun_out/dropin4
timeout -k 10 400 python3 tools/dropin_bench.py 100000 64 > gpurun_out/dropin4/c3.json 2> gpurun_out/dropin4/c3.err || exit 1
timeout -k 10 900 python3 tools/dropin_bench.py 1000000 64 > gpurun_out/dropin4/c4.json 2> gpurun_out/dropin4/c4.err || exit 1
