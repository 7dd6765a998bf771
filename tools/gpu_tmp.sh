#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FC_TRACE=1 timeout -k 10 300 python bench.py --config lfr1m_leiden --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/b_l1m_trace.err || exit 1
grep -E "leiden|step" gpurun_out/b_l1m_trace.err | tail -30
