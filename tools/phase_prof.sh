#!/bin/bash
# Decide-kernel phase cycles (FC_PHASE_PROF build in fastconsensus_amd/lib/phase/, built on the CPU host):
# cumulative s_memtime per phase of decide_wave, sampled on 1/64 of the blocks.
set -u
mkdir -p gpurun_out
FC_LIB_PATH=fastconsensus_amd/lib/phase/libfastconsensus_amd.so timeout -k 10 300 \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/phase.json 2> gpurun_out/phase.err
rc=$?; grep "phase cycles" gpurun_out/phase.err | tail -n 1; exit $rc
