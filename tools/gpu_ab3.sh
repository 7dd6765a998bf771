#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="base base@FC_PUSH_DIV=0 base@FC_PUSH_DIV=2 base@FC_TRACK_DIV=2 base@FC_TRACK_DIV=8 base@FC_TRACK_DIV=2,FC_PUSH_DIV=2 base@FC_TRACK_DIV=1,FC_PUSH_DIV=2"
timeout -k 10 600 python tools/cd_ab.py --reps 2 $V > gpurun_out/ab3_louv.out 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab3_louv.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/cd_ab.py --config lfr100k_lpm --algo 1 --reps 2 $V > gpurun_out/ab3_lpa.out 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab3_lpa.out; exit $rc
