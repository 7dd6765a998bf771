#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q -x tests/test_gpu_parity.py -k "twin or heavy or full_run or storage or replay" > gpurun_out/ab2_tests.out 2>&1; rc=$?
tail -3 gpurun_out/ab2_tests.out; [ $rc -eq 0 ] || exit $rc
V="base@FC_OWN_BALLOT=0 base base@FC_OWN_BALLOT=0 base"
timeout -k 10 400 python tools/cd_ab.py --reps 3 $V > gpurun_out/ab2_louv.out 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab2_louv.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/cd_ab.py --config lfr100k_lpm --algo 1 --reps 3 base@FC_OWN_BALLOT=0 base > gpurun_out/ab2_lpa.out 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab2_lpa.out; exit $rc
