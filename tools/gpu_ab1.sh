#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q -x tests/test_gpu_parity.py -k "twin or heavy or full_run or storage or replay" > gpurun_out/ab1_tests.out 2>&1; rc=$?
tail -3 gpurun_out/ab1_tests.out; [ $rc -eq 0 ] || exit $rc
V="base@FC_SLOT_LISTS=0,FC_OWN_BALLOT=0 base@FC_SLOT_LISTS=1,FC_OWN_BALLOT=0 base@FC_SLOT_LISTS=0,FC_OWN_BALLOT=1 base"
timeout -k 10 400 python tools/cd_ab.py --reps 2 $V > gpurun_out/ab1_louv.out 2>&1; rc=$?; cat gpurun_out/ab1_louv.out | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/cd_ab.py --config lfr100k_lpm --algo 1 --reps 2 $V > gpurun_out/ab1_lpa.out 2>&1; rc=$?; cat gpurun_out/ab1_lpa.out | grep -v amdgpu.ids; exit $rc
