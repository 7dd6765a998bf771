#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q -x tests/test_gpu_parity.py -k "twin or heavy or full_run or storage or replay" > gpurun_out/ab4_tests.out 2>&1; rc=$?
tail -3 gpurun_out/ab4_tests.out; [ $rc -eq 0 ] || exit $rc
V="base@FC_ORDER_SWEEPS=200 base@FC_ORDER_SWEEPS=2 base@FC_ORDER_SWEEPS=3 base base@FC_ORDER_SWEEPS=6"
timeout -k 10 600 python tools/cd_ab.py --reps 2 $V > gpurun_out/ab4_louv.out 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/cd_ab.py --config sbm4m --algo 1 --reps 1 base@FC_ORDER_SWEEPS=200 base > gpurun_out/ab4_sbm.out 2>&1; exit $?
