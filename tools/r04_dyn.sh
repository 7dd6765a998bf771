#!/bin/bash
# Dynamic item assignment in the replica-lane decide (FC_RL_DYN=1): twin parity subset with it, then A/B
set -u
OUT=gpurun_out/r04dyn
mkdir -p $OUT
export TMPDIR=/tmp
FC_RL_DYN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "twin or full_run or hybrid" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m --reps 3 base base@FC_RL_DYN=1 base base@FC_RL_DYN=1 && \
timeout -k 10 300 python3 tools/cd_ab.py --config lfr1m --algo 1 --reps 3 base base@FC_RL_DYN=1 && \
timeout -k 10 500 python3 tools/cd_ab.py --config sbm4m --algo 1 --reps 2 base base@FC_RL_DYN=1
