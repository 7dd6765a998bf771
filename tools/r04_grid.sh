#!/bin/bash
# Replica-lane decide grid: resident waves x mul (FC_RL_GRID_MUL; 0 = up to 8192 blocks)
set -u
OUT=gpurun_out/r04grid
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "twin or full_run or hybrid" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m --reps 3 base base@FC_RL_GRID_MUL=0 base@FC_RL_GRID_MUL=2 base base@FC_RL_GRID_MUL=0 && \
timeout -k 10 500 python3 tools/cd_ab.py --config sbm4m --algo 1 --reps 2 base base@FC_RL_GRID_MUL=0
