#!/bin/bash
# Occupancy bounds on k_rl_decide (variants w64: K16 6 waves / K32 4 waves; w53: 5 / 3) vs base, hybrid engine.
set -u
export TMPDIR=/tmp FC_AB_OPTS="cd_engine=2"
timeout -k 10 600 python3 tools/cd_ab.py --config lfr1m --reps 3 base w64 w53 base
