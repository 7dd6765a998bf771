#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in lfr100k lfr100k_lpm; do
  timeout -k 10 600 python bench.py --config $cfg --steps 3 --warmup 1 > gpurun_out/b_$cfg.out 2> gpurun_out/b_$cfg.err || { tail -20 gpurun_out/b_$cfg.err; exit 1; }
  tail -2 gpurun_out/b_$cfg.err
done
timeout -k 10 900 python bench.py --config sbm4m --steps 2 --warmup 1 > gpurun_out/b_sbm4m.out 2> gpurun_out/b_sbm4m.err || { tail -20 gpurun_out/b_sbm4m.err; exit 1; }
tail -3 gpurun_out/b_sbm4m.err
