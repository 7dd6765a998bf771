#!/bin/bash
# Round-3 bench lines: the default (driver) line with its CPU baseline, its rocprofv3 kernel stats,
# and the other configs' lines.
set -u
OUT=gpurun_out/fc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/lfr1m.json 2> $OUT/lfr1m.err || { echo "bench lfr1m failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lfr1m --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
for cfg in lfr100k lfr100k_lpm sbm4m; do
    timeout -k 10 400 python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo "bench $cfg failed"; exit 1; }
done
timeout -k 10 400 python3 bench.py --n-p 8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/np8.json 2> $OUT/np8.err || { echo "bench np8 failed"; exit 1; }
timeout -k 10 400 python3 bench.py --config lfr1m_leiden --steps 2 --warmup 1 --no-cpu-baseline > $OUT/leiden.json 2> $OUT/leiden.err || { echo "bench leiden failed"; exit 1; }
timeout -k 10 400 python3 bench.py --config lfr100k_infomap --steps 2 --warmup 1 --no-cpu-baseline > $OUT/infomap.json 2> $OUT/infomap.err || { echo "bench infomap failed"; exit 1; }
echo done
