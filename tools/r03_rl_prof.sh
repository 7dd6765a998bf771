#!/bin/bash
# Kernel stats of the replica-lane engine on LFR-1M (2 steps).
set -u
OUT=gpurun_out/rlprof
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lfr1m --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", tot / 1e6)
for r in rows[:30]:
    print("%8.2f ms %6s calls %8.1f us  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:100]))
PY
cp "$f" $OUT/kernel_stats.csv
