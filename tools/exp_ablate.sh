#!/bin/bash
# Decide-kernel ablations (FC_DBG bits: 1 no Sigma gathers, 2 no label gathers): sweep-0 decide time
set -u
export TMPDIR=/tmp
for dbg in ${DBGS:-0 1 2 3}; do
  OUT=gpurun_out/abl_$dbg; mkdir -p $OUT
  FC_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o tr --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/log 2>&1 || exit $?
  python3 - $OUT <<'PY'
import csv,glob,sys
p=glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True)[0]
rows=sorted(csv.DictReader(open(p)),key=lambda r:int(r["Start_Timestamp"]))
d=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in rows if "k_decide_light" in r["Kernel_Name"]]
print(sys.argv[1], "sweep0 decide us: %.0f  first %.0f last %.0f" % (sum(d[:32]), d[0], d[31]))
PY
done
