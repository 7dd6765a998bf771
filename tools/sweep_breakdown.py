#!/usr/bin/env python3
"""Per-sweep kernel time breakdown from a rocprofv3 kernel trace (k_sweep_end closes a sweep)."""
import csv, glob, sys
from collections import defaultdict
path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
sweeps, cur = [], defaultdict(float)
t0 = None
for r in rows:
    n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("fc::", "")
    if "rocprim" in n: n = "rocprim"
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if t0 is None: t0 = int(r["Start_Timestamp"])
    cur[n] += d
    if n == "k_sweep_end":
        cur["_wall"] = (int(r["End_Timestamp"]) - t0) / 1e3
        t0 = int(r["End_Timestamp"])
        sweeps.append(cur); cur = defaultdict(float)
keys = ["k_decide_light", "k_decide_heavy", "k_apply", "k_list_build", "k_list_offsets", "__amd_rocclr_fillBufferAligned", "_wall"]
print("sweep " + " ".join("%10s" % k[-10:] for k in keys))
for i, s in enumerate(sweeps[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]):
    print("%5d " % i + " ".join("%10.0f" % s.get(k, 0) for k in keys))
tot = defaultdict(float)
for s in sweeps:
    for k, v in s.items(): tot[k] += v
print("total " + " ".join("%10.0f" % tot.get(k, 0) for k in keys))
print("tail (after last sweep):", {k: round(v) for k, v in cur.items()})
