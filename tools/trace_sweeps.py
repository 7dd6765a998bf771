#!/usr/bin/env python3
"""Per-sweep view of a rocprofv3 kernel trace of bench.py: CD batches (k_cd_init), and per
sweep (consecutive k_decide_light launches of one grid) launches, grid, decide/apply time.
    python tools/trace_sweeps.py <kernel_trace.csv> [batch_from] [batch_to]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
batch, cur, out = -1, None, []
t_batch = {}
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_cd_init" in n:
        batch += 1
        cur = None
    if batch < 0:
        continue
    t_batch.setdefault(batch, {}).setdefault(n.split("(")[0][:40], 0.0)
    t_batch[batch][n.split("(")[0][:40]] += d
    if not (lo <= batch <= hi):
        continue
    if "k_decide_light" in n:
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        if cur is None or cur["grid"] != g or cur.get("closed"):
            cur = {"batch": batch, "grid": g, "n": 0, "dec": 0.0, "app": 0.0, "other": 0.0}
            out.append(cur)
        cur["n"] += 1
        cur["dec"] += d
    elif cur is not None and "k_apply" in n:
        cur["app"] += d
    elif cur is not None and ("k_list_count" in n or "k_cd_tail" in n):
        cur["closed"] = True
        if "k_cd_tail" in n:
            out.append({"batch": batch, "grid": -1, "n": 1, "dec": d, "app": 0.0, "other": 0.0})
for s in out:
    print("batch %2d grid %8d launches %3d decide %8.1f us apply %7.1f us" % (s["batch"], s["grid"], s["n"], s["dec"], s["app"]))
for b, t in sorted(t_batch.items()):
    if lo <= b <= hi:
        tot = sum(t.values())
        top = sorted(t.items(), key=lambda kv: -kv[1])[:5]
        print("batch %d: %.1f ms kernels; top %s" % (b, tot / 1e3, ", ".join("%s %.1f" % (k, v / 1e3) for k, v in top)))
