#!/usr/bin/env python3
"""Kernel time inside each closure window (first k_closure_sample .. k_scatter_cand) of a
rocprofv3 kernel trace: python tools/phase_windows.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
i, wins = 0, []
while i < len(rows):
    if "k_closure_sample" in rows[i]["Kernel_Name"]:
        j = i
        while j < len(rows) and "k_scatter_cand" not in rows[j]["Kernel_Name"]:
            j += 1
        wins.append((i, min(j, len(rows) - 1)))
        i = j + 1
    else:
        i += 1
for (i, j) in wins:
    t0, t1 = int(rows[i]["Start_Timestamp"]), int(rows[j]["End_Timestamp"])
    agg = {}
    for r in rows[i:j + 1]:
        n = r["Kernel_Name"].split("(")[0][-48:]
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(v[1] for v in agg.values())
    print("closure window %.2f ms, kernels %.2f ms, %d launches" % ((t1 - t0) / 1e6, busy / 1e6, j - i + 1))
    for n, (cnt, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:6]:
        print("   %-48s %4d %8.1f us" % (n, cnt, d / 1e3))
