#!/usr/bin/env python3
"""Per-launch join of tools/pmc_cd.sh passes (same program, same dispatch ids): for each
k_decide_light<true,int> launch its grid, duration (trace pass), TCC hits/misses and
FETCH_SIZE; grouped into sweeps (runs of one grid size) of each CD batch.
    python tools/pmc_per_launch.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "k_decide_light<true, int>"


def load(name):
    p = os.path.join(d, name, name + "_counter_collection.csv")
    out = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(p)):
        i = int(r["Dispatch_Id"])
        out[i][r["Counter_Name"]] = out[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[i] = (r["Kernel_Name"], int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
    return out, meta


l2, meta = load("l2")
fe, _ = load("fetch")
dur = {}
for r in csv.DictReader(open(os.path.join(d, "trace", "trace_kernel_trace.csv"))):
    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
groups = []
for i in sorted(meta):
    name, grid = meta[i]
    if want not in name:
        continue
    if not groups or groups[-1]["grid"] != grid or i - groups[-1]["last"] > 40:
        groups.append({"grid": grid, "n": 0, "us": 0.0, "hit": 0.0, "miss": 0.0, "fetch": 0.0, "first": i})
    g = groups[-1]
    g["last"] = i
    g["n"] += 1
    g["us"] += dur.get(i, 0.0)
    g["hit"] += l2[i].get("TCC_HIT_sum", 0)
    g["miss"] += l2[i].get("TCC_MISS_sum", 0)
    g["fetch"] += fe.get(i, {}).get("FETCH_SIZE", 0)
print("%6s %8s %4s %9s %10s %10s %6s %9s %9s" % ("first", "grid", "n", "us", "miss/M", "hit/M", "hit%", "Gmiss/s", "visits/M"))
for g in groups:
    vis = g["grid"] * 8 * g["n"] / 1e6
    print("%6d %8d %4d %9.0f %10.2f %10.2f %6.1f %9.1f %9.2f" % (
        g["first"], g["grid"], g["n"], g["us"], g["miss"] / 1e6, g["hit"] / 1e6,
        100 * g["hit"] / max(1, g["hit"] + g["miss"]), g["miss"] / max(1e-9, g["us"] * 1e3), vis))
