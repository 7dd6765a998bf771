#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of tools/profile.sh into profiles/ (per-kernel stats and
per-launch HBM bytes of the dominant kernel, FETCH_SIZE doubled per MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main(prof_dir, config, out_dir="profiles", tag="r01"):
    os.makedirs(out_dir, exist_ok=True)
    stats = rows(os.path.join(prof_dir, "trace", "**", "*kernel_stats.csv"))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fastconsensus_amd.build import built_hash
    # the library these counters came from (bench.py attaches traffic only to a same-hash run)
    summary = {"config": config, "csrc_hash": built_hash(), "kernels": []}
    for r in stats:
        summary["kernels"].append({k: r[k] for k in r})
    counters = defaultdict(lambda: defaultdict(list))
    for name in ("fetch", "write", "l2", "sq", "sq1", "sq2"):
        for r in rows(os.path.join(prof_dir, name, "**", "*counter_collection.csv")):
            kern = r.get("Kernel_Name", "?")
            short = kern.split("(")[0].split("<")[0].strip()
            if "k_decide_light" in kern:   # per instance: <true, int> is the consensus runs' Louvain kernel
                targs = kern.split("<", 1)[1].split(">")[0].replace(" ", "")
                short = "k_decide_light<%s>" % {"true,int": "louvain", "false,int": "lpa"}.get(targs, targs)
            elif re.search(r"k_rl_decide<", kern):   # the replica-lane decide family (every K / weight instance)
                short = "k_rl_decide<%s>" % ("louvain" if "k_rl_decide<true" in kern.replace(" ", "") else "lpa")
            elif "k_lv_" in kern:       # Leiden / Infomap kernels: one entry per kernel (all instances)
                # (anonymous-namespace names: "void fc::(anonymous namespace)::k_lv_decide<...>(...)")
                short = re.search(r"(k_lv_\w+)", kern).group(1)
            counters[short][r.get("Counter_Name", "?")].append(float(r.get("Counter_Value", "nan")))
    per = {}
    for kern, cs in counters.items():
        per[kern] = {c: (sum(v) / len(v), len(v)) for c, v in cs.items()}
    summary["counters_mean_per_launch"] = {k: {c: v[0] for c, v in d.items()} for k, d in per.items()}
    # the consensus runs' decide kernel: LPA for lpm workloads, else Louvain (<true,int>; the
    # load-time ordering pass runs <true,long> and is not counted)
    lpa = "lpm" in config or "sbm" in config
    dec = [k for k in per if k.startswith("k_decide_light<lpa" if lpa else "k_decide_light<louvain")]
    if dec:
        d = per[dec[0]]
        fetch = d.get("FETCH_SIZE", (None,))[0]
        write = d.get("WRITE_SIZE", (None,))[0]
        if fetch is not None and write is not None:
            # FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE reads 1/2 of a wide stream (guide §HBM)
            summary["decide_hbm_bytes_per_launch"] = (2.0 * fetch + write) * 1024.0
            summary["decide_hbm_bytes_per_launch_uncorrected"] = (fetch + write) * 1024.0
        hit, miss = d.get("TCC_HIT_sum", (None,))[0], d.get("TCC_MISS_sum", (None,))[0]
        if hit is not None and miss:
            summary["decide_l2_hit_rate"] = hit / (hit + miss)
    rl = [k for k in per if k == ("k_rl_decide<lpa>" if lpa else "k_rl_decide<louvain>")]
    if rl:
        d = per[rl[0]]
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            summary["rl_decide_hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"][0] + d["WRITE_SIZE"][0]) * 1024.0
            summary["rl_decide_hbm_bytes_per_launch_uncorrected"] = (d["FETCH_SIZE"][0] + d["WRITE_SIZE"][0]) * 1024.0
        hit, miss = d.get("TCC_HIT_sum", (None,))[0], d.get("TCC_MISS_sum", (None,))[0]
        if hit is not None and miss:
            summary["rl_decide_l2_hit_rate"] = hit / (hit + miss)
    # Leiden / Infomap: per-launch HBM bytes of their own kernels (bench attaches the dominant one)
    for kern in ("k_lv_decide", "k_lv_heavy"):
        d = per.get(kern)
        if d and "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            summary.setdefault("lv_hbm_bytes_per_launch", {})[kern] = (2.0 * d["FETCH_SIZE"][0] + d["WRITE_SIZE"][0]) * 1024.0
    with open(os.path.join(out_dir, "pmc_%s.json" % config), "w") as f:
        json.dump(summary, f, indent=1)
    # the rocprofv3 --stats summary itself, copied verbatim
    for p in glob.glob(os.path.join(prof_dir, "trace", "**", "*kernel_stats.csv"), recursive=True):
        with open(p) as fi, open(os.path.join(out_dir, "%s_%s_kernel_stats.csv" % (tag, config)), "w") as fo:
            fo.write(fi.read())
    print(json.dumps({k: v for k, v in summary.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:]))
