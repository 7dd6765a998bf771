#!/usr/bin/env python3
"""Consensus-NMI distributions of the device (GPU box) against the reference loop's records.

Runs the default engine (or the engine options given) over the C3 gate seeds of
tests/test_gpu_cd_parity.py and prints tests/dist_gates.check's line for each case, without
asserting: the numbers DESIGN.md's "Consensus distribution" table quotes.

    python tools/gates.py [c3_lpm] [c3_louvain] [c2] [--opt name=value ...] [--seeds a:b]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from tests import dist_gates, golden_io  # noqa: E402


def refsem(name):
    with open(os.path.join(golden_io.GOLDEN, "refsem_%s.json" % name)) as f:
        return json.load(f)


def graph(case):
    from fastconsensus_amd import synth
    if case == "c2":
        z = golden_io.load("lfr1k_louvain_np20")
        planted = np.load(golden_io.GOLDEN + "/lfr1k_mu04_planted.npy")[z.z["nodes"]]
        return z.N, z.edges_file, planted
    kw = {"avg_deg": 8, "max_deg": 25} if case == "c3_lpm" else {}
    u, v, planted = synth.lfr(100_000, 0.5, seed=42, **kw)
    return 100_000, np.stack([u, v], 1), planted


CASES = {"c3_lpm": (1, 64, 0.8, "lfr100k_sparse_lpm_np64", 0.0005, (300, 340)),
         "c3_louvain": (0, 64, 0.2, "lfr100k_louvain_np64", 0.0005, (300, 340)),
         "c2": (0, 20, 0.2, "lfr1k_louvain_np20", 0.015, (1000, 1400))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["c3_lpm", "c3_louvain"])
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--seeds", default="")
    ap.add_argument("--save", default="")
    a = ap.parse_args()
    import fastconsensus_amd as fc
    saved = {}
    for case in a.cases:
        algo, n_p, tau, name, tol, (s0, s1) = CASES[case]
        if a.seeds:
            s0, s1 = map(int, a.seeds.split(":"))
        n, e, planted = graph(case)
        got = []
        for seed in range(s0, s1):
            with fc.Engine(seed=seed) as eng:
                for kv in a.opt:
                    k, val = kv.split("=")
                    eng.set_option(k, int(val))
                eng.load_graph(n, e[:, 0], e[:, 1])
                labels, st = eng.run(algo, n_p, tau, 0.02)
            got.append(float(np.mean([dist_gates.nmi(planted, x) for x in labels])))
        ref = refsem(name)["nmi"]
        try:
            dist_gates.check(got, ref, tol, "%s %s" % (case, " ".join(a.opt) or "default"),
                             ks=True, p10_slack=0.0005 if case.startswith("c3") else dist_gates.P10_SLACK)
            print("  -> all gates pass", flush=True)
        except AssertionError as err:
            print("  -> FAILS", str(err).split(":")[0], flush=True)
        saved[case] = got
    if a.save:
        with open(a.save, "w") as f:
            json.dump(saved, f)


if __name__ == "__main__":
    main()
