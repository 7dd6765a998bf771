#!/usr/bin/env python3
"""Fixtures for the device Infomap tests: igraph's FULL Infomap partition (the greedy core plus
its single-node and sub-module re-partition rounds, restated as oracle/fc_oracle.c
orc_infomap_full) on the graphs tests/test_infomap.py uses.  The restatement takes ~100 s per
run at LFR-100k, so the GPU tests compare with these stored values instead of running it.
    python tests/golden/make_infomap_full.py      (CPU; writes infomap_full.json here)"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    from sklearn.metrics import normalized_mutual_info_score as nmi

    from fastconsensus_amd import synth
    from oracle import oracle as orc
    out = {}
    for name, n, mu, seeds in (("lfr1k_mu04", 1000, 0.4, range(8)), ("lfr100k_mu05", 100_000, 0.5, range(2))):
        u, v, planted = synth.lfr(n, mu, seed=42)
        g = orc.EdgeGraph.from_lines(n, np.stack([u, v], 1))
        runs = []
        for s in seeds:
            lab, L, Lc = orc.infomap_full(g, seed=s)
            runs.append({"seed": s, "L": L, "L_core": Lc, "modules": int(len(np.unique(lab))),
                         "nmi": float(nmi(planted, lab))})
            print(name, runs[-1], flush=True)
        out[name] = {"graph": "synth.lfr(%d, %.1f, seed=42)" % (n, mu), "runs": runs,
                     "L_mean": float(np.mean([r["L"] for r in runs])),
                     "modules_mean": float(np.mean([r["modules"] for r in runs])),
                     "nmi_mean": float(np.mean([r["nmi"] for r in runs]))}
    with open(os.path.join(HERE, "infomap_full.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
