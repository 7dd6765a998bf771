#!/usr/bin/env python3
"""Leiden quality per bucket setting (GPU box): mean modularity and community count of the
device Leiden on LFR-100k (8 replicas) and LFR-1M (4 replicas) for the environment given
(FC_LV_LEVEL_B / FC_LV_QUEUE_DIV are read by the engine at context creation)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

import fastconsensus_amd as fc
from fastconsensus_amd import synth
from oracle import oracle as orc

for n, reps in ((100_000, 8), (1_000_000, 4)):
    u, v, planted = synth.lfr(n, 0.5, seed=42)
    e = np.stack([u, v], 1)
    g = orc.EdgeGraph.from_lines(n, e)
    with fc.Engine(seed=5) as eng:
        eng.load_graph(n, u, v)
        eng.cd(3, 0, reps, reps, 0)
        lab = eng.get_labels(reps)
    q = np.mean([orc.modularity(g, x) for x in lab])
    k = np.mean([len(np.unique(x)) for x in lab])
    print("n=%d env LEVEL_B=%s REFINE_B=%s: Q %.5f k %.1f" % (n, os.environ.get("FC_LV_LEVEL_B"), os.environ.get("FC_LV_REFINE_B"), q, k), flush=True)
