"""Export cost of the final labelings (fc_get_labels into a caller host array: renumber kernels +
256 MB download) after one LFR-1M CD batch at n_p=64, into a touched pageable vs a pinned array.
Measured: 6.8 vs 6.7 ms -- the runtime's staging of a pageable destination is not the bound (a
pinned double-buffer with parallel host copies was tried: 7.4 ms, reverted)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import fastconsensus_amd as fc  # noqa: E402

cfg = bench.CONFIGS["lfr1m"]
n, u, v, _ = bench.make_graph(cfg, 42)
with fc.Engine(seed=42) as eng:
    eng.load_graph(n, u, v)
    eng.cd(0, 0, 64, 64, 0)
    page = np.zeros((64, n), np.int32)
    page.fill(1)
    pin = torch.empty((64, n), dtype=torch.int32, pin_memory=True).numpy()
    for name, out in (("pageable", page), ("pinned", pin)):
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            eng.get_labels_into(out, renumber=True)
            ts.append(1e3 * (time.perf_counter() - t))
        print("%s: %s ms" % (name, " ".join("%.1f" % x for x in ts)), flush=True)
