#!/usr/bin/env python3
"""Wall time of whole fc_run calls with the per-launch HIP-event timing off and on (does the
instrumentation bench.py enables cost time?).   python tools/timing_ab.py [config] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import fastconsensus_amd as fc
from fastconsensus_amd.core import ALGORITHMS

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "lfr100k_infomap"])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n, u, v, _ = bench.make_graph(cfg, 42)
host = np.zeros((cfg["n_p"], n), np.int32)
with fc.Engine(seed=42) as eng:
    eng.load_graph(n, u, v)
    eng.run(ALGORITHMS[cfg["algo"]], cfg["n_p"], cfg["tau"], cfg["delta"], out=host)   # warm
    for timing in (False, True, False, True):
        eng.set_timing(timing)
        ts = []
        for r in range(reps):
            t0 = time.perf_counter()
            eng.run(ALGORITHMS[cfg["algo"]], cfg["n_p"], cfg["tau"], cfg["delta"], out=host)
            ts.append(1e3 * (time.perf_counter() - t0))
        eng.collect_timing()
        print("timing=%d runs %s ms (min %.1f)" % (timing, [round(x, 1) for x in ts], min(ts)), flush=True)
