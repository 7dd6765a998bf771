#!/usr/bin/env python3
"""Closure sampler cost vs closure_rounds on the LFR-1M kept graph of iteration 0 (GPU box).
    python tools/closure_bench.py [n_p]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import fastconsensus_amd as fc  # noqa: E402

n_p = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = bench.CONFIGS["lfr1m"]
n, u, v, _ = bench.make_graph(cfg, 42)
with fc.Engine(seed=42) as eng:
    eng.load_graph(n, u, v)
    m0 = eng.m
    eng.cd(0, 0, n_p, n_p, 0)
    part = torch.zeros(m0, dtype=torch.int32, device="cuda")
    eng.consensus_partial(0, part)
    conv, kept, unc = eng.consensus_apply(0, n_p, 0.2, 0.02, part)
    print("m0 %d kept %d" % (m0, kept))
    for rounds in (1, 2, 4, 8, 16, 32):
        eng.set_option("closure_rounds", rounds)
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            nc = eng.closure_sample(m0, 0)
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t))
        print("rounds %2d: candidates %d, %.2f ms (min of 3)" % (rounds, nc, min(ts)), flush=True)
