#!/usr/bin/env python3
"""Per-rank triadic-closure time when the closure is split over W ranks (distributed.py
_closure_sharded), measured on ONE GPU: LFR-1M (the C4 graph), one louvain consensus
iteration at n_p = 8 (one GPU's share at N = 8), then

  * replicated: fc_closure_sample(L) -- what every rank paid before;
  * sharded W:  per block, rank 0's sub-range drawn (fc_closure_block_sample) plus the add of
    ALL ranks' lists (fc_closure_block_add, gathered lists prepared untimed by drawing the
    other ranks' sub-ranges on this GPU), + begin/finish.  The two all-gathers per block
    (counts, then the lists) are not in the figure; their payload is reported.

Prints one JSON line.  Usage: python3 tools/closure_shard_time.py [n] [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastconsensus_amd import Engine, synth  # noqa: E402


def main(n=1_000_000, reps=3):
    u, v, _ = synth.lfr(n, 0.5, seed=42)
    eng = Engine(seed=42)
    eng.load_graph(n, u, v)
    L = eng.graph_info()[2]
    eng.cd(0, 0, 8, 8, 0)
    part = torch.empty(eng.m, dtype=torch.int32, device="cuda")
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, 8, 0.2, 0.02, part)
    res = {"graph": "LFR n=%d mu=0.5 (C4), one louvain iteration, n_p=8" % n, "attempts": L}

    def sync():
        torch.cuda.synchronize()
        eng._L.fc_synchronize(eng._ctx)

    nc_full = eng.closure_sample(L, 0)
    ts = []
    for _ in range(reps):
        sync()
        t = time.perf_counter()
        eng.closure_sample(L, 0)
        sync()
        ts.append(time.perf_counter() - t)
    res["replicated_ms"] = 1e3 * min(ts)
    res["candidates"] = nc_full
    for W in (1, 2, 4, 8):
        best, gathered = None, 0
        for _ in range(reps):
            total = 0.0
            gathered = 0
            sync()
            t = time.perf_counter()
            blocks = eng.closure_begin(L, 0)
            sync()
            total += time.perf_counter() - t
            for b in range(blocks):
                t0, t1 = L * b // blocks, L * (b + 1) // blocks
                lists = []
                for r in range(W):       # the other ranks' lists (untimed)
                    lo, hi = t0 + (t1 - t0) * r // W, t0 + (t1 - t0) * (r + 1) // W
                    buf = torch.empty(2 * max(hi - lo, 1), dtype=torch.int64, device="cuda")
                    k = eng.closure_block_sample(b, lo, hi, buf)
                    lists.append(buf[:2 * k])
                allp = torch.cat(lists)
                gathered += allp.numel() * 8
                lo, hi = t0, t0 + (t1 - t0) // W
                own = torch.empty(2 * max(hi - lo, 1), dtype=torch.int64, device="cuda")
                sync()
                t = time.perf_counter()
                eng.closure_block_sample(b, lo, hi, own)        # rank 0's draw
                eng.closure_block_add(b, allp, allp.numel() // 2)
                sync()
                total += time.perf_counter() - t
            sync()
            t = time.perf_counter()
            nc = eng.closure_finish()
            sync()
            total += time.perf_counter() - t
            assert nc == nc_full, (W, nc, nc_full)
            best = total if best is None else min(best, total)
        res["sharded_W%d_ms" % W] = 1e3 * best
        res["sharded_W%d_gathered_MB_per_iteration" % W] = gathered / 1e6
    eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
