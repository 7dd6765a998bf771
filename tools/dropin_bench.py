#!/usr/bin/env python3
"""What a drop-in caller of fast_consensus() pays around the engine (GPU box):

    python tools/dropin_bench.py [n] [n_p]

Times, for the LFR graph of n nodes (mu=0.5, native generator):
  * networkx path: nx.Graph construction (outside fast_consensus, the caller's), then
    fastconsensus_amd.fast_consensus(G, 'louvain', n_p) split into IdGraph.from_networkx,
    the engine (create + upload + every iteration + final pass + download) and the conversion
    of the labelings to the reference's return type (list of dicts, fast_consensus.py:384);
  * IdGraph path: the same call on an IdGraph (no networkx conversion).
Prints one JSON line per path (ms per phase)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    n_p = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    import networkx as nx
    import numpy as np

    import fastconsensus_amd as fc
    from fastconsensus_amd import core, synth
    u, v, _ = synth.lfr(n, 0.5, seed=42)
    g = core.IdGraph(np.arange(n, dtype=np.int64), u, v)
    fc.fast_consensus(g, "louvain", n_p, seed=1)          # warm: library, device, allocations
    # IdGraph path, split
    t0 = time.perf_counter()
    with fc.Engine(device=0, seed=2) as eng:
        eng.set_option("store", core.store_order_pays(n_p))
        eng.load_graph(g.n, g.u, g.v)
        labels, st = eng.run(0, n_p, 0.2, 0.02)
    t1 = time.perf_counter()
    out = core.labels_to_output("louvain", g.labels, labels)
    t2 = time.perf_counter()
    res = {"path": "IdGraph", "n": n, "m": int(len(u)), "n_p": n_p, "engine_ms": 1e3 * (t1 - t0),
           "to_dicts_ms": 1e3 * (t2 - t1), "total_ms": 1e3 * (t2 - t0), "iterations": st["iterations"]}
    print(json.dumps(res), flush=True)
    del out
    # networkx path
    t0 = time.perf_counter()
    G = nx.Graph()
    G.add_nodes_from(range(n))
    G.add_edges_from(zip(u.tolist(), v.tolist()))
    t1 = time.perf_counter()
    ig = core.IdGraph.from_networkx(G)
    t2 = time.perf_counter()
    with fc.Engine(device=0, seed=3) as eng:
        eng.set_option("store", core.store_order_pays(n_p))
        eng.load_graph(ig.n, ig.u, ig.v)
        labels, st = eng.run(0, n_p, 0.2, 0.02)
    t3 = time.perf_counter()
    out = core.labels_to_output("louvain", ig.labels, labels)
    t4 = time.perf_counter()
    t5 = time.perf_counter()
    whole = fc.fast_consensus(G, "louvain", n_p, seed=4)     # the drop-in call itself, end to end
    t6 = time.perf_counter()
    res = {"path": "networkx", "n": n, "m": G.number_of_edges(), "n_p": n_p,
           "nx_graph_build_ms (caller)": 1e3 * (t1 - t0), "from_networkx_ms": 1e3 * (t2 - t1),
           "engine_ms": 1e3 * (t3 - t2), "to_dicts_ms": 1e3 * (t4 - t3),
           "fast_consensus_call_ms": 1e3 * (t6 - t5), "partitions": len(whole)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
