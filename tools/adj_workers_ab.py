#!/usr/bin/env python3
"""IdGraph.from_networkx at C4 size with different worker counts for the forked adjacency read
(FC_HOST_WORKERS), on one networkx graph built once.  Prints ms per worker count."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    import networkx as nx

    from fastconsensus_amd import core, synth
    u, v, _ = synth.lfr(n, 0.5, seed=42)
    G = nx.Graph()
    G.add_nodes_from(range(n))
    G.add_edges_from(zip(u.tolist(), v.tolist()))
    res = {}
    for w in [8, 4, 12, 16, 8, 24]:
        os.environ["FC_HOST_WORKERS"] = str(w)
        t = time.perf_counter()
        g = core.IdGraph.from_networkx(G)
        res.setdefault(w, []).append(round(1e3 * (time.perf_counter() - t), 1))
        assert g.u.size == u.size
    print(json.dumps({"n": n, "from_networkx_ms_by_workers": res, "cpus": len(os.sched_getaffinity(0))}))


if __name__ == "__main__":
    main()
