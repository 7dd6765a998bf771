"""Replica-lane engine vs its CPU twin on LFR-1k at growing difficulty (debug aid)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import fastconsensus_amd as fc
from oracle import oracle as orc
from tests import golden_io

case = golden_io.load("lfr1k_louvain_np20")
e = case.edges_file
for algo in (0, 1):
    for buckets, ms, n_r in [(1, 1, 1), (1, 1, 6), (2, 1, 1), (32, 1, 1), (32, 1, 6), (32, 2, 1), (32, 200, 1), (32, 200, 6),
                             (32, 200, 64)]:
        eng = fc.Engine(seed=99)
        eng.set_params(buckets=buckets, max_sweeps=ms)
        eng.set_option("chunk", 0)
        eng.set_option("prune", 0)
        eng.load_graph(case.N, e[:, 0], e[:, 1])
        eng.cd(algo, 0, n_r, n_r, 4)
        got = eng.get_labels(n_r)
        sigma = eng.node_map()
        g_int = orc.EdgeGraph.from_lines(case.N, np.stack([sigma[e[:, 0]], sigma[e[:, 1]]], 1))
        exp, sw = orc.engine_cd(algo, g_int, n_r, 0, 4, 99, buckets=buckets, max_sweeps=ms, chunk=0, prune=0)
        exp = exp[:, sigma]
        bad = (got != exp).sum(1)
        print("algo", algo, "buckets", buckets, "max_sweeps", ms, "n_r", n_r, "mismatch per replica", bad.tolist()[:8],
              "twin sweeps", sw.tolist()[:4], flush=True)
        if bad.any() and ms == 1 and buckets == 1:
            r = int(np.argmax(bad > 0))
            idx = np.nonzero(got[r] != exp[r])[0][:5]
            print("  nodes", idx.tolist(), "got", got[r, idx].tolist(), "exp", exp[r, idx].tolist())
        eng.close()
