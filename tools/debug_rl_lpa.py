#!/usr/bin/env python3
"""Debug aid (GPU box): first sweep at which the replica-lane engine's LPA on the weighted
consensus graph (tests/test_gpu_parity.py::test_cd_replica_lanes_visit_mode_bit_exact) departs
from the CPU twin, with the twin's LPA tie revisits on and off.
    python tools/debug_rl_lpa.py [n_r] [visit_div]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
n_r = int(sys.argv[1]) if len(sys.argv) > 1 else 64
os.environ["FC_RL_VISIT_DIV"] = sys.argv[2] if len(sys.argv) > 2 else "0"

import numpy as np  # noqa: E402

import fastconsensus_amd as fc  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from tests import test_gpu_parity as tp  # noqa: E402

case, eng = tp._weighted_consensus_engine(fc, 47)
eng.set_option("cd_engine", 1)
u, v, w, _ = eng.get_graph()
sigma = eng.node_map()
a_, b_ = sigma[u], sigma[v]
lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
o = np.lexsort((hi, lo))
g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
for S in range(1, 80):
    eng.set_params(0, S, 0)
    eng.cd(1, 0, n_r, n_r, 3)
    got = eng.get_labels(n_r)
    res = {}
    for ties in (1, 0):
        orc.lib().orc_set_lpa_ties(ties)
        exp, sw = orc.engine_cd(1, g_int, n_r, 0, 3, 47, shared=1, coarsen=0, max_sweeps=S)
        res[ties] = (got != exp[:, sigma])
    orc.lib().orc_set_lpa_ties(1)
    bad = np.argwhere(res[1])
    if len(bad):
        print("sweep cap", S, "mismatches (ties on)", len(bad), "ties off", int(res[0].sum()), "first", bad[:6].tolist())
        rr, x = bad[0]
        print("replica", rr, "node", x, "internal", sigma[x], "device label", got[rr, x])
        break
else:
    print("no mismatch up to 79 sweeps")
