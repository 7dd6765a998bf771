"""Load the golden fixtures written by tests/golden/make_golden.py (data only)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["karate_louvain_np50", "karate_lpm_np20", "lfr1k_louvain_np20", "lfr1k_lpm_np20",
         "karate_louvain_nc_np50", "lfr1k_louvain_nc_np20",    # nc: new_consensus.py's weight rule
         "lfr1k_mu055_lpm_np20", "lfr1k_mu03_lpm_np20",        # lpm where LPA finds structure
         "karate_infomap_np20", "lfr1k_infomap_np20"]          # infomap: the lpm loop (:260-310)
LEIDEN_CASES = ["karate_leiden_np20", "lfr1k_leiden_np20"]     # the leiden branch's exit (:204-258)


class Case:
    def __init__(self, name):
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.name = name
        # loop rule: 0 louvain, 1 lpm (and infomap: the same loop, :260-310), 2 louvain with the
        # new_consensus.py rule (FC_ALGO_LOUVAIN_NC), 3 leiden (:204-258)
        a = self.meta["algorithm"]
        self.algo = {"lpm": 1, "infomap": 1, "leiden": 3}.get(a, 2 if self.meta.get("rule") == "new_consensus" else 0)
        self.n_p = self.meta["n_p"]
        self.tau = self.meta["tau"]
        self.delta = self.meta["delta"]
        self.N = self.meta["N"]
        self.edges_file = self.z["edges_file"]
        n_p = self.n_p
        cd = self.z["cd_labels"]
        self.cd_batches = [cd[b * n_p:(b + 1) * n_p] for b in range(len(cd) // n_p)]
        self.pair_batches = []
        b = 0
        while "pairs%d" % b in self.z:
            self.pair_batches.append(self.z["pairs%d" % b])
            b += 1
        self.checks = [(self.z["check%d_edges" % c], self.meta["check_results"][c])
                       for c in range(self.meta["n_checks"])]
        self.adj = []
        b = 0
        while "adj%d_ptr" % b in self.z:
            self.adj.append((self.z["adj%d_ptr" % b], self.z["adj%d_nbr" % b], self.z["adj%d_w" % b]))
            b += 1

    def check_dict(self, c):
        e, _ = self.checks[c]
        out = {}
        for u, v, w in e:
            u, v = int(u), int(v)
            assert float(w).is_integer()
            out[(min(u, v), max(u, v))] = int(w)
        return out


def load(name):
    return Case(name)
