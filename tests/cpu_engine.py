"""CPU model of the engine's step API, built on the oracle (TEST INFRASTRUCTURE ONLY).

Drives fastconsensus_amd.distributed.run_sharded over gloo on CPU (the multi-rank logic:
replica ranges, k_last MAX / count SUM all-reduces, identical replicated updates), and is
compared bit-for-bit with the HIP engine on the GPU.  It restates the engine's semantics:
bucketed CD (oracle twin), closed-form consensus rule, counter-based closure sampler,
isolate repair and the age model.
"""
import numpy as np

from oracle import oracle as orc


class OracleEngine:
    def __init__(self, seed, buckets=None, chunk=16, prune=1, sigma=None, coarsen=8, prune_mark=1, shared=2,
                 dense_div=orc.DENSE_DIV):
        """sigma: node id -> internal id (the engine's fc_get_node_map); None = identity.  Defaults:
        the default (hybrid) CD engine, FC_OPT_CD_ENGINE=2; shared=0 models the classic engine,
        shared=1, coarsen=0 the replica-lane engine (FC_OPT_CD_ENGINE=1, cd_rl.hip: one shared
        visit order in every sweep, no coarse rounds)."""
        self.seed = int(seed)
        self.buckets = buckets
        self.chunk = chunk
        self.prune = prune
        self.coarsen = coarsen
        self.prune_mark = prune_mark
        self.shared = shared
        self.dense_div = dense_div
        self.sigma = None if sigma is None else np.asarray(sigma, np.int32)
        self.lab = None
        self.algo = 0                                 # the last consensus_apply's (engine: Ctx::clo_algo)

    # graph -----------------------------------------------------------------------------
    def load_graph(self, n, u, v):
        u, v = np.asarray(u), np.asarray(v)
        if self.sigma is None:
            self.sigma = np.arange(n, dtype=np.int32)
        self.npos = np.empty(n, np.int32)
        self.npos[self.sigma] = np.arange(n, dtype=np.int32)
        self.g0 = orc.EdgeGraph.from_lines(n, np.stack([self.sigma[u], self.sigma[v]], 1))
        self.m0 = self.g0.m
        self.reset_graph()

    def set_stream(self, s):
        pass

    def reset_graph(self):
        g = self.g0
        self.g = orc.EdgeGraph(g.N, g.u.copy(), g.v.copy(), g.w.copy(), g.age.copy())

    def graph_info(self):
        return self.g.N, self.g.m, self.m0

    @property
    def m(self):
        return self.g.m

    # steps -----------------------------------------------------------------------------
    def cd(self, algo, r0, count, n_p, iteration):
        if algo in (orc.LEIDEN, orc.INFOMAP):
            # the sequential restatements, one per replica, seeded by the GLOBAL replica index
            # (the device keys its randomness the same way, so results do not depend on sharding)
            rows = []
            for r in range(r0, r0 + count):
                sd = (self.seed * 0x9E3779B1 + r * 0x85EBCA77 + iteration * 0xC2B2AE3D) & (2**63 - 1)
                rows.append(orc.cd_batch(algo, 1, self.g, sd)[0][0])
            self.lab = np.stack(rows) if rows else np.zeros((0, self.g.N), np.int32)
        else:
            self.lab, _ = orc.engine_cd(algo, self.g, count, r0, iteration, self.seed, buckets=self.buckets,
                                        chunk=self.chunk, prune=self.prune, coarsen=self.coarsen,
                                        prune_mark=self.prune_mark, shared=self.shared, dense_div=self.dense_div)
        self.r0 = r0

    def consensus_partial(self, algo, out):
        g, lab = self.g, self.lab
        diff = lab[:, g.u] != lab[:, g.v]
        if algo == 0:
            idx = lab.shape[0] - 1 - np.argmax(diff[::-1], axis=0)
            res = np.where(diff.any(0), self.r0 + idx, -1)
        else:
            res = (~diff).sum(0)
        out.numpy()[:g.m] = res

    def consensus_apply(self, algo, n_p, tau, delta, part):
        g = self.g
        p = part.numpy()[:g.m].astype(np.int64)
        if algo == 0:
            nw = np.where((g.w == 0) | (g.w == n_p), 0, np.where(p < 0, n_p, g.w + n_p - 1 - p))
        elif algo == 2:                               # new_consensus.py:155-163
            nw = np.where((g.w == 0) | (g.w == n_p), g.w, p)
        else:
            nw = p
        nw = nw.astype(np.int32)
        keep = orc.threshold(nw, tau, n_p)
        self.kept = orc.EdgeGraph(g.N, g.u[keep], g.v[keep], nw[keep], g.age[keep])
        self.algo = algo                              # the closure's block count follows the loop
        conv, cnt = orc.check(self.kept.w, n_p, delta)
        return (conv if algo in (0, 2) else False), self.kept.m, cnt   # louvain loops have check #1

    def closure_sample(self, attempts, iteration):
        pairs = orc.closure_sample_pairs(self.kept, attempts, self.seed, iteration, orc.closure_rounds(self.algo))
        dummy = np.zeros((1, self.g.N), np.int32)
        cu, cv, _, cf = orc.closure_from_pairs(1, self.kept, pairs, dummy, 1)
        order = np.lexsort((cv, cu))                  # the device keeps candidates key-sorted
        self.cand = (cu[order], cv[order], cf[order])
        return len(cu)

    # sharded closure (distributed._closure_sharded): the rank's sub-range of a block as
    # (key, first attempt) pairs, the gathered lists re-assembled into the attempt-indexed pair
    # array, first occurrences kept -- the same candidates as closure_sample by construction
    def closure_begin(self, attempts, iteration):
        rounds = orc.closure_rounds(self.algo)
        self._clo = (orc.closure_sample_pairs(self.kept, attempts, self.seed, iteration, rounds), int(attempts))
        self._clo_got = []
        self._clo_next = 0
        return max(1, min(rounds, max(int(attempts), 1)))

    def closure_block_sample(self, block, lo, hi, out):
        assert block == self._clo_next, "closure blocks go in order"
        p = self._clo[0][lo:hi].astype(np.int64)
        t = np.arange(lo, hi, dtype=np.int64)
        ok = (p[:, 0] >= 0) & (p[:, 0] != p[:, 1])
        key = (np.minimum(p[:, 0], p[:, 1]) << 32) | np.maximum(p[:, 0], p[:, 1])
        key, t = key[ok], t[ok]
        _, first = np.unique(key, return_index=True)   # one entry per pair: its first attempt
        rows = np.stack([key[first], t[first]], 1).reshape(-1)
        out.numpy()[:rows.size] = rows
        return len(first)

    def closure_block_add(self, block, pairs, count):
        assert block == self._clo_next, "closure blocks go in order"
        if count:
            self._clo_got.append(pairs.numpy()[:2 * count].reshape(-1, 2).copy())
        self._clo_next += 1

    def closure_finish(self):
        attempts = self._clo[1]
        pairs = np.full((max(attempts, 1), 2), -1, np.int32)
        for g in self._clo_got:
            pairs[g[:, 1], 0] = g[:, 0] >> 32
            pairs[g[:, 1], 1] = g[:, 0] & 0xffffffff
        dummy = np.zeros((1, self.g.N), np.int32)
        cu, cv, _, cf = orc.closure_from_pairs(1, self.kept, pairs[:attempts], dummy, 1)
        order = np.lexsort((cv, cu))
        self.cand = (cu[order], cv[order], cf[order])
        return len(cu)

    def closure_partial(self, out):
        cu, cv, _ = self.cand
        out.numpy()[:len(cu)] = (self.lab[:, cu] == self.lab[:, cv]).sum(0)

    def closure_apply(self, algo, n_p, delta, counts, iteration):
        cu, cv, cf = self.cand
        base = np.int64(iteration + 1) << orc.AGE_ITER_SHIFT
        louv = algo in (0, 2)                          # lpm and infomap: weight-0 closure, no repair
        w = counts.numpy()[:len(cu)].astype(np.int32) if (louv and counts is not None) else \
            np.zeros(len(cu), np.int32)
        closure = orc.EdgeGraph(self.g.N, cu, cv, w, base + cf)
        parts = [self.kept, closure]
        if louv:
            deg = self.kept.degrees() + closure.degrees()
            ru, rv, rw, rx = orc.repair(self.g, deg, self.sigma)
            parts.append(orc.EdgeGraph(self.g.N, ru, rv, rw, base + orc.AGE_REPAIR_OFFSET + rx))
        self.g = orc.concat(parts)
        conv, _ = orc.check(self.g.w, n_p, delta)
        return conv, self.g.m

    def get_labels(self, count, renumber=False):
        node_order = self.lab[:, self.sigma]          # [r][t] = label of node t
        return orc.renumber(node_order) if renumber else node_order.copy()

    def get_labels_into(self, out, renumber=False):
        out[...] = self.get_labels(out.shape[0], renumber)
        return out

    def get_graph(self):
        """Node space, canonical and sorted (fc_get_graph)."""
        a, b = self.npos[self.g.u], self.npos[self.g.v]
        u, v = np.minimum(a, b), np.maximum(a, b)
        o = np.lexsort((v, u))
        return u[o], v[o], self.g.w[o], self.g.age[o]
