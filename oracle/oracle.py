"""CPU oracle for the consensus hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import
this module, and only as the checker (or the timed CPU baseline).  The product package
``fastconsensus_amd`` never imports it and has no CPU fallback.

It wraps ``fc_oracle.c`` (a CPU restatement of fast_consensus.py's Louvain/LPM loop,
see that file's header for what is pinned by golden vectors and what is statistical)
and adds a replay driver that re-runs the reference's while-loop
(fast_consensus.py:138-202 louvain, :260-310 lpm) with recorded community-detection
labelings and recorded closure samples.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libfcoracle.so")

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_lib = None

LOUVAIN, LPM, LOUVAIN_NC, LEIDEN, INFOMAP = 0, 1, 2, 3, 4   # LOUVAIN_NC: louvain with new_consensus.py's rule (:155-163)


def _cd_algo(algo):
    """Community-detection algorithm of a loop variant (the new_consensus.py rule runs Louvain)."""
    return algo if algo in (LPM, LEIDEN, INFOMAP) else LOUVAIN
AGE_ITER_SHIFT = 40          # closure/repair edges created in iteration b get ages >= (b+1) << 40
AGE_REPAIR_OFFSET = 1 << 39


def build():
    src = os.path.join(HERE, "fc_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, dbl, u64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_uint64
        L.orc_consensus.argtypes = [ctypes.c_int, i64, _i32p, _i32p, _i32p, ctypes.c_int, i64, _i32p, _i32p]
        L.orc_threshold.argtypes = [i64, _i32p, dbl, ctypes.c_int, _u8p]
        L.orc_threshold.restype = i64
        L.orc_check.argtypes = [i64, _i32p, ctypes.c_void_p, ctypes.c_int, dbl, ctypes.POINTER(i64)]
        L.orc_check.restype = ctypes.c_int
        L.orc_closure_pairs.argtypes = [ctypes.c_int, i64, _i32p, _i32p, i64, _i32p, ctypes.c_int, i64, _i32p,
                                        _i32p, _i32p, _i32p, _i64p]
        L.orc_closure_pairs.restype = i64
        L.orc_adjacency_order.argtypes = [i64, i64, _i32p, _i32p, _i32p, _i64p, ctypes.c_void_p, _i64p, _i32p,
                                          _i32p]
        L.orc_repair.argtypes = [i64, i64, _i32p, _i32p, _i32p, _i64p, ctypes.c_void_p, _i64p, _i32p, _i32p, _i32p,
                                 _i64p]
        L.orc_repair.restype = i64
        L.orc_sort_edges.argtypes = [i64, _i32p, _i32p, _i64p]
        L.orc_louvain_level0.argtypes = [i64, _i64p, _i32p, _i32p, u64, _i32p]
        L.orc_louvain_level0.restype = ctypes.c_int
        L.orc_lpa.argtypes = [i64, _i64p, _i32p, u64, _i32p, ctypes.c_int]
        L.orc_leiden.argtypes = [i64, _i64p, _i32p, ctypes.c_void_p, u64, _i32p]
        L.orc_leiden.restype = ctypes.c_int
        L.orc_infomap.argtypes = [i64, _i64p, _i32p, u64, ctypes.c_int, _i32p]
        L.orc_infomap.restype = ctypes.c_double
        L.orc_lpa.restype = ctypes.c_int
        L.orc_cd_batch.argtypes = [ctypes.c_int, ctypes.c_int, i64, _i64p, _i32p, _i32p, u64, _i32p, _i32p,
                                   ctypes.c_int]
        L.orc_modularity.argtypes = [i64, _i64p, _i32p, ctypes.c_void_p, _i32p]
        L.orc_modularity.restype = dbl
        L.orc_engine_cd.argtypes = [ctypes.c_int, i64, _i64p, _i32p, _i32p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p]
        L.orc_device_sigma.argtypes = [i64, u64, _i32p]
        L.orc_set_lpa_ties.argtypes = [ctypes.c_int]
        L.orc_set_lpa_coarsen.argtypes = [ctypes.c_int]
        L.orc_closure_sample.argtypes = [i64, _i64p, _i32p, i64, u64, ctypes.c_int, ctypes.c_int, _i32p]
        L.orc_build_csr.argtypes = [i64, i64, _i32p, _i32p, ctypes.c_void_p, _i64p, _i32p, _i32p]
        L.orc_infomap_full.argtypes = [i64, _i64p, _i32p, u64, ctypes.c_int, _i32p, ctypes.POINTER(dbl)]
        L.orc_infomap_full.restype = dbl
        L.orc_closure_sequential.argtypes = [i64, i64, _i32p, _i32p, i64, u64, _i32p]
        L.orc_closure_sequential.restype = i64
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


# ----------------------------------------------------------------------------- graph
class EdgeGraph:
    """Canonical undirected edge list: u < v (node-order ids), sorted by (u, v);
    int32 weights; int64 ages (creation order, for networkx adjacency order)."""

    def __init__(self, N, u, v, w, age):
        self.N = int(N)
        self.u, self.v = _c(u, np.int32), _c(v, np.int32)
        self.w, self.age = _c(w, np.int32), _c(age, np.int64)

    @property
    def m(self):
        return len(self.u)

    @staticmethod
    def from_lines(N, pairs):
        """Edge list in file order (ids) -> graph with weights 1 (fast_consensus.py:135-136).
        Self loops dropped; duplicates keep the first line (networkx semantics)."""
        pairs = np.asarray(pairs, np.int64).reshape(-1, 2)
        a, b = pairs[:, 0], pairs[:, 1]
        u, v = np.minimum(a, b), np.maximum(a, b)
        ok = u != v
        line = np.arange(len(pairs), dtype=np.int64)[ok]
        key = (u[ok] << 32) | v[ok]
        order = np.lexsort((line, key))
        key, line = key[order], line[order]
        first = np.ones(len(key), bool)
        first[1:] = key[1:] != key[:-1]
        key, line = key[first], line[first]
        return EdgeGraph(N, key >> 32, key & 0xFFFFFFFF, np.ones(len(key), np.int32), line)

    def sorted_by_key(self):
        perm = np.empty(self.m, np.int64)
        lib().orc_sort_edges(self.m, self.u, self.v, perm)
        return EdgeGraph(self.N, self.u[perm], self.v[perm], self.w[perm], self.age[perm])

    def subset(self, mask):
        return EdgeGraph(self.N, self.u[mask], self.v[mask], self.w[mask], self.age[mask])

    def csr(self):
        rowptr = np.empty(self.N + 1, np.int64)
        col = np.empty(2 * self.m, np.int32)
        cw = np.empty(2 * self.m, np.int32)
        lib().orc_build_csr(self.N, self.m, self.u, self.v, self.w.ctypes.data, rowptr, col, cw)
        return rowptr, col, cw

    def adjacency_order(self):
        ptr = np.empty(self.N + 1, np.int64)
        nbr = np.empty(2 * self.m, np.int32)
        nw = np.empty(2 * self.m, np.int32)
        lib().orc_adjacency_order(self.N, self.m, self.u, self.v, self.w, self.age, None, ptr, nbr, nw)
        return ptr, nbr, nw

    def degrees(self):
        return (np.bincount(self.u, minlength=self.N) + np.bincount(self.v, minlength=self.N)).astype(np.int64)

    def as_dict(self):
        return {(int(a), int(b)): int(c) for a, b, c in zip(self.u, self.v, self.w)}


def concat(graphs):
    N = graphs[0].N
    g = EdgeGraph(N, np.concatenate([x.u for x in graphs]), np.concatenate([x.v for x in graphs]),
                  np.concatenate([x.w for x in graphs]), np.concatenate([x.age for x in graphs]))
    return g.sorted_by_key()


# ----------------------------------------------------------------------------- steps
def consensus(algo, g, labels, n_p):
    labels = _c(labels, np.int32)
    assert labels.shape == (n_p, g.N)
    out = np.empty(g.m, np.int32)
    lib().orc_consensus(algo, g.m, g.u, g.v, g.w, n_p, g.N, labels, out)
    return out


def threshold(w, tau, n_p):
    keep = np.empty(len(w), np.uint8)
    lib().orc_threshold(len(w), _c(w, np.int32), float(tau), n_p, keep)
    return keep.astype(bool)


def check(w, n_p, delta):
    cnt = ctypes.c_int64()
    w = _c(w, np.int32)
    res = lib().orc_check(len(w), w, None, n_p, float(delta), ctypes.byref(cnt))
    return bool(res), int(cnt.value)


def closure_from_pairs(algo, g, pairs, labels, n_p):
    pairs = _c(pairs, np.int32).reshape(-1, 2)
    P = len(pairs)
    ou, ov, ow = (np.empty(max(P, 1), np.int32) for _ in range(3))
    of = np.empty(max(P, 1), np.int64)
    labels = _c(labels, np.int32)
    k = lib().orc_closure_pairs(_cd_algo(algo), g.m, g.u, g.v, P, pairs.reshape(-1), n_p, g.N, labels, ou, ov, ow,
                                of)
    return ou[:k].copy(), ov[:k].copy(), ow[:k].copy(), of[:k].copy()


# the engine's default closure blocks per algorithm (fc_ctx.h CLOSURE_ROUNDS_LOUVAIN / _LPM,
# FC_OPT_CLOSURE_ROUNDS = 0): louvain loops 4, lpm / infomap loops 16
CLOSURE_ROUNDS_LOUVAIN, CLOSURE_ROUNDS_LPM = 4, 16


def closure_rounds(algo):
    return CLOSURE_ROUNDS_LOUVAIN if algo in (LOUVAIN, LOUVAIN_NC) else CLOSURE_ROUNDS_LPM


def closure_sample_pairs(kept, attempts, seed, iteration, rounds=CLOSURE_ROUNDS_LOUVAIN):
    """Engine's device sampler, restated: the (a, b) pair of every attempt (or (-1, -1)), the
    attempts in `rounds` blocks, each drawing from the kept graph plus the earlier blocks'
    closure edges (orc_closure_sample)."""
    rowptr, col, _ = kept.csr()
    pairs = np.empty((max(int(attempts), 1), 2), np.int32)
    lib().orc_closure_sample(kept.N, rowptr, col, int(attempts), int(seed) & (2**64 - 1), int(iteration),
                             int(rounds), pairs)
    return pairs[:attempts]


def closure_sequential_pairs(kept, attempts, seed):
    """The reference's own closure loop (fast_consensus.py:175-184, :292-300): attempts one
    after the other on the growing graph; returns the pairs it added, in attempt order
    (orc_closure_sequential; the oracle's RNG, the reference's distribution)."""
    out = np.empty((max(int(attempts), 1), 2), np.int32)
    k = lib().orc_closure_sequential(kept.N, kept.m, kept.u, kept.v, int(attempts), int(seed) & (2**64 - 1), out)
    return out[:k].copy()


def refsem_run(algo, g0, n_p, tau, delta, seed, nthreads=0, max_iters=100):
    """The reference while-loop and final pass (fast_consensus.py:129-202 louvain, :260-310
    lpm, :383-392) with the oracle's sequential CD restatements (python-louvain level 0 /
    igraph LPA, one fresh stream per batch) and the SEQUENTIAL closure over the growing graph:
    the reference's semantics at sizes where running the reference script itself is infeasible
    (its np.random.choice(nodes) closure is O(L*N) per iteration).  Every step but the CD and the
    closure's RNG is the golden-pinned replay (`iterate`).  Returns (final labels [n_p][N],
    iterations)."""
    graph = g0
    L = g0.m                                        # L = G.number_of_edges(), :132/:144
    for it in range(max_iters):
        lab, _ = cd_batch(algo, n_p, graph, seed=seed * 1000003 + it, nthreads=nthreads)
        w_new = consensus(algo, graph, lab, n_p)
        keep = threshold(w_new, tau, n_p)
        kept = EdgeGraph(graph.N, graph.u[keep], graph.v[keep], w_new[keep], graph.age[keep])
        pairs = None
        if algo != LPM and check(kept.w, n_p, delta)[0]:
            break                                   # check #1: final pass on the old graph
        pairs = closure_sequential_pairs(kept, L, seed * 7919 + it)
        new, tr = iterate(algo, graph, lab, pairs, n_p, tau, delta, it)
        graph = new
        if tr["check2"][0]:
            break
    lab, _ = cd_batch(algo, n_p, graph, seed=seed * 1000003 + 999, nthreads=nthreads)
    return lab, it + 1


def repair(old, deg, sigma=None):
    """deg: int64 degrees of nextgraph after closure (updated in place).  sigma: node
    position -> id when ids are an internal numbering (visit and tie-break in node order);
    the returned x are node positions."""
    k_max = old.N
    ou, ov, ow = (np.empty(max(k_max, 1), np.int32) for _ in range(3))
    ox = np.empty(max(k_max, 1), np.int64)
    sg = None if sigma is None else np.ascontiguousarray(sigma, dtype=np.int32)
    k = lib().orc_repair(old.N, old.m, old.u, old.v, old.w, old.age, None if sg is None else sg.ctypes.data, deg,
                         ou, ov, ow, ox)
    return ou[:k].copy(), ov[:k].copy(), ow[:k].copy(), ox[:k].copy()


def cd_batch(algo, n_r, g, seed, nthreads=0):
    rowptr, col, cw = g.csr()
    lab = np.empty((n_r, g.N), np.int32)
    sw = np.empty(n_r, np.int32)
    lib().orc_cd_batch(_cd_algo(algo), n_r, g.N, rowptr, col, cw, int(seed) & (2**64 - 1), lab, sw, int(nthreads))
    return lab, sw


def infomap(g, seed, trials=10):
    """One restated igraph Infomap run (unweighted topology, fast_consensus.py:268); returns
    (labels, codelength in bits)."""
    rowptr, col, _ = g.csr()
    lab = np.empty(g.N, np.int32)
    L = lib().orc_infomap(g.N, rowptr, col, int(seed) & (2**64 - 1), int(trials), lab)
    return lab, L


def infomap_full(g, seed, trials=10):
    """igraph's infomap_partition outer loop (single-node and sub-module re-partition rounds)
    around the same greedy core (orc_infomap_full).  Returns (labels, codelength, the core-only
    codelength of the same trials)."""
    rowptr, col, _ = g.csr()
    lab = np.empty(g.N, np.int32)
    core = ctypes.c_double()
    L = lib().orc_infomap_full(g.N, rowptr, col, int(seed) & (2**64 - 1), int(trials), lab, ctypes.byref(core))
    return lab, L, core.value


DENSE_DIV = 0   # the engine's default (fc_ctx.h dense_div, FC_OPT_DENSE_DIV)
# the engine's default buckets per sweep (fc_ctx.h cd_buckets): Louvain 16, LPA 32
BUCKETS_LOUVAIN, BUCKETS_LPA = 16, 32


def cd_buckets(algo, buckets=None):
    if buckets:
        return int(buckets)
    return BUCKETS_LOUVAIN if algo in (LOUVAIN, LOUVAIN_NC) else BUCKETS_LPA


def device_sigma(n, seed):
    """The engine's internal vertex numbering for a seed (graph.hip k_sigma, relabel on)."""
    out = np.empty(max(int(n), 1), np.int32)
    lib().orc_device_sigma(int(n), int(seed) & (2**64 - 1), out)
    return out[:n]


def engine_cd(algo, g, n_r, rbase, iteration, seed, buckets=None, max_sweeps=200, chunk=16, prune=1, coarsen=8,
              prune_mark=1, shared=2, dense_div=DENSE_DIV):
    """CPU twin of the engine's bucketed CD (bit-exact target for the HIP kernels).  Defaults = the
    default engine (fc_ctx.h): the hybrid, FC_OPT_CD_ENGINE=2, shared=2 (a replica's full sweeps
    in the batch's shared order, its filtered sweeps in its own).  The classic engine (cd.hip
    alone, FC_OPT_CD_ENGINE=0) is shared=0; the replica-lane engine (FC_OPT_CD_ENGINE=1, cd_rl.hip)
    is shared=1 (one visit order shared by every replica in every sweep), coarsen=0."""
    rowptr, col, cw = g.csr()
    lab = np.empty((n_r, g.N), np.int32)
    sw = np.empty(n_r, np.int32)
    buckets = cd_buckets(algo, buckets)
    lib().orc_engine_cd(_cd_algo(algo), g.N, rowptr, col, cw, n_r, rbase, iteration, int(seed) & (2**64 - 1), buckets,
                        max_sweeps, chunk, prune, coarsen, prune_mark, shared, dense_div, lab, sw)
    return lab, sw


def renumber(labels):
    """Community ids -> 0..k-1 by first node (engine's output convention)."""
    out = np.empty_like(labels)
    for r, lab in enumerate(labels):
        _, first, inv = np.unique(lab, return_index=True, return_inverse=True)
        order = np.argsort(first)
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        out[r] = rank[inv]
    return out


def modularity(g, labels, weighted=True):
    rowptr, col, cw = g.csr()
    return lib().orc_modularity(g.N, rowptr, col, cw.ctypes.data if weighted else None,
                                _c(labels, np.int32))


# ----------------------------------------------------------------------------- replay
def iterate(algo, graph, labels, pairs, n_p, tau, delta, it):
    """One iteration of the reference while-loop with given labelings and closure
    samples.  Returns (new_graph or None, trace) where None means "break at check #1"
    (louvain: final pass runs on the old graph, fast_consensus.py:172-173)."""
    trace = {}
    w_new = consensus(algo, graph, labels, n_p)
    keep = threshold(w_new, tau, n_p)
    kept = EdgeGraph(graph.N, graph.u[keep], graph.v[keep], w_new[keep], graph.age[keep])
    trace["consensus_w"] = w_new
    trace["keep"] = keep
    trace["kept"] = kept
    base = np.int64(it + 1) << AGE_ITER_SHIFT
    if algo != LPM:
        conv1, cnt1 = check(kept.w, n_p, delta)
        trace["check1"] = (conv1, cnt1)
        if conv1:
            return None, trace
    cu, cv, cw, cf = closure_from_pairs(algo, kept, pairs, labels, n_p)
    closure = EdgeGraph(graph.N, cu, cv, cw, base + cf)
    trace["closure"] = closure
    parts = [kept, closure]
    if algo != LPM:
        deg = kept.degrees() + closure.degrees()
        ru, rv, rw, rx = repair(graph, deg)
        rep = EdgeGraph(graph.N, ru, rv, rw, base + AGE_REPAIR_OFFSET + rx)
        trace["repair"] = rep
        parts.append(rep)
    new = concat(parts)
    conv2, cnt2 = check(new.w, n_p, delta)
    trace["check2"] = (conv2, cnt2)
    return new, trace


def replay(algo, N, edge_lines, n_p, tau, delta, cd_batches, pair_batches, max_iters=1000):
    """Run the reference loop with recorded labelings (cd_batches[b] is [n_p][N]) and
    closure samples (pair_batches[b]).  Returns (graphs_at_batch_start, traces,
    final_batch_index)."""
    graph = EdgeGraph.from_lines(N, edge_lines)
    graphs, traces = [graph], []
    for it in range(max_iters):
        new, tr = iterate(algo, graph, cd_batches[it], pair_batches[it] if it < len(pair_batches) else
                          np.zeros((0, 2), np.int32), n_p, tau, delta, it)
        traces.append(tr)
        if new is None:                      # louvain check #1 break: keep old graph
            graphs.append(graph)
            return graphs, traces, it + 1
        graph = new
        graphs.append(graph)
        if tr["check2"][0]:
            return graphs, traces, it + 1
    raise RuntimeError("replay did not converge")
