"""Host side of the engine: the drop-in ``fast_consensus()`` and a thin ``Engine`` over
the C-ABI.  Mirrors fast_consensus.py:129-411 (same names, argument meaning, defaults
and return types); all compute runs in the HIP library.
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import (FC_ALGO_INFOMAP, FC_ALGO_LEIDEN, FC_ALGO_LOUVAIN, FC_ALGO_LOUVAIN_NC, FC_ALGO_LPM,
                   FastConsensusError, Stats, check, ptr)

ALGORITHMS = {"louvain": FC_ALGO_LOUVAIN, "lpm": FC_ALGO_LPM, "leiden": FC_ALGO_LEIDEN, "infomap": FC_ALGO_INFOMAP}
# consensus weight rules: fast_consensus.py (the named entry point) or the new_consensus.py
# fork's plain count that keeps converged edges (:155-163); louvain only
RULES = ("fast_consensus", "new_consensus")
OUT_OF_SCOPE = ("cnm",)
FINAL_PASS_ITER = 0x40000000  # iteration salt of the final pass (matches capi.cpp fc_run)


def torch_int32():
    import torch
    return torch.int32


def torch_int64():
    import torch
    return torch.int64


def algo_id(algorithm):
    if algorithm in ALGORITHMS:
        return ALGORITHMS[algorithm]
    if algorithm in OUT_OF_SCOPE:
        raise NotImplementedError("algorithm %r is outside this engine's scope (louvain, lpm, leiden and infomap only)"
                                  % algorithm)
    return None


class PinnedHost:
    """Page-locks (hipHostRegister) a caller-owned host array that the engine downloads labelings
    into (Engine.run(out=...), run_sharded(out=...)): the device -> host copy then runs as one
    direct DMA instead of being staged through the runtime's pinned bounce buffers.  A caller that
    keeps one output array pins it once, next to allocating it.  `ok` is False (and nothing is
    pinned) when the runtime refuses.  release() before the array is freed."""

    def __init__(self, array):
        import torch
        self._rt = torch._C._cudart
        self._ptr, self._n = int(array.ctypes.data), int(array.nbytes)
        self.ok = self._n > 0 and int(self._rt.cudaHostRegister(self._ptr, self._n, 0)) == 0

    def release(self):
        if self.ok:
            self._rt.cudaHostUnregister(self._ptr)
            self.ok = False


class Engine:
    """One device-resident consensus engine (one GPU, one host thread)."""

    def __init__(self, device=0, seed=None):
        L = _lib.load()
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")  # the reference is unseeded
        self.seed = int(seed) & (2 ** 64 - 1)
        self._ctx = ctypes.c_void_p()
        check(L.fc_create(int(device), self.seed, ctypes.byref(self._ctx)))
        self._L = L
        self.device = device

    # -- lifecycle ---------------------------------------------------------------
    def close(self):
        if self._ctx:
            self._L.fc_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_handle):
        check(self._L.fc_set_stream(self._ctx, stream_handle))
        self._shared_stream = stream_handle is not None

    def _dev(self, t):
        """Address of a caller device buffer.  Unless the engine runs on the caller's stream
        (set_stream), the work queued on that buffer by torch (e.g. the zero fill of
        torch.zeros) is drained first: the engine's own stream is not ordered after it."""
        if t is not None and not getattr(self, "_shared_stream", False) and hasattr(t, "is_cuda") and t.is_cuda:
            import torch
            torch.cuda.current_stream(t.device).synchronize()
        return ptr(t)

    def _written(self):
        """After a step that wrote a caller device buffer: unless the engine runs on the
        caller's stream, wait for it, so that torch may read the buffer on its own stream."""
        if not getattr(self, "_shared_stream", False):
            check(self._L.fc_synchronize(self._ctx))

    def set_timing(self, on=True):
        check(self._L.fc_set_timing(self._ctx, 1 if on else 0))

    def collect_timing(self):
        st = Stats()
        check(self._L.fc_collect_timing(self._ctx, ctypes.byref(st)))
        return st.as_dict()

    def set_params(self, buckets=0, max_sweeps=0, max_iters=0):
        check(self._L.fc_set_params(self._ctx, int(buckets), int(max_sweeps), int(max_iters)))

    def set_option(self, name, value):
        if name == "seed":
            value = int(value) & (2 ** 64 - 1)
            self.seed = value
            value = value - 2 ** 64 if value >= 2 ** 63 else value   # int64_t on the C side
        check(self._L.fc_set_option(self._ctx, _lib.OPTIONS[name], int(value)))

    # -- graph -----------------------------------------------------------------------
    def load_graph(self, n, u, v):
        u = np.ascontiguousarray(u, dtype=np.int32)
        v = np.ascontiguousarray(v, dtype=np.int32)
        assert u.shape == v.shape
        check(self._L.fc_load_graph(self._ctx, int(n), len(u), u, v))

    def node_map(self):
        """sigma[node id] = the engine's internal vertex id."""
        out = np.empty(self.n, np.int32)
        check(self._L.fc_get_node_map(self._ctx, out))
        return out

    def reset_graph(self):
        check(self._L.fc_reset_graph(self._ctx))

    def graph_info(self):
        n, m, m0 = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self._L.fc_graph_info(self._ctx, ctypes.byref(n), ctypes.byref(m), ctypes.byref(m0)))
        return n.value, m.value, m0.value

    @property
    def n(self):
        return self.graph_info()[0]

    @property
    def m(self):
        return self.graph_info()[1]

    def get_graph(self):
        _, m, _ = self.graph_info()
        u = np.empty(m, np.int32)
        v = np.empty(m, np.int32)
        w = np.empty(m, np.int32)
        age = np.empty(m, np.int64)
        check(self._L.fc_get_graph(self._ctx, ptr(u), ptr(v), ptr(w), ptr(age)))
        return u, v, w, age

    def get_nextgraph(self):
        m = ctypes.c_int64()
        check(self._L.fc_get_nextgraph(self._ctx, ctypes.byref(m), None, None, None, None))
        u, v, w = (np.empty(m.value, np.int32) for _ in range(3))
        age = np.empty(m.value, np.int64)
        check(self._L.fc_get_nextgraph(self._ctx, ctypes.byref(m), ptr(u), ptr(v), ptr(w), ptr(age)))
        return u, v, w, age

    # -- one-shot driver ------------------------------------------------------------------
    def run(self, algo, n_p, tau, delta, out=None):
        """Whole fast_consensus run; returns ([n_p][n] int32 labelings, stats).  `out`: an
        optional C-contiguous int32 host array of that shape to write into (a caller that runs
        repeatedly keeps one: a fresh 256 MB array costs ~20 ms of OS page zeroing on first
        touch, more than the PCIe download itself)."""
        n = self.n
        if out is None:
            labels = np.empty((n_p, n), np.int32)
        else:
            if not (isinstance(out, np.ndarray) and out.dtype == np.int32 and out.shape == (n_p, n)
                    and out.flags.c_contiguous):
                raise ValueError("out must be a C-contiguous int32 array of shape (n_p, n)")
            labels = out
        st = Stats()
        check(self._L.fc_run(self._ctx, int(algo), int(n_p), float(tau), float(delta), ptr(labels),
                             ctypes.byref(st)))
        return labels, st.as_dict()

    # -- step API (distributed driver, replay) ------------------------------------------
    def cd(self, algo, rbegin, rcount, n_p_total, iteration):
        check(self._L.fc_cd(self._ctx, int(algo), int(rbegin), int(rcount), int(n_p_total), int(iteration)))

    def set_labels(self, labels):
        """Install host labelings [count][n] (node order).  Any integer community ids are
        accepted: a row with ids outside [0, n) (1-based memberships, sparse or negative ids)
        is compacted first -- ids only matter through equality (fc_set_labels requires
        [0, n))."""
        labels = np.asarray(labels)
        if labels.ndim != 2 or labels.shape[1] != self.n:
            raise ValueError("labelings must have shape (count, %d)" % self.n)
        if labels.size and (labels.min() < 0 or labels.max() >= self.n):
            labels = np.stack([np.unique(row, return_inverse=True)[1].reshape(-1) for row in labels])
        labels = np.ascontiguousarray(labels, dtype=np.int32)
        check(self._L.fc_set_labels(self._ctx, labels.shape[0], labels))

    def replica_info(self):
        """(local replica count, first global replica index, n_p of the run)."""
        n, b, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._L.fc_replica_info(self._ctx, ctypes.byref(n), ctypes.byref(b), ctypes.byref(t)))
        return n.value, b.value, t.value

    def _check_count(self, count):
        n_r = self.replica_info()[0]
        if count != n_r:
            raise ValueError("the engine holds %d local labelings, %d requested" % (n_r, count))

    def get_labels(self, count, renumber=False, dev_out=None):
        """[count][n] labelings in node order (count must equal the local replica count): a
        new numpy array, or written into the device tensor `dev_out` (int32, >= count*n
        elements) when given."""
        self._check_count(count)
        if dev_out is not None:
            if dev_out.dtype != torch_int32() or dev_out.numel() < count * self.n:
                raise ValueError("dev_out must be an int32 tensor of >= %d elements" % (count * self.n))
            check(self._L.fc_get_labels(self._ctx, self._dev(dev_out), int(dev_out.numel()), 1 if renumber else 0))
            return dev_out
        out = np.empty((count, self.n), np.int32)
        check(self._L.fc_get_labels(self._ctx, ptr(out), out.size, 1 if renumber else 0))
        return out

    def get_labels_into(self, out, renumber=False):
        """Like get_labels(out.shape[0], ...) into a caller-owned C-contiguous int32 host array."""
        if not (isinstance(out, np.ndarray) and out.dtype == np.int32 and out.ndim == 2 and out.shape[1] == self.n
                and out.flags.c_contiguous):
            raise ValueError("out must be a C-contiguous int32 array of shape (count, %d)" % self.n)
        self._check_count(out.shape[0])
        check(self._L.fc_get_labels(self._ctx, ptr(out), out.size, 1 if renumber else 0))
        return out

    def consensus_partial(self, algo, dev_out):
        check(self._L.fc_consensus_partial(self._ctx, int(algo), self._dev(dev_out)))
        self._written()

    def consensus_apply(self, algo, n_p, tau, delta, dev_partial):
        conv, kept, unc = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
        check(self._L.fc_consensus_apply(self._ctx, int(algo), int(n_p), float(tau), float(delta),
                                         self._dev(dev_partial), ctypes.byref(conv), ctypes.byref(kept),
                                         ctypes.byref(unc)))
        return bool(conv.value), kept.value, unc.value

    def closure_sample(self, attempts, iteration):
        nc = ctypes.c_int64()
        check(self._L.fc_closure_sample(self._ctx, int(attempts), int(iteration), ctypes.byref(nc)))
        return nc.value

    # sharded closure (distributed.py, world > 1): same candidates as closure_sample
    def closure_begin(self, attempts, iteration):
        """Returns the number of closure blocks; block b covers attempts
        [attempts*b//blocks, attempts*(b+1)//blocks)."""
        nb = ctypes.c_int()
        check(self._L.fc_closure_begin(self._ctx, int(attempts), int(iteration), ctypes.byref(nb)))
        return nb.value

    def closure_block_sample(self, block, t_lo, t_hi, dev_out):
        """Draws attempts [t_lo, t_hi) of `block` into dev_out (int64 tensor, (key, first
        attempt) pairs); returns the number of pairs."""
        if dev_out.dtype != torch_int64() or dev_out.numel() < 2 * max(t_hi - t_lo, 0):
            raise ValueError("dev_out must be an int64 tensor of >= %d elements" % (2 * (t_hi - t_lo)))
        k = ctypes.c_int64()
        check(self._L.fc_closure_block_sample(self._ctx, int(block), int(t_lo), int(t_hi), self._dev(dev_out),
                                              int(dev_out.numel() // 2), ctypes.byref(k)))
        self._written()
        return k.value

    def closure_block_add(self, block, dev_in, count):
        check(self._L.fc_closure_block_add(self._ctx, int(block), self._dev(dev_in) if count else None, int(count)))

    def closure_finish(self):
        nc = ctypes.c_int64()
        check(self._L.fc_closure_finish(self._ctx, ctypes.byref(nc)))
        return nc.value

    def closure_set_pairs(self, pairs, iteration):
        pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        nc = ctypes.c_int64()
        check(self._L.fc_closure_set_pairs(self._ctx, len(pairs), ptr(pairs), int(iteration), ctypes.byref(nc)))
        return nc.value

    def closure_partial(self, dev_out):
        check(self._L.fc_closure_partial(self._ctx, self._dev(dev_out)))
        self._written()

    def closure_apply(self, algo, n_p, delta, dev_counts, iteration):
        conv, m = ctypes.c_int(), ctypes.c_int64()
        check(self._L.fc_closure_apply(self._ctx, int(algo), int(n_p), float(delta), self._dev(dev_counts),
                                       int(iteration), ctypes.byref(conv), ctypes.byref(m)))
        return bool(conv.value), m.value


# ------------------------------------------------------------------------------------ inputs
ADJ_PARALLEL_MIN = 4_000_000     # adjacency entries from which read_adjacency forks workers


def host_workers():
    """Worker processes for the host conversion: FC_HOST_WORKERS, else min(8, the CPUs this
    process may run on)."""
    env = os.environ.get("FC_HOST_WORKERS")
    if env is not None:
        return max(1, int(env))
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 1
    return max(1, min(8, cpus))


ADJ_DEADLINE_S = 30.0            # forked read: workers still running after this (+0.2 us per entry) are killed


def _fork_safe():
    """The forked read runs only in a process with no other Python thread (a thread could hold
    an interpreter-level lock -- import, logging, a user lock -- that a child would wait on
    forever) and when FC_HOST_FORK is not 0.  Native runtime threads (a HIP runtime started by
    an earlier Engine) do not block it: the children run dict iteration and numpy only (the
    interpreter's allocator under the GIL, glibc malloc, which resets its locks at fork), never
    touch the GPU and leave through os._exit; the deadline in _reap covers the rest."""
    import threading
    return os.environ.get("FC_HOST_FORK", "1") != "0" and threading.active_count() == 1


def _reap(pids, deadline):
    """Wait for the forked workers with WNOHANG polling until `deadline` (time.monotonic());
    past it the rest are killed and reaped.  True iff every worker exited with status 0."""
    import signal
    import time
    ok, left = True, list(pids)
    while left:
        for pid in list(left):
            done, status = os.waitpid(pid, os.WNOHANG)
            if done:
                left.remove(pid)
                ok = ok and status == 0
        if left and time.monotonic() > deadline:
            for pid in left:
                try:
                    os.kill(pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                os.waitpid(pid, 0)
            return False
        if left:
            time.sleep(0.002)
    return ok


def read_adjacency(rows, lens, key=None):
    """The keys of the dicts `rows` (row i has lens[i] keys), concatenated into int64, each
    through `key` when given.  Reading 27.5 M dict keys is CPython-bound (~0.1 us per key, most
    of it a cache miss on the key object), so large adjacencies are read by forked workers,
    each chaining a contiguous range of rows into a shared anonymous mapping (no pickling: the
    children see the parent's dicts copy-on-write).  Any worker failure, or workers still
    running at the deadline (killed), falls back to the serial read; a process with other
    Python threads reads serially (_fork_safe)."""
    import itertools
    tot = int(lens.sum())
    W = host_workers() if hasattr(os, "fork") else 1

    def serial(lo, hi, cnt):
        it = itertools.chain.from_iterable(rows[lo:hi])
        return np.fromiter(it if key is None else map(key, it), np.int64, count=cnt)

    if W <= 1 or tot < ADJ_PARALLEL_MIN or not _fork_safe():
        return serial(0, len(rows), tot)
    import mmap
    import time
    off = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    cut = np.searchsorted(off, np.linspace(0, tot, W + 1).astype(np.int64))
    cut[0], cut[-1] = 0, len(rows)
    buf = mmap.mmap(-1, tot * 8)                   # MAP_SHARED | MAP_ANONYMOUS: children write it
    flat = np.frombuffer(buf, np.int64)
    pids = []
    try:
        for w in range(W):
            lo, hi = int(cut[w]), int(cut[w + 1])
            if hi <= lo:
                continue
            pid = os.fork()
            if pid == 0:                               # child: fill its range, leave without cleanup
                code = 1
                try:
                    flat[off[lo]:off[hi]] = serial(lo, hi, int(off[hi] - off[lo]))
                    code = 0
                finally:
                    os._exit(code)
            pids.append(pid)
    finally:
        ok = _reap(pids, time.monotonic() + ADJ_DEADLINE_S + tot * 2e-7)
    if len(pids) == 0 or not ok:
        del flat
        buf.close()
        return serial(0, len(rows), tot)
    out = flat.copy()
    del flat
    buf.close()
    return out


class IdGraph:
    """A graph in engine form: node labels in node order + edges as node-order ids, in an
    order whose per-node first occurrences reproduce networkx adjacency order."""

    def __init__(self, labels, u, v):
        lab = np.asarray(labels)
        if lab.ndim != 1:      # tuple nodes (grid graphs ...): one object per node, not a 2-D array
            lab = np.fromiter(labels, dtype=object, count=len(labels))
        self.labels = lab
        self.u = np.ascontiguousarray(u, dtype=np.int32)
        self.v = np.ascontiguousarray(v, dtype=np.int32)

    @property
    def n(self):
        return len(self.labels)

    @staticmethod
    def from_networkx(G):
        """Node order = G.nodes(); for each node x, its later neighbours are emitted in
        G.adj[x] order (that is the order G.copy() keeps, fast_consensus.py:131).  The
        adjacency is read at C speed (dict keys chained into numpy) and mapped to indices by a
        lookup array when the nodes are small non-negative integers (by a dict otherwise).
        Past ADJ_PARALLEL_MIN adjacency entries the read is split over forked workers
        (read_adjacency)."""
        if G.is_directed():
            raise TypeError("fast_consensus needs an undirected graph")
        nodes = list(G.nodes())
        n = len(nodes)
        adj = getattr(G, "_adj", None)
        rows = list(adj.values()) if isinstance(adj, dict) and len(adj) == n else None
        if rows is None or (n and (next(iter(adj)) != nodes[0] or list(adj) != nodes)):
            rows = [G.adj[x] for x in nodes]        # adjacency not keyed in node order: per node
        lens = np.fromiter(map(len, rows), np.int64, count=n)
        if n and all(type(x) is int for x in nodes[:1]) and all(isinstance(x, (int, np.integer)) for x in nodes) \
                and min(nodes) >= 0 and max(nodes) < 4 * n + 1024:
            lut = np.full(max(nodes) + 1, -1, np.int64)
            lut[np.asarray(nodes, np.int64)] = np.arange(n, dtype=np.int64)
            nbr = lut[read_adjacency(rows, lens)]
        else:
            idx = {x: i for i, x in enumerate(nodes)}
            nbr = read_adjacency(rows, lens, idx.__getitem__)
        src = np.repeat(np.arange(n, dtype=np.int64), lens)
        keep = nbr > src
        return IdGraph(nodes, src[keep].astype(np.int32), nbr[keep].astype(np.int32))

    @staticmethod
    def from_edgelist_file(path):
        """Native parser (nx.read_edgelist(path, nodetype=int) semantics, :434)."""
        L = _lib.load()
        n, m = ctypes.c_int64(), ctypes.c_int64()
        check(L.fc_read_edgelist(path.encode(), ctypes.byref(n), ctypes.byref(m), None, None, None))
        labels = np.empty(n.value, np.int64)
        u = np.empty(m.value, np.int32)
        v = np.empty(m.value, np.int32)
        check(L.fc_read_edgelist(path.encode(), ctypes.byref(n), ctypes.byref(m), ptr(labels), ptr(u), ptr(v)))
        return IdGraph(labels, u, v)


class Cover:
    """What ``leidenalg.find_partition(...).as_cover()`` returns (fast_consensus.py:123), as far
    as the reference uses it: iterating yields the clusters (lists of igraph vertex ids,
    ascending), ``membership[j]`` is ``[cluster of vertex j]`` (:465-466) and ``len`` is the
    number of clusters.  igraph vertex j is the j-th smallest node label (``nx_to_igraph``
    adds ``sorted(G.nodes())``, :47).  Clusters are numbered by decreasing size, as leidenalg
    renumbers its communities (ties: the cluster holding the smaller vertex first).  Parity
    unpinned: leidenalg is absent here, so this numbering (and the Leiden/Infomap partitions
    themselves) are checked only against the restatement in oracle/fc_oracle.c."""

    def __init__(self, vertex_labels):
        lab = np.asarray(vertex_labels)
        k = int(lab.max()) + 1 if lab.size else 0
        sizes = np.bincount(lab, minlength=k)
        first = np.full(k, lab.size, np.int64)
        np.minimum.at(first, lab, np.arange(lab.size))
        order = np.lexsort((first, -sizes))
        rank = np.empty(k, np.int64)
        rank[order] = np.arange(k)
        self._m = rank[lab] if lab.size else lab.astype(np.int64)
        self._k = k

    def __len__(self):
        return self._k

    def __iter__(self):
        idx = np.argsort(self._m, kind="stable")
        bounds = np.searchsorted(self._m[idx], np.arange(self._k + 1))
        for c in range(self._k):
            yield idx[bounds[c]:bounds[c + 1]].tolist()

    def __getitem__(self, c):
        return np.flatnonzero(self._m == c).tolist()

    @property
    def membership(self):
        return [[int(c)] for c in self._m]

    def sizes(self):
        return np.bincount(self._m, minlength=self._k).tolist()


def labels_to_output(algorithm, node_labels, labels):
    """Engine labelings [n_p][N] -> the reference's return type (fast_consensus.py:383-392):
    louvain: list of dict node -> community (insertion order = node order, as
    python-louvain builds it); lpm and infomap: list of set of frozenset of nodes; leiden:
    list of ``Cover`` (igraph vertex ids, :385-388)."""
    out = []
    nodes = list(node_labels.tolist())
    if algorithm == "leiden":
        vid = np.argsort(np.argsort(np.asarray(node_labels), kind="stable"), kind="stable")   # node -> vertex id
        for lab in labels:
            vl = np.empty(len(lab), np.int64)
            vl[vid] = lab
            out.append(Cover(vl))
        return out
    na = np.asarray(node_labels)
    # louvain: each dict is a copy of one key template (no rehashing as it grows), then its
    # values are set in node order -- ~10 % less than dict(zip(...)) per 1M-entry labeling
    tmpl = dict.fromkeys(nodes) if algorithm == "louvain" else None
    for lab in labels:
        if algorithm == "louvain":
            d = tmpl.copy()
            d.update(zip(nodes, lab.tolist()))
            out.append(d)
        else:
            # the communities as runs of one stable sort by label (C speed; a frozenset per run)
            lab = np.asarray(lab)
            order = np.argsort(lab, kind="stable")
            sl = lab[order]
            b = [0] + (np.flatnonzero(sl[1:] != sl[:-1]) + 1).tolist() + [len(sl)]
            srt = na[order].tolist()
            out.append({frozenset(srt[b[i]:b[i + 1]]) for i in range(len(b) - 1)} if len(sl) else set())
    return out


def store_order_pays(replicas, algorithm=None, cd_engine=0):
    """Label storage order (FC_OPT_STORE) for a GPU that will hold `replicas` replicas: the
    one-replica ordering pass at load costs ~4 ms on LFR-1M and saves gather misses of the
    classic CD engine (the default) in proportion to the replicas (measured: n_p=8 61.7 ms
    without vs 63.0 with, n_p=16 89.0 vs 87.0, n_p=64 saves ~20 ms).  The replica-lane engine
    (cd_engine=1) reads labels node-major and gains nothing from it for louvain / lpm."""
    if cd_engine == 1 and algorithm in (FC_ALGO_LOUVAIN, FC_ALGO_LPM, FC_ALGO_LOUVAIN_NC, "louvain", "lpm"):
        return 0
    return 1 if replicas >= 12 else 0


def relabel_for(algorithm):
    """FC_OPT_RELABEL for a run of `algorithm`: infomap's union levels gather neighbour state by
    internal id and assign buckets by a hash of it, so a community-ordered numbering (2) puts
    a vertex's in-community neighbours on shared lines (LFR-100k infomap 1.56 -> 1.46 s per
    call, same output; profiles/r06_ab.txt); every other algorithm keeps the random numbering
    (1) its chunked visit orders need."""
    return 2 if algorithm in (FC_ALGO_INFOMAP, "infomap") else 1


def fast_consensus(G, algorithm='louvain', n_p=20, thresh=0.2, delta=0.02, *, seed=None, device=0,
                   return_stats=False, rule="fast_consensus"):
    """Drop-in for fast_consensus.py:129 ``fast_consensus(G, algorithm, n_p, thresh, delta)``.

    G: an undirected networkx Graph (weights are ignored: the reference resets them to 1,
    :135-136) or an ``IdGraph``.  Returns a list of n_p partitions -- dicts for louvain,
    sets of frozensets for lpm and infomap, ``Cover`` objects for leiden -- or None for an unknown
    algorithm (the reference's loop
    ``break``s and returns None, :380-381).  ``seed`` makes the run reproducible (the
    reference is unseeded).  ``rule="new_consensus"`` (louvain only) switches to the
    new_consensus.py fork's weight rule (:155-163).
    """
    algo = algo_id(algorithm)
    if algo is None:
        return None
    if rule not in RULES:
        raise ValueError("rule must be one of %s" % (RULES,))
    if rule == "new_consensus":
        if algo != FC_ALGO_LOUVAIN:
            raise ValueError("the new_consensus.py rule exists for louvain only")
        algo = FC_ALGO_LOUVAIN_NC
    g = G if isinstance(G, IdGraph) else IdGraph.from_networkx(G)
    if algo == FC_ALGO_LEIDEN and not np.issubdtype(np.asarray(g.labels).dtype, np.integer):
        # The engine's leiden loop is the one-iteration exit the reference takes when its
        # str(vertex id)-keyed lookup (:97) never matches an int node (:214-217).  With other
        # node types that lookup can match and the reference runs a real loop: not modelled.
        raise NotImplementedError("algorithm='leiden' is modelled for integer node labels only "
                                  "(fast_consensus.py:97, :214-217)")
    with Engine(device=device, seed=seed) as eng:
        eng.set_option("store", store_order_pays(n_p, algo))
        eng.set_option("relabel", relabel_for(algo))
        eng.load_graph(g.n, g.u, g.v)
        labels, stats = eng.run(algo, int(n_p), float(thresh), float(delta))
    out = labels_to_output(algorithm, g.labels, labels)
    return (out, stats) if return_stats else out


def check_consensus_graph(G, n_p, delta):
    """fast_consensus.py:17-37 on a networkx graph (host utility, not the hot path)."""
    count = sum(1 for w in (d.get("weight") for _, _, d in G.edges(data=True)) if w != 0 and w != n_p)
    return not (count > delta * G.number_of_edges())


def group_to_partition(partition):
    """fast_consensus.py:55-71: {node: community} -> communities in first-appearance order."""
    part = {}
    for node, c in partition.items():
        part.setdefault(c, []).append(node)
    return part.values()
