"""The drop-in host conversion (fast_consensus.py:129-136 input, :383-384 output): the forked
adjacency read equals the serial one, for integer and non-integer nodes and for graphs whose
adjacency dict is not keyed in node order."""
import networkx as nx
import numpy as np
import pytest

from fastconsensus_amd import core


def _graph(n, seed, relabel=None):
    rng = np.random.default_rng(seed)
    G = nx.Graph()
    G.add_nodes_from(rng.permutation(n).tolist())
    G.add_edges_from(zip(rng.integers(0, n, 6 * n).tolist(), rng.integers(0, n, 6 * n).tolist()))
    G.remove_edges_from(nx.selfloop_edges(G))
    return nx.relabel_nodes(G, relabel) if relabel else G


@pytest.mark.parametrize("kind", ["int", "str", "reordered"])
@pytest.mark.parametrize("workers", [1, 3, 8])
def test_forked_adjacency_read_equals_serial(monkeypatch, kind, workers):
    n = 3000
    G = _graph(n, 5, {i: "v%d" % i for i in range(n)} if kind == "str" else None)
    if kind == "reordered":     # node insertion order != _adj order is impossible in nx; fake a view
        class H(nx.Graph):
            pass
        H2 = H()
        H2.add_nodes_from(reversed(list(G.nodes())))
        H2.add_edges_from(G.edges())
        H2._node = dict(reversed(list(H2._node.items())))
        G = H2
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 10 ** 12)
    a = core.IdGraph.from_networkx(G)
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 1)
    monkeypatch.setenv("FC_HOST_WORKERS", str(workers))
    b = core.IdGraph.from_networkx(G)
    assert list(a.labels) == list(b.labels) == list(G.nodes())
    np.testing.assert_array_equal(a.u, b.u)
    np.testing.assert_array_equal(a.v, b.v)
    # every edge once, as node-order indices, later neighbour in G.adj order
    idx = {x: i for i, x in enumerate(G.nodes())}
    exp = [(idx[x], idx[y]) for x in G.nodes() for y in G.adj[x] if idx[y] > idx[x]]
    assert list(zip(b.u.tolist(), b.v.tolist())) == exp


def test_louvain_output_dicts_are_node_ordered():
    nodes = np.array([5, 2, 9, 0])
    lab = np.array([[0, 1, 0, 2], [3, 3, 3, 3]], np.int32)
    out = core.labels_to_output("louvain", nodes, lab)
    assert out == [{5: 0, 2: 1, 9: 0, 0: 2}, {5: 3, 2: 3, 9: 3, 0: 3}]
    assert [list(d) for d in out] == [[5, 2, 9, 0]] * 2 and all(type(d) is dict for d in out)


def _count_forks(monkeypatch):
    import os
    calls = []
    real = os.fork

    def fork():
        calls.append(1)
        return real()
    monkeypatch.setattr(os, "fork", fork)
    return calls


def test_fast_consensus_twice_forked_read_after_engine_attempt(monkeypatch):
    """fast_consensus(G) twice in one process past ADJ_PARALLEL_MIN: the second call's forked
    adjacency read runs after the first call loaded the HIP library and created (on a GPU box)
    or tried to create (here: FC_ENODEV) an Engine.  Both reads fork and equal the serial one."""
    import fastconsensus_amd as fc
    G = _graph(4000, 9)
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 10 ** 12)
    ser = core.IdGraph.from_networkx(G)
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 1000)
    monkeypatch.setenv("FC_HOST_WORKERS", "4")
    forks = _count_forks(monkeypatch)
    seen = []
    real_from = core.IdGraph.from_networkx

    def spy(g):
        seen.append(real_from(g))
        return seen[-1]
    monkeypatch.setattr(core.IdGraph, "from_networkx", staticmethod(spy))
    for _ in range(2):
        try:
            fc.fast_consensus(G, "louvain", n_p=2, seed=1)
        except Exception as e:          # no GPU here: the Engine refuses after the conversion
            assert "GPU" in str(e) or "device" in str(e).lower() or "ENODEV" in str(e), e
    assert len(seen) == 2 and len(forks) >= 8
    for g in seen:
        np.testing.assert_array_equal(g.u, ser.u)
        np.testing.assert_array_equal(g.v, ser.v)


def test_forked_read_skipped_with_python_threads(monkeypatch):
    """Another Python thread alive: the read is serial (no fork), same result."""
    import threading
    G = _graph(3000, 11)
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 1)
    monkeypatch.setenv("FC_HOST_WORKERS", "4")
    forks = _count_forks(monkeypatch)
    stop = threading.Event()
    t = threading.Thread(target=stop.wait)
    t.start()
    try:
        a = core.IdGraph.from_networkx(G)
    finally:
        stop.set()
        t.join()
    assert forks == []
    b = core.IdGraph.from_networkx(G)
    assert len(forks) == 4
    np.testing.assert_array_equal(a.u, b.u)
    np.testing.assert_array_equal(a.v, b.v)


def test_forked_read_deadline_kills_and_falls_back(monkeypatch):
    """Workers still running at the deadline are killed and reaped; the serial read answers."""
    import os
    import time
    parent = os.getpid()
    rows = [{i + 1: None, i + 2: None} for i in range(5000)]
    lens = np.full(len(rows), 2, np.int64)

    def key(x):
        if os.getpid() != parent:      # only the forked workers hang
            time.sleep(60)
        return x
    monkeypatch.setattr(core, "ADJ_PARALLEL_MIN", 1)
    monkeypatch.setattr(core, "ADJ_DEADLINE_S", 0.5)
    monkeypatch.setenv("FC_HOST_WORKERS", "3")
    t = time.monotonic()
    got = core.read_adjacency(rows, lens, key)
    assert time.monotonic() - t < 20
    np.testing.assert_array_equal(got, np.array([[i + 1, i + 2] for i in range(5000)]).ravel())
