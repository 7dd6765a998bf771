"""CLI drop-in contract (fast_consensus.py:414-466) against the reference's own CLI run
(tests/golden/cli_*.json, produced by running the reference script): validation messages
and exit status, output directory names, and the output files byte for byte (louvain) /
as sets of communities (lpm, whose line order is Python set order)."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = golden_io.GOLDEN


def _golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return meta, z["final_labels"], z["nodes"]


def _args(argv):
    from fastconsensus_amd.cli import DEFAULT_TAU, build_parser
    a = build_parser().parse_args(["-f", "graph.txt"] + argv)
    if a.t is None:
        a.t = DEFAULT_TAU.get(a.alg, 0.2)
    return a


def test_argument_errors_match_reference():
    with open(os.path.join(GOLDEN, "cli_arg_errors.json")) as f:
        cases = json.load(f)
    for c in cases:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "fast_consensus.py"),
                            "-f", os.path.join(GOLDEN, "karate_club.txt")] + c["argv"],
                           capture_output=True, text=True, cwd=ROOT)
        assert p.stdout == c["stdout"], c["argv"]
        assert p.returncode == c["returncode"] == 0


def test_louvain_output_tree_byte_exact(tmp_path):
    from fastconsensus_amd.cli import output_dirs, write_outputs
    from fastconsensus_amd.core import labels_to_output
    meta, labels, nodes = _golden("cli_karate_louvain")
    args = _args(meta["argv"])
    assert sorted(output_dirs(args)) == meta["dirs"]
    write_outputs(args, labels_to_output("louvain", nodes, labels), root=str(tmp_path))
    got = {}
    for d in meta["dirs"]:
        for fn in os.listdir(tmp_path / d):
            got[d + "/" + fn] = (tmp_path / d / fn).read_text()
    assert got == meta["files"]


def test_lpm_output_tree_same_communities(tmp_path):
    from fastconsensus_amd.cli import output_dirs, write_outputs
    from fastconsensus_amd.core import labels_to_output
    meta, labels, nodes = _golden("cli_karate_lpm")
    args = _args(meta["argv"])
    assert sorted(output_dirs(args)) == meta["dirs"]
    write_outputs(args, labels_to_output("lpm", nodes, labels), root=str(tmp_path))
    mem_dir = [d for d in meta["dirs"] if d.startswith("memberships")][0]
    assert os.listdir(tmp_path / mem_dir) == []          # created but empty for lpm
    for key, text in meta["files"].items():
        ours = (tmp_path / key).read_text()
        as_sets = lambda t: sorted(sorted(map(int, ln.split())) for ln in t.strip().split("\n"))
        assert as_sets(ours) == as_sets(text), key


def test_native_parser_matches_networkx(tmp_path):
    import networkx as nx
    from fastconsensus_amd.core import IdGraph
    p = tmp_path / "g.txt"
    p.write_text("# comment\n5 7\n7 9 0.5\n\n9 5\n5 7\n3 3\n11\n")  # dup, self loop, 1-col line
    g = IdGraph.from_edgelist_file(str(p))
    G = nx.read_edgelist(str(p), nodetype=int, data=False)
    assert list(g.labels) == list(G.nodes())
    edges = {tuple(sorted((int(g.labels[a]), int(g.labels[b])))) for a, b in zip(g.u, g.v)}
    assert edges == {tuple(sorted(e)) for e in G.edges()}
    g2 = IdGraph.from_edgelist_file(os.path.join(GOLDEN, "karate_club.txt"))
    K = nx.read_edgelist(os.path.join(GOLDEN, "karate_club.txt"), nodetype=int)
    assert list(g2.labels) == list(K.nodes()) and len(g2.u) == K.number_of_edges()


def test_networkx_input_order_is_adjacency_order():
    """IdGraph.from_networkx emits each node's later neighbours in G.adj order, which is
    what the repair tie-break needs (fast_consensus.py:131, :194)."""
    import networkx as nx
    from fastconsensus_amd.core import IdGraph
    G = nx.Graph()
    G.add_edges_from([(3, 1), (1, 2), (3, 0), (2, 0), (1, 0)])
    g = IdGraph.from_networkx(G)
    assert list(g.labels) == [3, 1, 2, 0]
    # node 1 (id 1): later neighbours in adjacency order: 2 (id 2), then 0 (id 3)
    pairs = list(zip(g.u.tolist(), g.v.tolist()))
    assert pairs.index((1, 2)) < pairs.index((1, 3))


@pytest.mark.parametrize("labels", ["ints", "shuffled", "strings", "sparse_ints", "tuples"])
def test_networkx_conversion_matches_literal_walk(labels):
    """The vectorised IdGraph.from_networkx equals the literal walk (every node in G.nodes()
    order, its later neighbours in G.adj order) for integer, shuffled, string and sparse labels."""
    import random
    import networkx as nx
    from fastconsensus_amd.core import IdGraph
    G = nx.gnm_random_graph(600, 2500, seed=3)
    if labels == "shuffled":
        perm = list(G.nodes())
        random.Random(5).shuffle(perm)
        H = nx.Graph()
        H.add_nodes_from(perm)
        H.add_edges_from(G.edges())
        G = H
    elif labels == "strings":
        G = nx.relabel_nodes(G, {i: "v%d" % (i * 7 % 600) for i in G.nodes()})
    elif labels == "sparse_ints":
        G = nx.relabel_nodes(G, {i: i * 100003 for i in G.nodes()})
    elif labels == "tuples":                       # grid-style nodes: one object each, not a 2-D array
        G = nx.relabel_nodes(G, {i: (i // 30, i % 30) for i in G.nodes()})
    nodes = list(G.nodes())
    idx = {x: i for i, x in enumerate(nodes)}
    exp = [(idx[x], idx[z]) for x in nodes for z in G.adj[x] if idx[z] > idx[x]]
    g = IdGraph.from_networkx(G)
    assert list(g.labels) == nodes
    assert list(zip(g.u.tolist(), g.v.tolist())) == exp


@pytest.mark.parametrize("kind", ["ints", "strings", "tuples"])
def test_partition_output_matches_literal_grouping(kind):
    """labels_to_output (lpm / infomap: a set of frozensets per labeling, fast_consensus.py:383-392)
    equals the literal per-node grouping, for integer, string and tuple nodes and ragged labels."""
    from fastconsensus_amd.core import IdGraph, labels_to_output
    rng = np.random.default_rng(7)
    n = 500
    nodes = {"ints": list(range(n)), "strings": ["v%d" % (i * 7 % n) for i in range(n)],
             "tuples": [(i // 25, i % 25) for i in range(n)]}[kind]
    g = IdGraph(nodes, np.zeros(0, np.int32), np.zeros(0, np.int32))
    labels = np.stack([rng.integers(0, k, n) for k in (1, 7, 200, n)]).astype(np.int32)
    out = labels_to_output("lpm", g.labels, labels)
    for lab, got in zip(labels, out):
        groups = {}
        for x, c in zip(nodes, lab.tolist()):
            groups.setdefault(c, []).append(x)
        assert got == {frozenset(v) for v in groups.values()}
    d = labels_to_output("louvain", g.labels, labels[:1])[0]
    assert list(d.keys()) == nodes and list(d.values()) == labels[0].tolist()
    assert labels_to_output("lpm", g.labels, labels[:0]) == []


def test_unknown_and_out_of_scope_algorithms():
    import networkx as nx
    import fastconsensus_amd as fc
    G = nx.karate_club_graph()
    assert fc.fast_consensus(G, algorithm="no-such-alg") is None   # reference: returns None
    for alg in ("cnm",):
        with pytest.raises(NotImplementedError):
            fc.fast_consensus(G, algorithm=alg)
