#!/usr/bin/env python3
"""Generate golden vectors for the consensus hot path FROM THE REFERENCE ITSELF.

Runs in the development container only (needs /root/reference; the GPU box never
runs this).  The reference script `/root/reference/fast_consensus.py` is executed
unmodified; only its three un-vendored third-party imports are replaced by stubs:

* ``community`` (python-louvain 0.15, requirements.txt:5): ``generate_dendrogram`` /
  ``partition_at_level`` return a level-0 partition produced by a *stand-in*
  (networkx ``louvain_partitions`` first level, seeded).  python-louvain is not
  installed, so the Louvain arithmetic itself is not pinned.
* ``igraph`` (python-igraph 0.9.7, requirements.txt:4): a minimal ``Graph`` whose
  ``community_label_propagation().as_cover()`` runs networkx ``asyn_lpa_communities``
  (unweighted, seeded) on the vertex-id graph that ``nx_to_igraph``
  (fast_consensus.py:41-52) builds.
* ``leidenalg``: ``find_partition(...).as_cover()`` returns a seeded networkx louvain level 0
  (stand-in), and the module's ``mp.Pool`` is a serial map, so the reference's leiden
  branch runs in this process and its exit point is recorded.

Every community-detection result is RECORDED, as are the closure samples
(``random.sample`` at fast_consensus.py:181/297), the adjacency order of ``graph``
at each iteration start, and every graph passed to ``check_consensus_graph``
(fast_consensus.py:172, :201, :309).  Replaying the recorded labelings and
closure pairs through our implementation must reproduce every recorded graph
bit-exactly (weights, keep masks, convergence decisions, closure/repair edges).

The same harness runs the ``new_consensus.py`` fork (its weight rule, :155-163, is the
``louvain_nc`` variant).

Usage:  python tests/golden/make_golden.py [nc|r03]   (writes tests/golden/*.npz, *.json;
        ``nc``: only the new_consensus.py cases; ``r03``: only the round-3 cases)
"""
import contextlib
import importlib.util
import io
import json
import os
import random
import runpy
import shutil
import sys
import tempfile
import types

import numpy as np
import networkx as nx

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/fast_consensus.py"
REF_NC = "/root/reference/new_consensus.py"   # fork with the plain-count weight rule (:155-163)
KARATE = "/root/reference/examples/karate_club.txt"
sys.dont_write_bytecode = True


class Recorder:
    def __init__(self):
        self.reset(None)

    def reset(self, node_index):
        self.node_index = node_index        # node label -> id (node order of G)
        self.cd_labels = []                 # list of int arrays (N,), id space
        self.cd_graph_adj = []              # adjacency snapshot per CD call batch start
        self.checks = []                    # (edges u,v,w in id space) per check call
        self.pairs = []                     # closure pairs, list per iteration
        self.cur_pairs = None
        self.calls = 0
        self.n_p = None
        self.max_calls = None
        self.seed = 0


REC = Recorder()


def adj_snapshot(graph):
    """Flattened adjacency in networkx order: (ptr, nbr, w) in id space, node order."""
    idx = REC.node_index
    ptr = [0]
    nbr, wts = [], []
    for u in graph.nodes():
        for v, d in graph.adj[u].items():
            nbr.append(idx[v])
            wts.append(float(d.get("weight", 1.0)))
        ptr.append(len(nbr))
    return np.array(ptr, np.int64), np.array(nbr, np.int32), np.array(wts, np.float64)


def _on_cd_call(graph):
    if REC.max_calls is not None and REC.calls >= REC.max_calls:
        raise RuntimeError("golden generator: too many CD calls (loop did not converge)")
    if REC.calls % REC.n_p == 0:
        if graph is not None:
            REC.cd_graph_adj.append(adj_snapshot(graph))
        # a new iteration (or the final pass) starts: open a new closure-pair list
        REC.cur_pairs = []
        REC.pairs.append(REC.cur_pairs)
    REC.calls += 1


def _labels_from_sets(graph, sets):
    idx = REC.node_index
    lab = np.full(len(idx), -1, np.int32)
    for c, members in enumerate(sets):
        for v in members:
            lab[idx[v]] = c
    assert (lab >= 0).all()
    return lab


# ---------------------------------------------------------------- stub: community
def _generate_dendrogram(graph, part_init=None, weight="weight", resolution=1.0,
                         randomize=None, random_state=None):
    _on_cd_call(graph)
    rs = REC.seed * 100003 + REC.calls
    level0 = next(iter(nx.community.louvain_partitions(graph, weight=weight, seed=rs)))
    lab = _labels_from_sets(graph, level0)
    REC.cd_labels.append(lab)
    # python-louvain returns dict node->community, insertion order = graph node order
    return [{v: int(lab[REC.node_index[v]]) for v in graph.nodes()}]


def _partition_at_level(dendrogram, level):
    return dict(dendrogram[level])


community_stub = types.ModuleType("community")
community_stub.generate_dendrogram = _generate_dendrogram
community_stub.partition_at_level = _partition_at_level


# ---------------------------------------------------------------- stub: igraph
class _Cover:
    def __init__(self, comms):
        self._c = comms

    def as_cover(self):
        return self._c


class _ES(dict):
    pass


class Graph:
    def __init__(self):
        self.names = []
        self.edges = []
        self.es = _ES()

    def add_vertices(self, names):
        self.names = list(names)

    def add_edges(self, edges):
        self.edges = [(int(a), int(b)) for a, b in edges]

    def __setitem__(self, key, value):
        pass  # weights are ignored by community_label_propagation() as called

    def community_label_propagation(self, *a, **k):
        # vertex ids 0..n-1; the reference requires node labels 0..N-1 (README:62)
        H = nx.Graph()
        H.add_nodes_from(range(len(self.names)))
        H.add_edges_from(self.edges)
        _on_cd_call(None)  # vertex-id graph: adjacency order is igraph's, not recorded
        rs = REC.seed * 100003 + REC.calls
        comms = [sorted(c) for c in nx.community.asyn_lpa_communities(H, weight=None, seed=rs)]
        lab = np.full(len(self.names), -1, np.int32)
        for ci, c in enumerate(comms):
            for v in c:
                lab[REC.node_index[v]] = ci  # igraph vertex id == node label (README:62)
        REC.cd_labels.append(lab)
        return _Cover(comms)


def _community_infomap(self, *a, **k):
    # stand-in for igraph's Infomap (absent): networkx louvain level 0 on the vertex-id graph,
    # unweighted as called (fast_consensus.py:268, :390); only the loop around it is pinned
    H = nx.Graph()
    H.add_nodes_from(range(len(self.names)))
    H.add_edges_from(self.edges)
    _on_cd_call(None)
    rs = REC.seed * 100003 + REC.calls
    comms = [sorted(c) for c in next(iter(nx.community.louvain_partitions(H, seed=rs)))]
    lab = np.full(len(self.names), -1, np.int32)
    for ci, c in enumerate(comms):
        for v in c:
            lab[REC.node_index[v]] = ci
    REC.cd_labels.append(lab)
    return _Cover(comms)


Graph.community_infomap = _community_infomap

igraph_stub = types.ModuleType("igraph")
igraph_stub.Graph = Graph


# ---------------------------------------------------------------- stub: leidenalg
class _LeidenResult:
    def __init__(self, comms):
        self._c = comms

    def as_cover(self):
        return self._c


def _find_partition(graph, partition_type, weights=None, seed=None, n_iterations=2, **k):
    """Stand-in for leidenalg.find_partition (absent): a seeded networkx louvain level 0 on the
    vertex-id graph nx_to_igraph built (fast_consensus.py:123).  Clusters are lists of igraph
    vertex ids, as as_cover() yields them."""
    H = nx.Graph()
    H.add_nodes_from(range(len(graph.names)))
    H.add_edges_from(graph.edges)
    _on_cd_call(None)
    rs = REC.seed * 100003 + REC.calls * 7 + int(seed or 0)
    comms = [sorted(c) for c in next(iter(nx.community.louvain_partitions(H, seed=rs)))]
    lab = np.full(len(graph.names), -1, np.int32)
    for ci, c in enumerate(comms):
        for v in c:
            lab[REC.node_index[v]] = ci      # vertex id == node label for 0..N-1 graphs (README:62)
    REC.cd_labels.append(lab)
    return _LeidenResult(comms)


leiden_stub = types.ModuleType("leidenalg")
leiden_stub.find_partition = _find_partition
leiden_stub.ModularityVertexPartition = object


class _SerialPool:
    """multiprocessing.Pool replaced by a serial map (fast_consensus.py:210-211, :386-387):
    the recorder and the seeded RNGs live in this process."""

    def __init__(self, processes=None):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def map(self, f, it):
        return [f(x) for x in it]


mp_stub = types.ModuleType("multiprocessing")
mp_stub.Pool = _SerialPool


# ---------------------------------------------------------------- recording RNG proxy
class _RecordingRandom:
    """Stands in for the `random` module inside the reference namespace."""

    def __getattr__(self, name):
        return getattr(random, name)

    def sample(self, population, k):
        out = random.sample(population, k)
        if k == 2 and REC.cur_pairs is not None:
            idx = REC.node_index
            REC.cur_pairs.append((idx[out[0]], idx[out[1]]))
        return out


def load_reference(path=REF):
    sys.modules["community"] = community_stub
    sys.modules["igraph"] = igraph_stub
    sys.modules["leidenalg"] = leiden_stub
    spec = importlib.util.spec_from_file_location("fc_reference_%d" % len(path), path)
    fc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fc)
    fc.mp = mp_stub
    orig_check = fc.check_consensus_graph

    def check_wrapper(G, n_p, delta):
        idx = REC.node_index
        e = np.array([(idx[u], idx[v], G[u][v]["weight"]) for u, v in G.edges()],
                     dtype=np.float64).reshape(-1, 3)
        res = orig_check(G, n_p=n_p, delta=delta)
        REC.checks.append((e, bool(res)))
        return res

    fc.check_consensus_graph = check_wrapper
    fc.random = _RecordingRandom()
    return fc


def run_case(fc, name, edgefile, algorithm, n_p, tau, delta, seed, max_iters=30, rule="fast_consensus"):
    G = nx.read_edgelist(edgefile, nodetype=int)
    nodes = list(G.nodes())
    REC.reset({v: i for i, v in enumerate(nodes)})
    REC.n_p, REC.seed = n_p, seed
    REC.max_calls = n_p * (max_iters + 1)
    random.seed(seed)
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):   # new_consensus.py prints progress
        out = fc.fast_consensus(G, algorithm=algorithm, n_p=n_p, thresh=tau, delta=delta)
    n_cd = len(REC.cd_labels)
    assert n_cd % n_p == 0
    n_batches = n_cd // n_p
    # edge list in file order (id space) -- what our ingest sees
    edges_file = []
    with open(edgefile) as f:
        for line in f:
            p = line.split()
            if len(p) >= 2:
                edges_file.append((REC.node_index[int(p[0])], REC.node_index[int(p[1])]))
    arrays = {
        "nodes": np.array(nodes, np.int64),
        "edges_file": np.array(edges_file, np.int32),
        "cd_labels": np.stack(REC.cd_labels).astype(np.int32),
    }
    for b, (ptr, nbr, w) in enumerate(REC.cd_graph_adj):
        arrays[f"adj{b}_ptr"] = ptr
        arrays[f"adj{b}_nbr"] = nbr
        arrays[f"adj{b}_w"] = w
    check_meta = []
    for c, (e, res) in enumerate(REC.checks):
        arrays[f"check{c}_edges"] = e
        check_meta.append(res)
    for b, pl in enumerate(REC.pairs):
        arrays[f"pairs{b}"] = np.array(pl, np.int32).reshape(-1, 2)
    # final output as labels (id space)
    finals = []
    for part in out:
        if algorithm == "leiden":            # as_cover(): clusters of igraph vertex ids (== node ids here)
            lab = np.full(len(nodes), -1, np.int32)
            for ci, c in enumerate(part):
                for v in c:
                    lab[REC.node_index[v]] = ci
        elif isinstance(part, dict):
            lab = np.array([part[v] for v in nodes], np.int32)
        else:
            lab = np.full(len(nodes), -1, np.int32)
            for ci, c in enumerate(sorted(sorted(x) for x in part)):
                for v in c:
                    lab[REC.node_index[v]] = ci
        finals.append(lab)
    arrays["final_labels"] = np.stack(finals)
    meta = {
        "name": name, "algorithm": algorithm, "n_p": n_p, "tau": tau, "delta": delta,
        "seed": seed, "N": len(nodes), "m": G.number_of_edges(),
        "n_cd_batches": n_batches, "check_results": check_meta,
        "n_checks": len(REC.checks),
        "stand_in": "networkx %s louvain_partitions level0 / asyn_lpa_communities" % nx.__version__,
        "reference": "%s (ytabatabaee/fastconsensus @ 2025-02-25)" % (
            "fast_consensus.py" if rule == "fast_consensus" else "new_consensus.py"),
        "rule": rule,
    }
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(name, meta["N"], meta["m"], "batches", n_batches, "checks", check_meta)
    return out


def run_cli_case(name, edgefile, argv, seed):
    """Run the reference CLI (fast_consensus.py:414-466) and record its output tree."""
    tmp = tempfile.mkdtemp()
    shutil.copy(edgefile, os.path.join(tmp, "graph.txt"))
    cwd = os.getcwd()
    G = nx.read_edgelist(edgefile, nodetype=int)
    REC.reset({v: i for i, v in enumerate(G.nodes())})
    n_p = int(argv[argv.index("-np") + 1])
    REC.n_p, REC.seed, REC.max_calls = n_p, seed, n_p * 40
    random.seed(seed)
    np.random.seed(seed)
    old_argv = sys.argv
    os.chdir(tmp)
    try:
        sys.argv = ["fast_consensus.py", "-f", "graph.txt"] + argv
        g = {"__name__": "__main__"}
        sys.modules["community"] = community_stub
        sys.modules["igraph"] = igraph_stub
        sys.modules["leidenalg"] = types.ModuleType("leidenalg")
        runpy.run_path(REF, run_name="__main__")
    finally:
        sys.argv = old_argv
        os.chdir(cwd)
    files = {}
    for root, _, fnames in os.walk(tmp):
        for fn in fnames:
            p = os.path.join(root, fn)
            rel = os.path.relpath(p, tmp)
            if rel == "graph.txt":
                continue
            with open(p) as f:
                files[rel] = f.read()
    dirs = sorted(d for d in os.listdir(tmp) if os.path.isdir(os.path.join(tmp, d)))
    finals = np.stack(REC.cd_labels[-n_p:])
    shutil.rmtree(tmp)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), final_labels=finals,
                        nodes=np.array(list(G.nodes()), np.int64))
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump({"argv": argv, "dirs": dirs, "files": files}, f, indent=0, sort_keys=True)
    print(name, "dirs", dirs, "files", len(files))


def run_arg_errors():
    """Validation messages + exit status of the CLI (fast_consensus.py:73-88, :430-432)."""
    import subprocess
    cases = [["-d", "1.5"], ["-d", "-0.5"], ["--alg", "bogus"], ["-t", "1.5"], ["-t", "-1"]]
    results = []
    stub_dir = tempfile.mkdtemp()
    for m in ("community", "igraph", "leidenalg"):
        with open(os.path.join(stub_dir, m + ".py"), "w") as f:
            f.write("")
    for argv in cases:
        env = dict(os.environ, PYTHONPATH=stub_dir, PYTHONDONTWRITEBYTECODE="1")
        p = subprocess.run([sys.executable, REF, "-f", KARATE] + argv, capture_output=True,
                           text=True, env=env, cwd=stub_dir)
        results.append({"argv": argv, "stdout": p.stdout, "returncode": p.returncode})
    shutil.rmtree(stub_dir)
    with open(os.path.join(HERE, "cli_arg_errors.json"), "w") as f:
        json.dump(results, f, indent=1)
    print("arg errors", [(r["argv"], r["returncode"], r["stdout"].strip()) for r in results])


def make_lfr1k():
    path = os.path.join(HERE, "lfr1k_mu04.txt")
    G = nx.LFR_benchmark_graph(1000, 3, 1.5, 0.4, average_degree=20, max_degree=50,
                               min_community=20, max_community=100, seed=42)
    G.remove_edges_from(nx.selfloop_edges(G))
    comm = np.full(G.number_of_nodes(), -1, np.int32)
    for ci, c in enumerate(sorted({tuple(sorted(G.nodes[v]["community"])) for v in G})):
        for v in c:
            comm[v] = ci
    with open(path, "w") as f:
        for u, v in G.edges():
            f.write("%d %d\n" % (u, v))
    np.save(os.path.join(HERE, "lfr1k_mu04_planted.npy"), comm)
    return path


def main_nc():
    """Cases of the new_consensus.py rule only (existing fixtures untouched)."""
    karate = os.path.join(HERE, "karate_club.txt")
    lfr = os.path.join(HERE, "lfr1k_mu04.txt")
    nc = load_reference(REF_NC)
    run_case(nc, "karate_louvain_nc_np50", karate, "louvain", 50, 0.2, 0.1, seed=11, rule="new_consensus")
    run_case(nc, "lfr1k_louvain_nc_np20", lfr, "louvain", 20, 0.2, 0.02, seed=13, rule="new_consensus")


def main_r03():
    """Round-3 cases (existing fixtures untouched):
    * lpm on the native LFR n=1000 mu=0.55 graph, where LPA finds structure (the networkx
      mu=0.4 graph floods to one community), so the recorded LPA labelings are non-degenerate;
    * the leiden branch (fast_consensus.py:204-258, final pass :385-388) with leidenalg and
      the process pool stubbed: records where the reference exits;
    * the infomap branch (the lpm loop, :260-310, with community_infomap, :268, :390)."""
    karate = os.path.join(HERE, "karate_club.txt")
    lfr = os.path.join(HERE, "lfr1k_mu04.txt")
    mu055 = os.path.join(HERE, "lfr1k_mu055_synth.txt")
    fc = load_reference()
    run_case(fc, "karate_leiden_np20", karate, "leiden", 20, 0.2, 0.02, seed=31)
    run_case(fc, "lfr1k_leiden_np20", lfr, "leiden", 20, 0.2, 0.02, seed=32)
    if os.environ.get("FC_GOLDEN_ONLY") == "leiden":
        return
    # a fixed seed, no selection (main_r04 also summarises seeds 21..40)
    run_case(fc, "lfr1k_mu055_lpm_np20", mu055, "lpm", 20, 0.8, 0.02, seed=21)
    # a graph well inside LPA's detectable range (native LFR n=1000 mu=0.3): every replica finds structure
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from fastconsensus_amd import synth
    mu03 = os.path.join(HERE, "lfr1k_mu03_synth.txt")
    u, v, planted = synth.lfr(1000, 0.3, seed=8)
    with open(mu03, "w") as f:
        for a, b in zip(u.tolist(), v.tolist()):
            f.write("%d %d\n" % (a, b))
    np.save(os.path.join(HERE, "lfr1k_mu03_synth_planted.npy"), planted)
    run_case(fc, "lfr1k_mu03_lpm_np20", mu03, "lpm", 20, 0.8, 0.02, seed=41)
    run_case(fc, "karate_infomap_np20", karate, "infomap", 20, 0.6, 0.02, seed=33)
    run_case(fc, "lfr1k_infomap_np20", lfr, "infomap", 20, 0.6, 0.02, seed=34)


def main_r04():
    """The mu=0.55 lpm fixture at a FIXED seed (21).  Round 3 kept, of seeds 21..40, the one
    whose first reference LPA batch had the most structured replicas: a cherry-picked sample.
    Now every seed's first batch is summarised in lfr1k_mu055_lpm_firstbatch.json (structured
    replicas and their NMI to the planted partition), and the detectability test compares the
    device with that pooled distribution (20 seeds x 20 replicas)."""
    from sklearn.metrics import normalized_mutual_info_score as nmi
    mu055 = os.path.join(HERE, "lfr1k_mu055_synth.txt")
    planted = np.load(os.path.join(HERE, "lfr1k_mu055_synth_planted.npy"))
    fc = load_reference()
    seeds, structured, nmis = list(range(21, 41)), [], []
    for seed in seeds[::-1]:                 # seed 21 last: its run is the fixture left on disk
        run_case(fc, "lfr1k_mu055_lpm_np20", mu055, "lpm", 20, 0.8, 0.02, seed=seed)
        pl = planted[np.array(list(REC.node_index), np.int64)]   # id space (node order of the read graph)
        ok = [x for x in REC.cd_labels[:20] if len(np.unique(x)) > 1]
        structured.append(len(ok))
        nmis.append([float(nmi(pl, x)) for x in ok])
    with open(os.path.join(HERE, "lfr1k_mu055_lpm_firstbatch.json"), "w") as f:
        json.dump({"graph": "lfr1k_mu055_synth.txt", "algorithm": "lpm", "n_p": 20, "seeds": seeds[::-1],
                   "structured": structured, "structured_nmi": nmis,
                   "structured_fraction": sum(structured) / (20.0 * len(seeds)),
                   "note": "first CD batch of the reference run (fast_consensus.py:270, networkx asyn_lpa stand-in) "
                           "per seed; the fixture lfr1k_mu055_lpm_np20 is the seed-21 run"}, f, indent=1)


def main():
    if sys.argv[1:] == ["r04"]:
        return main_r04()
    if sys.argv[1:] == ["nc"]:
        return main_nc()
    if sys.argv[1:] == ["r03"]:
        return main_r03()
    shutil.copy(KARATE, os.path.join(HERE, "karate_club.txt"))
    karate = os.path.join(HERE, "karate_club.txt")
    lfr = make_lfr1k()
    fc = load_reference()
    run_case(fc, "karate_louvain_np50", karate, "louvain", 50, 0.2, 0.1, seed=1)
    run_case(fc, "karate_lpm_np20", karate, "lpm", 20, 0.8, 0.02, seed=2)
    run_case(fc, "lfr1k_louvain_np20", lfr, "louvain", 20, 0.2, 0.02, seed=3)
    run_case(fc, "lfr1k_lpm_np20", lfr, "lpm", 20, 0.8, 0.02, seed=4)
    run_cli_case("cli_karate_louvain", karate, ["--alg", "louvain", "-np", "10", "-t", "0.2", "-d", "0.1"], seed=5)
    run_cli_case("cli_karate_lpm", karate, ["--alg", "lpm", "-np", "5"], seed=6)
    run_arg_errors()
    main_nc()


if __name__ == "__main__":
    main()
