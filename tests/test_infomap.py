"""Infomap branch (fast_consensus.py:260-310 with the infomap CD :267-268, final pass :389-390).

python-igraph is absent, so community_infomap() is "parity unpinned": the oracle restates
igraph's algorithm -- the core (oracle/fc_oracle.c orc_infomap: the two-level map equation,
greedy passes in random order, aggregation by modules, best of 10 trials) and the full
partition with its single-node and sub-module re-partition rounds (orc_infomap_full) -- and the
device, which runs the core, is held statistically to the FULL restatement (stored values,
tests/golden/infomap_full.json, make_infomap_full.py) as well as to the core, with the
tolerances written in each test.  Around the CD the
infomap branch IS the lpm loop (co-membership count, threshold, weight-0 closure, check after
closure), pinned bit-exactly by the lpm golden replays.
"""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as orc
from tests import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def plogp(p):
    p = np.asarray(p, np.float64)
    out = np.zeros_like(p)
    nz = p > 0
    out[nz] = p[nz] * np.log2(p[nz])
    return out


def codelength(N, e, lab):
    """Two-level map equation (bits) of a partition of an unweighted undirected graph."""
    deg = np.bincount(e.ravel(), minlength=N).astype(np.float64)
    W = deg.sum()
    k = int(lab.max()) + 1
    tot = np.bincount(lab, weights=deg, minlength=k)
    cut = lab[e[:, 0]] != lab[e[:, 1]]
    out = np.bincount(lab[e[cut, 0]], minlength=k) + np.bincount(lab[e[cut, 1]], minlength=k)
    q, p = out / W, tot / W
    return float(plogp(q.sum()) - 2 * plogp(q).sum() - plogp(deg / W).sum() + plogp(q + p).sum())


def nmi(a, b):
    from sklearn.metrics import normalized_mutual_info_score
    return normalized_mutual_info_score(a, b)


def lfr(n, mu, seed=42):
    from fastconsensus_amd import synth
    u, v, planted = synth.lfr(n, mu, seed=seed)
    return n, np.stack([u, v], 1), planted


def karate():
    e = np.loadtxt(os.path.join(golden_io.GOLDEN, "karate_club.txt"), dtype=np.int64)[:, :2]
    nodes, e = np.unique(e, return_inverse=True)
    return len(nodes), e.reshape(-1, 2).astype(np.int32)


# ------------------------------------------------------------------------------ CPU: oracle
def test_oracle_infomap_codelength_and_recovery():
    n, e, planted = lfr(1000, 0.4)
    g = orc.EdgeGraph.from_lines(n, e)
    lab, L = orc.infomap(g, seed=1)
    assert abs(L - codelength(n, e, lab)) < 1e-9          # the returned codelength is the map equation
    assert nmi(planted, lab) > 0.95
    assert L <= codelength(n, e, planted) + 1e-9           # at least as short as the planted modules
    lab1, L1 = orc.infomap(g, seed=1, trials=1)
    assert L <= L1 + 1e-12                                 # best of 10 includes the first trial


def test_oracle_infomap_karate():
    """igraph's community_infomap finds 3 modules, L = 4.3118 bits, on Zachary's karate club
    (a published value); the restated core reaches it."""
    n, e = karate()
    g = orc.EdgeGraph.from_lines(n, e)
    lab, L = orc.infomap(g, seed=3)
    assert L <= 4.312 and len(np.unique(lab)) == 3


@pytest.mark.parametrize("graph", ["karate", "lfr1k_mu04", "lfr1k_mu06", "lesmis"])
def test_core_vs_repartition_rounds_gap(graph):
    """igraph's infomap_partition wraps the greedy core in alternating single-node and
    sub-module re-partition rounds (restated in orc_infomap_full; the engine and orc_infomap run
    the core only).  Measured gap, core-only minus full codelength over the same 10 trials:
    0 on karate, LFR-1k mu=0.4/0.6, les Miserables, LFR-10k mu=0.5/0.6 and LFR-100k mu=0.5;
    0.0102 % on LFR-10k mu=0.7.  Held here to <= 0.05 %, full <= core."""
    import networkx as nx
    from fastconsensus_amd import synth
    if graph == "karate":
        n, e = karate()
    elif graph == "lesmis":
        G = nx.convert_node_labels_to_integers(nx.les_miserables_graph())
        n, e = G.number_of_nodes(), np.array(G.edges(), np.int32)
    else:
        u, v, _ = synth.lfr(1000, 0.4 if graph.endswith("04") else 0.6, seed=42)
        n, e = 1000, np.stack([u, v], 1)
    g = orc.EdgeGraph.from_lines(n, e)
    lab, L, Lc = orc.infomap_full(g, seed=1)
    print("%s: full %.6f bits, core %.6f bits, gap %.4f %%, %d modules" % (graph, L, Lc, 100 * (Lc - L) / Lc,
                                                                        len(np.unique(lab))))
    assert L <= Lc + 1e-9
    assert (Lc - L) / Lc <= 5e-4
    if graph == "karate":
        assert abs(L - 4.3118) < 1e-4 and len(np.unique(lab)) == 3


# ------------------------------------------------------------------------------ device
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def fcmod():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fastconsensus_amd as fc
    return fc


def device_infomap(fcmod, n, e, count, seed, rbegin=0, total=None, trials=None):
    with fcmod.Engine(seed=seed) as eng:
        if trials:
            eng.set_option("infomap_trials", trials)
        eng.load_graph(n, e[:, 0], e[:, 1])
        eng.cd(4, rbegin, count, total or count, 0)
        return eng.get_labels(count)


def full_restatement(name):
    """igraph's full Infomap partition (core + re-partition rounds, orc_infomap_full), stored."""
    import json
    with open(os.path.join(golden_io.GOLDEN, "infomap_full.json")) as f:
        return json.load(f)[name]


# Tolerances (LFR-1k, 16 replicas): mean codelength within 0.5 % of the core restatement's and
# of igraph's full partition's (stored, 8 seeds), mean NMI to planted >= restatement - 0.02.
@pytest.mark.gpu
def test_infomap_lfr1k_vs_restatement(fcmod):
    n, e, planted = lfr(1000, 0.4)
    g = orc.EdgeGraph.from_lines(n, e)
    dev = device_infomap(fcmod, n, e, 16, seed=11)
    ref = [orc.infomap(g, seed=s)[0] for s in range(8)]
    full = full_restatement("lfr1k_mu04")
    Ld = np.mean([codelength(n, e, x) for x in dev])
    Lr = np.mean([codelength(n, e, x) for x in ref])
    nd = np.mean([nmi(planted, x) for x in dev])
    nr = np.mean([nmi(planted, x) for x in ref])
    print("infomap LFR-1k device L %.4f NMI %.4f | core restatement L %.4f NMI %.4f | full L %.4f NMI %.4f"
          % (Ld, nd, Lr, nr, full["L_mean"], full["nmi_mean"]))
    assert abs(Ld - Lr) <= 0.005 * Lr
    assert abs(Ld - full["L_mean"]) <= 0.005 * full["L_mean"]
    assert nd >= nr - 0.02 and nd >= full["nmi_mean"] - 0.02


# Tolerances (C3-size LFR-100k, 4 device replicas / 2 stored runs of the full restatement, 10
# trials each): mean codelength within 0.5 %, module count within 10 %, NMI >= full - 0.02.
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_infomap_lfr100k_vs_restatement(fcmod):
    n, e, planted = lfr(100_000, 0.5)
    g = orc.EdgeGraph.from_lines(n, e)
    dev = device_infomap(fcmod, n, e, 4, seed=21)
    full = full_restatement("lfr100k_mu05")       # igraph's full partition (2 stored runs of 10 trials)
    Ld = np.mean([codelength(n, e, x) for x in dev])
    kd = np.mean([len(np.unique(x)) for x in dev])
    nd = np.mean([nmi(planted, x) for x in dev])
    Lr, kr = full["L_mean"], full["modules_mean"]
    print("infomap LFR-100k device L %.4f k %.0f NMI %.4f | full restatement L %.4f k %.0f NMI %.4f"
          % (Ld, kd, nd, Lr, kr, full["nmi_mean"]))
    assert abs(Ld - Lr) <= 0.005 * Lr
    assert abs(kd - kr) <= 0.10 * kr
    assert nd >= full["nmi_mean"] - 0.02


# Tolerance (karate, 8 replicas of 10 trials): the best replica reaches igraph's 4.3118 bits;
# the mean is within 0.5 % of the restatement's mean over 8 seeds (measured: all 8 at 4.3118,
# like the restatement; single trials spread over 4.3118-4.39 on both).
@pytest.mark.gpu
def test_infomap_karate_device(fcmod):
    n, e = karate()
    g = orc.EdgeGraph.from_lines(n, e)
    Ld = [codelength(n, e, x) for x in device_infomap(fcmod, n, e, 8, seed=5)]
    Lr = [orc.infomap(g, seed=s)[1] for s in range(8)]
    print("infomap karate device", np.round(Ld, 4), "restatement", np.round(Lr, 4))
    assert min(Ld) <= 4.312
    assert abs(np.mean(Ld) - np.mean(Lr)) <= 0.005 * np.mean(Lr)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["karate", "lfr1k"])
def test_infomap_one_replica_empty_bucket_lists(fcmod, graph):
    """One replica of one trial: at the aggregate levels a handful of modules is spread over
    32 buckets, so most of a pass's bucket lists are empty (leiden.hip skips them: no
    zero-block launch, whose error state would surface in a later HIP call).  Deterministic,
    a valid partition, codelength within the single-trial spread of the restatement."""
    if graph == "karate":
        n, e = karate()
    else:
        n, e, _ = lfr(1000, 0.4)
    g = orc.EdgeGraph.from_lines(n, e)
    for seed in (3, 4, 5):
        a = device_infomap(fcmod, n, e, 1, seed=seed, trials=1)
        b = device_infomap(fcmod, n, e, 1, seed=seed, trials=1)
        assert np.array_equal(a, b) and a.shape == (1, n)
        Ld = codelength(n, e, a[0])
        Lr = [orc.infomap(g, seed=s, trials=1)[1] for s in range(8)]
        print("infomap %s one trial: device L %.4f | restatement single trials %.4f..%.4f" % (
            graph, Ld, min(Lr), max(Lr)))
        assert Ld <= max(Lr) * 1.01


@pytest.mark.gpu
def test_infomap_community_ordered_numbering(fcmod):
    """FC_OPT_RELABEL = 2 (the numbering infomap runs use, core.relabel_for): the internal ids
    follow the communities of a one-replica ordering run -- a bijection, neighbours mostly
    numbered close together -- and the device Infomap on it stays within the tolerances of
    test_infomap_lfr1k_vs_restatement (mean codelength within 0.5 %, NMI >= restatement - 0.02);
    a whole infomap run on it equals the sharded driver's."""
    from fastconsensus_amd.distributed import run_sharded
    n, e, planted = lfr(1000, 0.4)
    g = orc.EdgeGraph.from_lines(n, e)
    with fcmod.Engine(seed=11) as eng:
        eng.set_option("relabel", 2)
        eng.load_graph(n, e[:, 0], e[:, 1])
        sigma = eng.node_map()
        assert np.array_equal(np.sort(sigma), np.arange(n))
        gap = np.median(np.abs(sigma[e[:, 0]] - sigma[e[:, 1]]))
        eng.cd(4, 0, 16, 16, 0)
        dev = eng.get_labels(16)
        eng.set_option("infomap_trials", 2)
        labels, st = eng.run(4, 8, 0.6, 0.02)
        sh, st2 = run_sharded(eng, 4, 8, 0.6, 0.02)
    ref = [orc.infomap(g, seed=s)[0] for s in range(8)]
    Ld = np.mean([codelength(n, e, x) for x in dev])
    Lr = np.mean([codelength(n, e, x) for x in ref])
    nd = np.mean([nmi(planted, x) for x in dev])
    nr = np.mean([nmi(planted, x) for x in ref])
    print("relabel 2: median neighbour id gap %d (random numbering ~%d); L %.4f vs %.4f, NMI %.4f vs %.4f"
          % (gap, n // 3, Ld, Lr, nd, nr))
    assert gap < n // 10
    assert abs(Ld - Lr) <= 0.005 * Lr and nd >= nr - 0.02
    assert np.array_equal(labels, sh) and st2["iterations"] == st["iterations"]


@pytest.mark.gpu
def test_infomap_sharding_independent_and_deterministic(fcmod):
    n, e, _ = lfr(1000, 0.4)
    full = device_infomap(fcmod, n, e, 6, seed=99, trials=3)
    again = device_infomap(fcmod, n, e, 6, seed=99, trials=3)
    part = device_infomap(fcmod, n, e, 2, seed=99, rbegin=2, total=6, trials=3)
    assert np.array_equal(full, again)
    assert np.array_equal(full[2:4], part)


@pytest.mark.gpu
def test_infomap_consensus_run(fcmod):
    """The lpm loop around Infomap: exits after closure (check :309), native == sharded driver."""
    n, e, planted = lfr(1000, 0.4)
    from fastconsensus_amd.distributed import run_sharded
    with fcmod.Engine(seed=7) as eng:
        eng.set_option("infomap_trials", 2)
        eng.load_graph(n, e[:, 0], e[:, 1])
        labels, st = eng.run(4, 8, 0.6, 0.02)
        sh, st2 = run_sharded(eng, 4, 8, 0.6, 0.02)
    assert st["exit_check"] == 2 and st["iterations"] >= 1
    assert np.array_equal(labels, sh) and st2["iterations"] == st["iterations"]
    assert np.mean([nmi(planted, x) for x in labels]) > 0.95


@pytest.mark.gpu
def test_fast_consensus_infomap_and_cli(fcmod, tmp_path):
    import networkx as nx
    G = nx.read_edgelist(golden_io.GOLDEN + "/karate_club.txt", nodetype=int)
    out = fcmod.fast_consensus(G, algorithm="infomap", n_p=4, thresh=0.6, seed=2)
    assert len(out) == 4
    for p in out:
        assert isinstance(p, set) and all(isinstance(c, frozenset) for c in p)
        assert set().union(*p) == set(G.nodes())
    shutil.copy(os.path.join(golden_io.GOLDEN, "karate_club.txt"), tmp_path / "karate.txt")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "fast_consensus.py"), "-f", "karate.txt", "--alg",
                        "infomap", "-np", "3"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    outd = tmp_path / "out_partitions_t0.6_d0.02_np3"     # default tau for infomap: 0.6 (:426)
    assert sorted(os.listdir(outd)) == ["1", "2", "3"]
    assert os.listdir(tmp_path / "memberships_t0.6_d0.02_np3") == []
