"""GPU parity: the HIP path through the C-ABI against the reference's golden vectors and
the CPU oracle.  Bit-exact for all integer work; statistical for community detection
quality (the reference's CD libraries are absent: "parity unpinned").
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import golden_io

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def fcmod():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fastconsensus_amd as fc
    return fc


def dev_i32(n):
    return torch.zeros(max(int(n), 1), dtype=torch.int32, device="cuda")


def as_dict(u, v, w):
    return {(int(a), int(b)): int(c) for a, b, c in zip(u, v, w)}


# ------------------------------------------------------------------------- golden replay
@pytest.mark.parametrize("name", golden_io.CASES)
def test_replay_golden_through_capi(fcmod, name):
    """Recorded labelings + closure samples -> every graph the reference checked, bit-exact
    (weights, keep set, check decisions, closure/repair edges, exit point), plus ages
    identical to the oracle's (they decide the repair tie-break)."""
    case = golden_io.load(name)
    ograph, otraces, ofinal = orc.replay(case.algo, case.N, case.edges_file, case.n_p, case.tau, case.delta,
                                         case.cd_batches, case.pair_batches)
    eng = fcmod.Engine(seed=1)
    e = case.edges_file
    eng.load_graph(case.N, e[:, 0], e[:, 1])
    c = 0
    it = 0
    while True:
        eng.set_labels(case.cd_batches[it])
        m = eng.m
        part = dev_i32(m)
        eng.consensus_partial(case.algo, part)
        conv1, kept, unc = eng.consensus_apply(case.algo, case.n_p, case.tau, case.delta, part)
        ku, kv, kw, kage = eng.get_nextgraph()
        assert len(ku) == kept
        tr = otraces[it]
        np.testing.assert_array_equal(kw, tr["kept"].w)
        np.testing.assert_array_equal(kage, tr["kept"].age)
        if case.algo != 1:
            assert as_dict(ku, kv, kw) == case.check_dict(c)
            assert conv1 == case.checks[c][1]
            c += 1
            if conv1:
                break
        ncand = eng.closure_set_pairs(case.pair_batches[it], it)
        assert ncand == tr["closure"].m
        cnt = dev_i32(ncand)
        if ncand and case.algo != 1:
            eng.closure_partial(cnt)
        conv2, m_new = eng.closure_apply(case.algo, case.n_p, case.delta, cnt if case.algo != 1 else None, it)
        u, v, w, age = eng.get_graph()
        assert as_dict(u, v, w) == case.check_dict(c)
        g2 = ograph[it + 1]
        np.testing.assert_array_equal(age, g2.age)
        assert conv2 == case.checks[c][1]
        c += 1
        it += 1
        if conv2:
            break
    assert c == len(case.checks)
    eng.close()


# ------------------------------------------------------------------------- consensus at scale
@pytest.mark.parametrize("n_p,algo", [(64, 0), (64, 1), (20, 0), (7, 1), (128, 1), (3, 0)])
def test_consensus_update_random_vs_oracle(fcmod, n_p, algo):
    rng = np.random.default_rng(n_p * 7 + algo)
    N, m = 100_000, 600_000
    u = rng.integers(0, N, m).astype(np.int32)
    v = rng.integers(0, N, m).astype(np.int32)
    lab = rng.integers(0, 3, (n_p, N)).astype(np.int32)
    eng = fcmod.Engine(seed=2)
    eng.load_graph(N, u, v)
    g = orc.EdgeGraph.from_lines(N, np.stack([u, v], 1))
    gu, gv, gw, gage = eng.get_graph()
    np.testing.assert_array_equal(gu, g.u)
    np.testing.assert_array_equal(gv, g.v)
    np.testing.assert_array_equal(gage, g.age)
    eng.set_labels(lab)
    part = dev_i32(eng.m)
    eng.consensus_partial(algo, part)
    tau = 0.5 if algo == 0 else 0.8
    conv, kept, unc = eng.consensus_apply(algo, n_p, tau, 0.02, part)
    w_ref = orc.consensus(algo, g, lab, n_p)
    keep = orc.threshold(w_ref, tau, n_p)
    ku, kv, kw, kage = eng.get_nextgraph()
    np.testing.assert_array_equal(ku, g.u[keep])
    np.testing.assert_array_equal(kv, g.v[keep])
    np.testing.assert_array_equal(kw, w_ref[keep])
    oc, ocnt = orc.check(w_ref[keep], n_p, 0.02)
    assert unc == ocnt
    if algo == 0:
        assert conv == oc
    eng.close()


def test_consensus_second_iteration_weights(fcmod):
    """Louvain rule with prior weights not in {0, n_p}: run two consensus rounds."""
    case = golden_io.load("lfr1k_louvain_np20")
    eng = fcmod.Engine(seed=3)
    e = case.edges_file
    eng.load_graph(case.N, e[:, 0], e[:, 1])
    graphs, traces, _ = orc.replay(case.algo, case.N, e, case.n_p, case.tau, case.delta, case.cd_batches,
                                   case.pair_batches)
    # iteration 1 on the reference's post-repair graph: labels of batch 1
    eng.set_labels(case.cd_batches[0])
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    nc = eng.closure_set_pairs(case.pair_batches[0], 0)
    cnt = dev_i32(nc)
    eng.closure_partial(cnt)
    eng.closure_apply(0, case.n_p, case.delta, cnt, 0)
    eng.set_labels(case.cd_batches[1])
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    ku, kv, kw, _ = eng.get_nextgraph()
    np.testing.assert_array_equal(kw, traces[1]["kept"].w)
    # the w + (n_p - 1 - k_last) branch (fast_consensus.py:153-159) with w' > n_p: on the same
    # iteration-1 graph, partition 0 random and every later partition one community, so an edge
    # of prior weight w not in {0, n_p} that partition 0 splits gets w + n_p - 1 > n_p
    g1 = graphs[1]
    assert ((g1.w != 0) & (g1.w != case.n_p) & (g1.w > 1)).any()
    lab2 = np.zeros((case.n_p, case.N), np.int32)
    lab2[0] = np.random.default_rng(5).integers(0, 4, case.N)
    eng.reset_graph()
    eng.set_labels(case.cd_batches[0])
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    eng.closure_set_pairs(case.pair_batches[0], 0)
    eng.closure_partial(cnt)
    eng.closure_apply(0, case.n_p, case.delta, cnt, 0)
    eng.set_labels(lab2)
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    conv, kept, unc = eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    w_ref = orc.consensus(0, g1, lab2, case.n_p)
    keep = orc.threshold(w_ref, case.tau, case.n_p)
    ku, kv, kw, _ = eng.get_nextgraph()
    np.testing.assert_array_equal(ku, g1.u[keep])
    np.testing.assert_array_equal(kv, g1.v[keep])
    np.testing.assert_array_equal(kw, w_ref[keep])
    assert (kw > case.n_p).any(), "no edge took the w + (n_p - 1 - k_last) > n_p branch"
    assert unc == orc.check(w_ref[keep], case.n_p, case.delta)[1]
    eng.close()


# ------------------------------------------------------------------------- CD kernels vs CPU twin
def _twin(eng, algo, N, e, count, r0, iteration, seed, **kw):
    """The CPU twin on the engine's internal numbering (fc_get_node_map), labels returned
    in node order like fc_get_labels."""
    sigma = eng.node_map()
    assert np.array_equal(np.sort(sigma), np.arange(N))
    g_int = orc.EdgeGraph.from_lines(N, np.stack([sigma[e[:, 0]], sigma[e[:, 1]]], 1))
    lab, sw = orc.engine_cd(algo, g_int, count, r0, iteration, seed, **kw)
    return lab[:, sigma], sw


@pytest.mark.parametrize("n,seed", [(1000, 100), (1000, 259), (34, 7), (1_000_003, 42)])
def test_node_map_is_the_oracle_device_sigma(fcmod, n, seed):
    """fc_get_node_map equals orc.device_sigma (graph.hip k_sigma restated), so the CPU model
    predicts a device run of any seed exactly (tools/semantics_dist.py SEM_DEVSIGMA)."""
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n, 4 * n).astype(np.int32)
    v = rng.integers(0, n, 4 * n).astype(np.int32)
    with fcmod.Engine(seed=seed) as eng:
        eng.load_graph(n, u, v)
        np.testing.assert_array_equal(eng.node_map(), orc.device_sigma(n, seed))


def _lfr1k_graph():
    case = golden_io.load("lfr1k_louvain_np20")
    return case, orc.EdgeGraph.from_lines(case.N, case.edges_file)


# tail: FC_OPT_TAIL_VISITS -- 0 keeps every sweep on the multi-kernel path; a huge value
# hands every sweep after the first two to the per-replica tail kernel (classic engine)
TAILS = [0, 1 << 40]
# FC_OPT_CD_ENGINE: 0 classic (cd.hip), 1 replica-lane (cd_rl.hip; twin shared=1, coarsen=0),
# 2 hybrid (twin shared=2): test engine 2 runs the full sweeps on the replica-lane engine
# (rl_min_replicas=1), test engine 3 the same semantics on cd.hip alone (a batch too narrow)
ENGINES = [0, 1, 2, 3]
SHARED = {0: 0, 1: 1, 2: 2, 3: 2}


def _set_engine(eng, engine):
    eng.set_option("cd_engine", min(engine, 2))
    if engine >= 2:
        eng.set_option("rl_min_replicas", 1 if engine == 2 else 1 << 30)
        eng.set_option("rl_min_vertices", 1)


def _engine(eng, engine, tail=0, coarsen=0):
    """Select the CD engine; returns the twin's keyword arguments.  The replica-lane engine has
    no tail kernel or coarse rounds: its tail / coarsen variants are duplicates and skipped."""
    if engine == 1:
        if tail != TAILS[0] or coarsen != 0:
            pytest.skip("replica-lane engine: no tail kernel / coarse rounds")
        eng.set_option("cd_engine", 1)
        return {"shared": 1, "coarsen": 0}
    _set_engine(eng, engine)
    eng.set_option("tail_visits", tail)
    eng.set_option("coarsen", coarsen)
    return {"shared": SHARED[engine], "coarsen": coarsen}


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("coarsen", [0, 8])
@pytest.mark.parametrize("tail", TAILS)
@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("buckets,chunk,prune", [(32, 0, 0), (5, 0, 0), (32, 16, 0), (7, 16, 0), (32, 0, 1),
                                                 (5, 16, 1)])
def test_cd_bit_exact_vs_twin(fcmod, algo, buckets, chunk, prune, tail, coarsen, engine):
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=99)
    kw = _engine(eng, engine, tail, coarsen)
    eng.set_params(buckets=buckets)
    eng.set_option("chunk", chunk)
    eng.set_option("prune", prune)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    n_r = 6
    eng.cd(algo, 0, n_r, n_r, 4)
    got = eng.get_labels(n_r)
    exp, sw = _twin(eng, algo, case.N, case.edges_file, n_r, 0, 4, 99, buckets=buckets, chunk=chunk, prune=prune, **kw)
    np.testing.assert_array_equal(got, exp)
    # sharding invariance: replicas 2..4 alone give the same labelings
    eng.cd(algo, 2, 3, n_r, 4)
    np.testing.assert_array_equal(eng.get_labels(3), exp[2:5])
    # renumbered output
    np.testing.assert_array_equal(eng.get_labels(3, renumber=True), orc.renumber(exp[2:5]))
    eng.close()


@pytest.mark.parametrize("algo", [0, 1])
def test_cd_hybrid_many_buckets_falls_back(fcmod, algo):
    """FC_OPT_BUCKETS past what the replica-lane sweep record holds (339 buckets x 6 degree
    classes in the pinned scratch): the hybrid runs the batch on cd.hip with the same
    semantics instead of failing, bit-exact against the twin."""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=61)
    kw = _engine(eng, 2, 0, 0)
    eng.set_params(buckets=512)
    eng.set_option("chunk", 0)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(algo, 0, 9, 9, 2)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, 9, 0, 2, 61, buckets=512, chunk=0, prune=1, **kw)
    np.testing.assert_array_equal(eng.get_labels(9), exp)
    eng.close()


@pytest.mark.parametrize("engine", [2, 3])
@pytest.mark.parametrize("dense_div", [0, 2, 4, 16])
@pytest.mark.parametrize("algo", [0, 1])
def test_cd_hybrid_dense_lists_bit_exact_vs_twin(fcmod, algo, dense_div, engine):
    """FC_OPT_DENSE_DIV: a filtered sweep whose list still holds >= N/dense_div vertices keeps the
    shared order in single-bucket rounds (0: only full sweeps do) -- on the replica-lane kernels
    (engine 2) and on cd.hip alone (3), the input graph and a weighted consensus graph."""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=57)
    kw = _engine(eng, engine, 0, 8)
    eng.set_option("dense_div", dense_div)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(algo, 0, 12, 12, 5)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, 12, 0, 5, 57, dense_div=dense_div, **kw)
    np.testing.assert_array_equal(eng.get_labels(12), exp)
    eng.close()
    case, eng = _weighted_consensus_engine(fcmod, 59)
    kw = _engine(eng, engine, 0, 8)
    eng.set_option("dense_div", dense_div)
    u, v, w, _ = eng.get_graph()
    sigma = eng.node_map()
    a_, b_ = sigma[u], sigma[v]
    lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
    o = np.lexsort((hi, lo))
    g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
    eng.cd(algo, 0, 12, 12, 6)
    exp, _ = orc.engine_cd(algo, g_int, 12, 0, 6, 59, dense_div=dense_div, **kw)
    np.testing.assert_array_equal(eng.get_labels(12), exp[:, sigma])
    eng.close()


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("n_r", [1, 13, 33, 64, 70, 130])
def test_cd_replica_lanes_bit_exact_vs_twin(fcmod, algo, n_r):
    """Replica-lane engine at every lane layout: lane groups of 8 (up to 8 vertices per wave),
    16, 64, and banks of 64 past 64 local replicas; a shard [r0, r0 + k) of a larger batch."""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=41)
    eng.set_option("cd_engine", 1)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(algo, 0, n_r, n_r, 1)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, n_r, 0, 1, 41, shared=1, coarsen=0)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp)
    if n_r > 2:
        k = n_r // 2
        eng.cd(algo, 1, k, n_r, 1)
        np.testing.assert_array_equal(eng.get_labels(k), exp[1:1 + k])
    eng.close()


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("visit_div", ["0", "1000000"])
@pytest.mark.parametrize("n_r", [6, 64, 70])
def test_cd_replica_lanes_visit_mode_bit_exact(fcmod, algo, visit_div, n_r, monkeypatch):
    """Replica-lane engine with its sparse-sweep visit mode never (0) / always (huge) chosen:
    one lane per (entry, replica) visit decides exactly as a wave per entry; weighted
    consensus graph too (Leiden-style marks)."""
    monkeypatch.setenv("FC_RL_VISIT_DIV", visit_div)
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=43)
    eng.set_option("cd_engine", 1)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(algo, 0, n_r, n_r, 2)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, n_r, 0, 2, 43, shared=1, coarsen=0)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp)
    eng.close()
    case, eng = _weighted_consensus_engine(fcmod, 47)
    eng.set_option("cd_engine", 1)
    u, v, w, _ = eng.get_graph()
    sigma = eng.node_map()
    a_, b_ = sigma[u], sigma[v]
    lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
    o = np.lexsort((hi, lo))
    g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
    eng.cd(algo, 0, n_r, n_r, 3)
    exp, _ = orc.engine_cd(algo, g_int, n_r, 0, 3, 47, shared=1, coarsen=0)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp[:, sigma])
    eng.close()


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("coarsen", [0, 8])
@pytest.mark.parametrize("tail", TAILS)
@pytest.mark.parametrize("algo", [0, 1])
def test_cd_unit_prune_mark2_bit_exact_vs_twin(fcmod, algo, tail, coarsen, engine):
    """FC_OPT_PRUNE_MARK=2: the sweep-end marks (k_mark_lm) on the unit-weight input graph too."""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=23)
    kw = _engine(eng, engine, tail, coarsen)
    eng.set_option("prune_mark", 2)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(algo, 0, 6, 6, 2)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, 6, 0, 2, 23, prune_mark=2, **kw)
    np.testing.assert_array_equal(eng.get_labels(6), exp)
    eng.close()


def _heavy_graph(seed, hub_deg):
    """Communities + a few hubs whose degree exceeds the light (64) and LDS (2048) paths."""
    rng = np.random.default_rng(seed)
    N = 6000
    blocks = rng.integers(0, 60, N)
    u = rng.integers(0, N, 60000)
    v = rng.integers(0, N, 60000)
    same = blocks[u] == blocks[v]
    keep = same | (rng.random(len(u)) < 0.2)
    u, v = u[keep], v[keep]
    hubs = []
    for h in range(4):
        nb = rng.choice(N, hub_deg, replace=False)
        hubs.append(np.stack([np.full(hub_deg, h), nb], 1))
    e = np.concatenate([np.stack([u, v], 1)] + hubs).astype(np.int32)
    return N, e


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("tail", TAILS)
@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("hub_deg,chunk,prune", [(300, 0, 0), (3000, 0, 0), (3000, 16, 0), (3000, 0, 1)])
def test_cd_heavy_rows_bit_exact(fcmod, algo, hub_deg, chunk, prune, tail, engine):
    N, e = _heavy_graph(5, hub_deg)
    eng = fcmod.Engine(seed=7)
    kw = _engine(eng, engine, tail)
    eng.set_option("chunk", chunk)
    eng.set_option("prune", prune)
    eng.load_graph(N, e[:, 0], e[:, 1])
    eng.cd(algo, 0, 4, 4, 1)
    got = eng.get_labels(4)
    exp, _ = _twin(eng, algo, N, e, 4, 0, 1, 7, chunk=chunk, prune=prune, **kw)
    np.testing.assert_array_equal(got, exp)
    eng.close()


def _weighted_consensus_engine(fcmod, seed):
    """An engine holding a weighted consensus graph (weights 0..n_p): one louvain iteration of
    the step API on LFR-1k with the reference run's recorded labelings and closure pairs."""
    case = golden_io.load("lfr1k_louvain_np20")
    eng = fcmod.Engine(seed=seed)
    e = case.edges_file
    eng.load_graph(case.N, e[:, 0], e[:, 1])
    eng.set_labels(case.cd_batches[0])
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    nc = eng.closure_set_pairs(case.pair_batches[0], 0)
    cnt = dev_i32(nc)
    eng.closure_partial(cnt)
    eng.closure_apply(0, case.n_p, case.delta, cnt, 0)
    return case, eng


@pytest.mark.parametrize("groups", ["2", "3", "4", "5"])
@pytest.mark.parametrize("n_r", [6, 64])
@pytest.mark.parametrize("algo", [0, 1])
def test_cd_replica_lanes_class_groups_bit_exact(fcmod, algo, n_r, groups, monkeypatch):
    """The replica-lane decide's degree classes (16 | 24 | 32 | 48 | 64 keys) launched one per
    class or merged into the wider network (FC_RL_GROUPS_LOUV / _LPA = 3, 4, 5): the same
    decisions whichever network sorts a row -- bit-exact against the twin, per-lane rows (6
    replicas) and one unit per wave (64), on the input graph and a weighted consensus graph."""
    monkeypatch.setenv("FC_RL_GROUPS_LOUV", groups)
    monkeypatch.setenv("FC_RL_GROUPS_LPA", groups)
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=71)
    kw = _engine(eng, 1)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    deg = np.bincount(case.edges_file.ravel(), minlength=case.N)
    assert deg.max() > 24 and ((deg > 16) & (deg <= 24)).any() and ((deg > 32) & (deg <= 48)).any()
    eng.cd(algo, 0, n_r, n_r, 2)
    exp, _ = _twin(eng, algo, case.N, case.edges_file, n_r, 0, 2, 71, **kw)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp)
    eng.close()
    case, eng = _weighted_consensus_engine(fcmod, 73)
    eng.set_option("cd_engine", 1)
    u, v, w, _ = eng.get_graph()
    sigma = eng.node_map()
    a_, b_ = sigma[u], sigma[v]
    lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
    o = np.lexsort((hi, lo))
    g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
    eng.cd(algo, 0, n_r, n_r, 3)
    exp, _ = orc.engine_cd(algo, g_int, n_r, 0, 3, 73, shared=1, coarsen=0)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp[:, sigma])
    eng.close()


@pytest.mark.parametrize("u1", ["0", "1"])
@pytest.mark.parametrize("n_r", [64, 70])
def test_cd_replica_lanes_wide_weights_bit_exact(fcmod, n_r, u1, monkeypatch):
    """Consensus weights past 8 bits (300 labelings: weights up to 300) take the replica-lane
    decide's separate weight row (WM_WIDE); with >= 64 local replicas one unit per wave, its row
    read an item ahead (FC_RL_U1=1) or per lane (0): both bit-exact against the twin."""
    monkeypatch.setenv("FC_RL_U1", u1)
    case = golden_io.load("lfr1k_louvain_np20")
    eng = fcmod.Engine(seed=53)
    e = case.edges_file
    eng.load_graph(case.N, e[:, 0], e[:, 1])
    n_w = 300
    eng.set_labels(np.tile(case.cd_batches[0], (n_w // case.n_p, 1)))
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, n_w, case.tau, case.delta, part)
    nc = eng.closure_set_pairs(case.pair_batches[0], 0)
    cnt = dev_i32(nc)
    eng.closure_partial(cnt)
    eng.closure_apply(0, n_w, case.delta, cnt, 0)
    eng.set_option("cd_engine", 1)
    u, v, w, _ = eng.get_graph()
    assert w.max() >= 256, "no weight past 8 bits"
    sigma = eng.node_map()
    a_, b_ = sigma[u], sigma[v]
    lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
    o = np.lexsort((hi, lo))
    g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
    eng.cd(0, 0, n_r, n_r, 3)
    exp, _ = orc.engine_cd(0, g_int, n_r, 0, 3, 53, shared=1, coarsen=0)
    np.testing.assert_array_equal(eng.get_labels(n_r), exp[:, sigma])
    eng.close()


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("coarsen", [0, 8])
@pytest.mark.parametrize("tail", TAILS)
@pytest.mark.parametrize("prune_mark", [0, 1])
@pytest.mark.parametrize("algo", [0, 1])
def test_cd_weighted_prune_mark_bit_exact_vs_twin(fcmod, algo, prune_mark, tail, coarsen, engine):
    """CD (Louvain and LPA) on a weighted consensus graph, where FC_OPT_PRUNE_MARK=1 (default) tracks from sweep 1
    and marks at sweep end only the neighbours that ended in another community (k_mark_lm, and
    the tail kernel's mover list): bit-exact against the twin in both modes, on both engines, on
    the multi-kernel path and the tail kernel, with and without coarse rounds."""
    case, eng = _weighted_consensus_engine(fcmod, 31)
    kw = _engine(eng, engine, tail, coarsen)
    eng.set_option("prune_mark", prune_mark)
    u, v, w, _ = eng.get_graph()
    assert w.max() > 1
    sigma = eng.node_map()
    a, b = sigma[u], sigma[v]
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    o = np.lexsort((hi, lo))
    g_int = orc.EdgeGraph(case.N, lo[o], hi[o], w[o], np.zeros(len(o), np.int64))
    n_r = 6
    eng.cd(algo, 0, n_r, n_r, 3)
    got = eng.get_labels(n_r)
    exp, _ = orc.engine_cd(algo, g_int, n_r, 0, 3, 31, prune_mark=prune_mark, **kw)
    np.testing.assert_array_equal(got, exp[:, sigma])
    eng.close()


def test_louvain_quality_vs_sequential_restatement(fcmod):
    """Statistical parity of Louvain level 0: modularity and NMI within tolerance of the
    python-louvain restatement (tolerances: dQ 0.01 on the mean, NMI 0.03)."""
    from sklearn.metrics import normalized_mutual_info_score as nmi
    case, g = _lfr1k_graph()
    planted = np.load(golden_io.GOLDEN + "/lfr1k_mu04_planted.npy")[case.z["nodes"]]
    eng = fcmod.Engine(seed=11)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.cd(0, 0, 16, 16, 0)
    lab = eng.get_labels(16)
    q = np.mean([orc.modularity(g, l) for l in lab])
    s = np.mean([nmi(planted, l) for l in lab])
    ref, _ = orc.cd_batch(0, 16, g, seed=5)
    q_ref = np.mean([orc.modularity(g, l) for l in ref])
    s_ref = np.mean([nmi(planted, l) for l in ref])
    assert q > q_ref - 0.01, (q, q_ref)
    assert s > s_ref - 0.03, (s, s_ref)
    eng.close()


# ------------------------------------------------------------------------- end to end
def test_run_lfr1k_well_formed(fcmod):
    """A whole run: shape, statistics, and labels renumbered 0..k-1 by first node.  (Consensus
    quality against the reference loop: tests/test_gpu_cd_parity.py.)"""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=21)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    labels, st = eng.run(0, 20, 0.2, 0.02)
    assert labels.shape == (20, case.N)
    assert st["iterations"] >= 1 and st["partition_edges"] > 0 and st["exit_check"] in (1, 2)
    for l in labels:
        assert l[0] == 0 and l.max() == len(np.unique(l)) - 1
        first = np.unique(l, return_index=True)[1]
        assert np.all(np.diff(first) > 0)          # community c first appears before c + 1
    eng.close()


def test_fast_consensus_networkx_dropin(fcmod):
    import networkx as nx
    G = nx.read_edgelist(golden_io.GOLDEN + "/karate_club.txt", nodetype=int)
    out = fcmod.fast_consensus(G, algorithm="louvain", n_p=10, thresh=0.2, delta=0.1, seed=3)
    assert len(out) == 10 and all(set(p) == set(G.nodes()) for p in out)
    assert list(out[0].keys()) == list(G.nodes())
    out = fcmod.fast_consensus(G, algorithm="lpm", n_p=6, thresh=0.8, delta=0.02, seed=3)
    assert len(out) == 6
    for p in out:
        assert isinstance(p, set) and all(isinstance(c, frozenset) for c in p)
        assert set().union(*p) == set(G.nodes())
    assert fcmod.fast_consensus(G, algorithm="unknown", n_p=2) is None
    with pytest.raises(NotImplementedError):
        fcmod.fast_consensus(G, algorithm="cnm", n_p=2)


def test_determinism_same_seed(fcmod):
    case, _ = _lfr1k_graph()
    res = []
    for _ in range(2):
        eng = fcmod.Engine(seed=1234)
        eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
        labels, st = eng.run(0, 8, 0.2, 0.02)
        res.append((labels, eng.get_graph()))
        eng.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        np.testing.assert_array_equal(a, b)


def test_run_into_caller_buffer(fcmod):
    """run(out=...) writes the same labelings into a reused host array (bench.py's path)."""
    case, _ = _lfr1k_graph()
    with fcmod.Engine(seed=99) as eng:
        eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
        ref, st_ref = eng.run(0, 8, 0.2, 0.02)
        out = np.full((8, case.N), -7, np.int32)
        for _ in range(2):
            got, st = eng.run(0, 8, 0.2, 0.02, out=out)
            assert got is out
            assert {k: v for k, v in st.items() if not k.endswith("_ms")} == \
                {k: v for k, v in st_ref.items() if not k.endswith("_ms")}
            np.testing.assert_array_equal(out, ref)
        with pytest.raises(ValueError):
            eng.run(0, 8, 0.2, 0.02, out=np.zeros((7, case.N), np.int32))


def test_closure_sampler_properties(fcmod):
    """Device closure: every new edge joins two neighbours of some node in the GROWING graph
    (post-threshold graph plus the closure edges of earlier attempt blocks,
    fast_consensus.py:175-184), was absent from the post-threshold graph, and carries the
    co-membership count (:186-190)."""
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=5)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    lab = case.cd_batches[0]
    eng.set_labels(lab)
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    ku, kv, kw, _ = eng.get_nextgraph()
    kept = set(zip(ku.tolist(), kv.tolist()))
    nbrs = [set() for _ in range(case.N)]
    for a, b in kept:
        nbrs[a].add(b)
        nbrs[b].add(a)
    nc = eng.closure_sample(g.m, 0)
    assert nc > 0
    cnt = dev_i32(nc)
    eng.closure_partial(cnt)
    eng.closure_apply(0, case.n_p, case.delta, cnt, 0)
    u, v, w, age = eng.get_graph()
    new = [(a, b, c, t) for a, b, c, t in zip(u, v, w, age) if (a, b) not in kept]
    closure = [x for x in new if ((x[3] >> 40) == 1) and not (x[3] & (1 << 39))]
    assert len(closure) == nc
    for a, b, _, _ in closure:
        nbrs[a].add(b)
        nbrs[b].add(a)
    for a, b, c, _ in closure[:2000]:
        assert (nbrs[a] & nbrs[b]) - {a, b}, "closure edge must close a 2-path"
        assert c == int((lab[:, a] == lab[:, b]).sum())
    eng.close()


# ------------------------------------------------------------------------- whole runs, bit-exact
@pytest.mark.parametrize("algo,n_p,tau,chunk,prune,relabel,tail",
                         [(0, 10, 0.2, 0, 0, 0, 0), (0, 12, 0.2, 16, 0, 1, 16384), (1, 4, 0.8, 0, 0, 0, 16384),
                          (0, 20, 0.2, 0, 0, 1, 0), (0, 10, 0.2, 0, 1, 1, 16384), (1, 6, 0.8, 16, 1, 1, 0),
                          (1, 6, 0.8, 16, 1, 1, 16384), (0, 10, 0.2, 16, 1, 1, 0), (0, 10, 0.2, 16, 1, 1, 16384),
                          (2, 10, 0.2, 16, 1, 1, 16384), (2, 12, 0.2, 0, 0, 0, 0),
                          (0, 10, 0.2, 16, 1, 2, 0), (1, 6, 0.8, 16, 1, 2, 16384),
                          # 64 replicas: one unit per wave in the replica-lane decide (rl_sorted_u1)
                          (0, 64, 0.2, 16, 1, 1, 0), (1, 64, 0.8, 16, 1, 1, 0)])
@pytest.mark.parametrize("engine", ENGINES)
def test_full_run_bit_exact_vs_cpu_model(fcmod, algo, n_p, tau, chunk, prune, relabel, tail, engine):
    """fc_run on the device == the oracle-backed CPU model of the engine driven by the same
    loop (bucketed CD twin, consensus rule, Philox closure sampler, repair, ages): final
    partitions AND the final graph are identical (n_p=10 runs 9 iterations)."""
    from fastconsensus_amd.distributed import run_sharded
    from tests.cpu_engine import OracleEngine
    case, _ = _lfr1k_graph()
    e = case.edges_file
    eng = fcmod.Engine(seed=17)
    _set_engine(eng, engine)
    if engine != 1:
        eng.set_option("tail_visits", tail)
    elif tail:
        pytest.skip("replica-lane engine: no tail kernel")
    eng.set_option("chunk", chunk)
    eng.set_option("prune", prune)
    eng.set_option("relabel", relabel)
    eng.set_params(max_iters=50)
    eng.load_graph(case.N, e[:, 0], e[:, 1])
    sigma = eng.node_map()
    if not relabel:
        assert np.array_equal(sigma, np.arange(case.N))
    cpu = OracleEngine(seed=17, chunk=chunk, prune=prune, sigma=sigma, shared=SHARED[engine],
                       coarsen=0 if engine == 1 else 8)
    cpu.load_graph(case.N, e[:, 0], e[:, 1])
    exp_labels, exp_st = run_sharded(cpu, algo, n_p, tau, 0.02, device="cpu", max_iters=50)
    labels, st = eng.run(algo, n_p, tau, 0.02)
    assert st["iterations"] == exp_st["iterations"]
    assert st["partition_edges"] == exp_st["partition_edges"]
    np.testing.assert_array_equal(labels, exp_labels)
    for a, b in zip(eng.get_graph(), cpu.get_graph()):
        np.testing.assert_array_equal(a, b)
    # the Python sharded driver (world = 1, torch stream) == the native driver
    labels2, st2 = run_sharded(eng, algo, n_p, tau, 0.02, device="cuda", max_iters=50)
    np.testing.assert_array_equal(labels2, labels)
    assert st2["partition_edges"] == st["partition_edges"]
    eng.close()


@pytest.mark.parametrize("algo", [0, 1, 2])
def test_label_storage_order_is_storage_only(fcmod, algo):
    """FC_OPT_STORE (label rows in community order, from a Louvain run at load) changes
    where labels live, never a decision: identical partitions and final graph with it off."""
    case, _ = _lfr1k_graph()
    e = case.edges_file
    out = []
    for store in (0, 1):
        eng = fcmod.Engine(seed=5)
        eng.set_option("store", store)
        eng.load_graph(case.N, e[:, 0], e[:, 1])
        labels, st = eng.run(algo, 10, 0.2 if algo != 1 else 0.8, 0.02)
        out.append((labels, st["iterations"], eng.get_graph()))
        eng.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
    for a, b in zip(out[0][2], out[1][2]):
        np.testing.assert_array_equal(a, b)


# ------------------------------------------------------------------------- full BASELINE sizes
@pytest.fixture(scope="module")
def lfr1m():
    from fastconsensus_amd import synth
    u, v, planted = synth.lfr(1_000_000, 0.5, seed=42)
    return 1_000_000, u, v, planted


def test_c4_consensus_update_bit_exact_full_size(fcmod, lfr1m):
    """BASELINE configs[3] size (n=1M, m~13.8M, n_p=64): one consensus update on device
    labelings (64 Louvain replicas) is bit-exact against the oracle's literal rule."""
    n, u, v, _ = lfr1m
    eng = fcmod.Engine(seed=3)
    eng.load_graph(n, u, v)
    eng.cd(0, 0, 64, 64, 0)
    lab = eng.get_labels(64)
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    conv, kept, unc = eng.consensus_apply(0, 64, 0.2, 0.02, part)
    g = orc.EdgeGraph.from_lines(n, np.stack([u, v], 1))
    w_ref = orc.consensus(0, g, lab, 64)
    keep = orc.threshold(w_ref, 0.2, 64)
    ku, kv, kw, _ = eng.get_nextgraph()
    assert kept == int(keep.sum())
    np.testing.assert_array_equal(kw, w_ref[keep])
    np.testing.assert_array_equal(ku, g.u[keep])
    assert (conv, unc) == orc.check(w_ref[keep], 64, 0.02)
    eng.close()


def test_c4_run_properties_full_size(fcmod, lfr1m):
    """Whole louvain consensus at the metric's size: deterministic for a seed, partitions are
    well-formed, every node is covered, and NMI to the planted communities is high."""
    from sklearn.metrics import normalized_mutual_info_score as nmi
    n, u, v, planted = lfr1m
    outs = []
    for _ in range(2):
        eng = fcmod.Engine(seed=11)
        eng.load_graph(n, u, v)
        labels, st = eng.run(0, 64, 0.2, 0.02)
        outs.append((labels, st, eng.get_graph()[2].sum()))
        eng.close()
    (l1, s1, w1), (l2, s2, w2) = outs
    np.testing.assert_array_equal(l1, l2)
    assert s1["partition_edges"] == s2["partition_edges"] and w1 == w2
    assert s1["exit_check"] in (1, 2) and not s1["hit_iter_cap"]
    for row in l1[:4]:
        assert row.min() == 0 and row[0] == 0 and row.max() + 1 == len(np.unique(row))
    assert nmi(planted, l1[0]) > 0.8


def test_repair_many_isolates_bit_exact(fcmod):
    """Isolate repair (fast_consensus.py:193-195) with more isolates than the single-workgroup
    fixpoint holds (k > 16384: the multi-block Jacobi path) and with few (LDS path): one
    consensus iteration through the step API on a sparse random graph, device == CPU model
    (graph, weights, ages)."""
    from tests.cpu_engine import OracleEngine
    for N, m in ((60_000, 45_000), (6_000, 4_500)):
        rng = np.random.default_rng(N)
        u = rng.integers(0, N, m).astype(np.int32)
        v = rng.integers(0, N, m).astype(np.int32)
        lab = rng.integers(0, 3, (4, N)).astype(np.int32)
        eng = fcmod.Engine(seed=9)
        eng.set_option("relabel", 0)
        eng.load_graph(N, u, v)
        cpu = OracleEngine(seed=9)
        cpu.load_graph(N, u, v)
        eng.set_labels(lab)
        cpu.lab = lab.copy()
        cpu.r0 = 0
        part = dev_i32(eng.m)
        eng.consensus_partial(0, part)
        eng.consensus_apply(0, 4, 0.8, 0.02, part)
        cpart = torch.zeros(cpu.m + 1, dtype=torch.int32)
        cpu.consensus_partial(0, cpart)
        cpu.consensus_apply(0, 4, 0.8, 0.02, cpart)
        nc = eng.closure_sample(m, 0)
        assert nc == cpu.closure_sample(m, 0)
        cnt = dev_i32(nc)
        eng.closure_partial(cnt)
        ccnt = torch.zeros(max(nc, 1), dtype=torch.int32)
        cpu.closure_partial(ccnt)
        _, m1 = eng.closure_apply(0, 4, 0.02, cnt, 0)
        _, cm1 = cpu.closure_apply(0, 4, 0.02, ccnt, 0)
        assert m1 == cm1
        deg = np.bincount(np.concatenate([cpu.kept.u, cpu.kept.v]), minlength=N)
        print("N %d: kept %d, isolated after threshold %d, closure %d, graph %d" % (N, cpu.kept.m, int((deg == 0).sum()), nc, m1))
        for a, b in zip(eng.get_graph(), cpu.get_graph()):
            np.testing.assert_array_equal(a, b)
        eng.close()


def _sharded_closure(eng, attempts, world, order_rng):
    """distributed._closure_sharded's schedule on ONE engine: every block's W sub-ranges drawn
    one after the other (the ranks), their lists concatenated in a shuffled rank order."""
    blocks = eng.closure_begin(attempts, 0)
    for b in range(blocks):
        t0, t1 = attempts * b // blocks, attempts * (b + 1) // blocks
        lists = []
        for r in range(world):
            lo, hi = t0 + (t1 - t0) * r // world, t0 + (t1 - t0) * (r + 1) // world
            buf = torch.empty(2 * max(hi - lo, 1), dtype=torch.int64, device="cuda")
            k = eng.closure_block_sample(b, lo, hi, buf)
            lists.append(buf[:2 * k].clone())
        order = order_rng.permutation(world)
        allp = torch.cat([lists[g] for g in order]) if lists else None
        eng.closure_block_add(b, allp, int(allp.numel() // 2))
    return eng.closure_finish()


@pytest.mark.parametrize("world", [1, 3, 8])
def test_closure_sharded_equals_single(fcmod, world):
    """The multi-GPU closure (each block's attempts split over W ranks, lists all-gathered,
    fc_closure_block_add) leaves exactly fc_closure_sample's candidates: graph, weights and
    ages after closure_apply equal the single-rank device run (itself pinned to the CPU model
    by test_repair_many_isolates_bit_exact and the full-run tests)."""
    case, g = _lfr1k_graph()
    lab = case.cd_batches[0]
    graphs = []
    for sharded in (False, True):
        eng = fcmod.Engine(seed=5)
        eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
        eng.set_labels(lab)
        part = dev_i32(eng.m)
        eng.consensus_partial(0, part)
        eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
        nc = _sharded_closure(eng, g.m, world, np.random.default_rng(world)) if sharded else \
            eng.closure_sample(g.m, 0)
        assert nc > 0
        cnt = dev_i32(nc)
        eng.closure_partial(cnt)
        eng.closure_apply(0, case.n_p, case.delta, cnt, 0)
        graphs.append(eng.get_graph())
        eng.close()
    for a, b in zip(*graphs):
        np.testing.assert_array_equal(a, b)
    print("W=%d: %d candidates, graph %d edges" % (world, nc, len(graphs[1][0])))


def test_closure_block_api_errors(fcmod):
    """Blocks must go in order, ranges must lie inside their block, outputs must be large
    enough (FastConsensusError, nothing drawn)."""
    from fastconsensus_amd import FastConsensusError
    case, g = _lfr1k_graph()
    eng = fcmod.Engine(seed=5)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    eng.set_labels(case.cd_batches[0])
    part = dev_i32(eng.m)
    eng.consensus_partial(0, part)
    eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)
    buf = torch.empty(2 * g.m, dtype=torch.int64, device="cuda")
    with pytest.raises(FastConsensusError):
        eng.closure_block_sample(0, 0, 10, buf)                    # before closure_begin
    blocks = eng.closure_begin(g.m, 0)
    assert blocks == orc.closure_rounds(0)                          # the default block count (fc_ctx.h closure_blocks)
    t1 = g.m // blocks
    with pytest.raises(FastConsensusError):
        eng.closure_block_sample(1, t1, t1 + 5, buf)               # block 0 not added yet
    with pytest.raises(FastConsensusError):
        eng.closure_block_sample(0, 0, t1 + 1, buf)                # past the block
    with pytest.raises(FastConsensusError):
        eng.closure_finish()                                       # blocks missing
    # a begun sequence goes stale when the one-rank sampler, a consensus update or a graph
    # reset runs in between (they reset the table and the graph the blocks read)
    for stale in (lambda: eng.closure_sample(g.m, 0), lambda: eng.reset_graph(),
                  lambda: eng.consensus_apply(0, case.n_p, case.tau, case.delta, part)):
        eng.closure_begin(g.m, 0)
        stale()
        with pytest.raises(FastConsensusError):
            eng.closure_block_sample(0, 0, 10, buf)
    eng.close()
