"""The closure sampler's one documented deviation, measured against the reference.

The reference samples its L = m attempts SEQUENTIALLY from the growing graph
(fast_consensus.py:175-190 louvain, :292-304 lpm): a closure edge added by attempt t is a
neighbour for attempt t+1 and `has_edge` sees it.  The device runs the L attempts in 8
consecutive blocks; a block draws in parallel from the post-threshold graph plus every
closure edge the earlier blocks found (consensus.hip k_closure_sample, restated bit-exactly
by the twin; tests/test_gpu_cd_parity.py checks the device against it).

For every golden iteration the reference ran, the reference's own closure (its recorded
samples on its kept graph) is compared with the device sampler on the SAME kept graph over
8 seeds.  Measured (this file prints it): LFR-1k louvain it 0 (the kept graph of 5,252 edges
more than doubles during closure) 5,951 reference candidates vs 6,065 +- 42 device (+1.9 %;
a sequential restatement averages 6,124 over 6 seeds: the reference's one sample is low;
16 blocks give 6,070, LFR-1M shows no difference from 2 blocks up); LFR-1k lpm 12,417 vs
12,401 +- 44; mean closure weight 19.61 vs 19.60.  With ONE block
(every attempt from the post-threshold graph, round 1's sampler) the count was 5,647 (-5.1 %)
and the whole consensus lost ~0.025 NMI against the reference loop on LFR-1k
(tests/test_engine_semantics.py).  Tolerances: candidate count within 4 % of the reference
(LFR-1k), mean co-membership weight of the closure edges within 3 % (louvain).  Karate
(6-13 candidates) is printed only.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import golden_io


def _measure(name, seeds=8):
    case = golden_io.load(name)
    graphs, traces, _ = orc.replay(case.algo, case.N, case.edges_file, case.n_p, case.tau, case.delta,
                                   case.cd_batches, case.pair_batches)
    L = graphs[0].m
    rows = []
    for it, tr in enumerate(traces):
        if "closure" not in tr:
            continue
        kept = tr["kept"]
        cnt, wmean = [], []
        for s in range(seeds):
            pairs = orc.closure_sample_pairs(kept, L, s, it, orc.closure_rounds(case.algo))
            cu, _, cw, _ = orc.closure_from_pairs(case.algo, kept, pairs, case.cd_batches[it], case.n_p)
            cnt.append(len(cu))
            wmean.append(float(cw.mean()) if len(cw) else 0.0)
        ref = tr["closure"]
        rows.append({"it": it, "kept": kept.m, "ref": ref.m, "dev": float(np.mean(cnt)), "sd": float(np.std(cnt)),
                     "ref_w": float(ref.w.mean()) if ref.m else 0.0, "dev_w": float(np.mean(wmean))})
    return case, rows


@pytest.mark.parametrize("name", ["lfr1k_louvain_np20", "lfr1k_lpm_np20"])
def test_closure_candidates_vs_reference_sequential_sampler(name):
    case, rows = _measure(name)
    assert rows
    for r in rows:
        print(name, r)
        assert abs(r["dev"] - r["ref"]) <= 0.04 * r["ref"], r
        if case.algo != 1:
            assert abs(r["dev_w"] - r["ref_w"]) <= 0.03 * r["ref_w"], r
        else:
            assert r["ref_w"] == 0.0 and r["dev_w"] == 0.0      # lpm closure weight is always 0 (:302-304)


def test_closure_small_graph_printed():
    for name in ("karate_louvain_np50", "karate_lpm_np20"):
        _, rows = _measure(name)
        for r in rows:
            print(name, r)
            assert r["dev"] > 0


def test_blocked_vs_sequential_closure_at_c3():
    """BASELINE configs[2] scale (LFR n=100k mu=0.5): the engine's blocked sampler (orc.CLOSURE_ROUNDS_LOUVAIN blocks,
    orc_closure_sample = the device's, bit for bit) against the reference's SEQUENTIAL sampler
    over the growing graph (orc_closure_sequential: fast_consensus.py:175-184, its distribution
    with the oracle's RNG) on the same post-threshold graph of a 16-replica louvain consensus
    (restated CD).  Candidate count within 1.5 % and mean closure weight within 2 % (means over 3
    seeds each; printed)."""
    from fastconsensus_amd import synth
    n = 100_000
    u, v, _ = synth.lfr(n, 0.5, seed=42)
    g = orc.EdgeGraph.from_lines(n, np.stack([u, v], 1))
    n_p = 16
    lab, _ = orc.cd_batch(0, n_p, g, seed=3, nthreads=8)
    w = orc.consensus(0, g, lab, n_p)
    keep = orc.threshold(w, 0.2, n_p)
    kept = orc.EdgeGraph(n, g.u[keep], g.v[keep], w[keep], g.age[keep])
    blk, seq = [], []
    for s in range(3):
        pairs = orc.closure_sample_pairs(kept, g.m, s, 0)
        cu, _, cw, _ = orc.closure_from_pairs(0, kept, pairs, lab, n_p)
        blk.append((len(cu), float(cw.mean())))
        sp = orc.closure_sequential_pairs(kept, g.m, 100 + s)
        su, _, sw, _ = orc.closure_from_pairs(0, kept, sp, lab, n_p)
        seq.append((len(su), float(sw.mean())))
    b, q = np.mean(blk, 0), np.mean(seq, 0)
    print("C3 closure: kept %d, blocked %.0f candidates (mean weight %.3f), sequential %.0f (%.3f): %+.2f %%"
          % (kept.m, b[0], b[1], q[0], q[1], 100 * (b[0] - q[0]) / q[0]))
    assert abs(b[0] - q[0]) <= 0.015 * q[0]
    assert abs(b[1] - q[1]) <= 0.02 * q[1]
