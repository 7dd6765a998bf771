#!/usr/bin/env python3
"""Which engine deviation moves the C3 sparse lpm consensus NMI?  (CPU only; test infrastructure.)

The device's consensus NMI on the sparse LFR-100k lpm case (synth.lfr(100000, 0.5, seed=42,
avg_deg=8, max_deg=25), n_p=64, tau 0.8, delta 0.02) sat ~0.0008 below the reference loop's
(orc.refsem_run: the reference's loop with sequential igraph LPA and the sequential closure).
tests/cpu_engine.py's OracleEngine is bit-exact with the device, so each of the engine's
deviations can be switched off on the CPU, one at a time, inside the same sharded loop:

    model     the default engine (shared=2, 32 buckets, pruning with tie revisits, 4 closure blocks)
    classic   per-replica visit orders in every sweep (shared=0)
    b<k>      k buckets per LPA sweep instead of 32
    noprune   every sweep visits every vertex
    seqclo    the reference's sequential closure sampler instead of the blocked one
    clo<k>    the blocked sampler in k blocks instead of 4
    seqcd     the sequential LPA restatement (orc_lpa, as refsem) instead of the bucketed twin
    refsem    orc.refsem_run itself (reference loop, sequential CD and closure)

    python tools/lpm_ablate.py NSEEDS variant [variant ...]      (env: ABL_WORKERS, ABL_SEED0)
"""
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

N = 100_000
GRAPH = {}


def graph():
    if not GRAPH:
        from fastconsensus_amd import synth
        u, v, planted = synth.lfr(N, 0.5, seed=42, avg_deg=8, max_deg=25)
        GRAPH.update(e=np.stack([u, v], 1), planted=planted)
    return GRAPH["e"], GRAPH["planted"]


def _init():
    os.environ["OMP_NUM_THREADS"] = "1"


def make_engine(variant, seed):
    from oracle import oracle as orc
    from tests.cpu_engine import OracleEngine
    kw = {}
    if variant == "classic":
        kw["shared"] = 0
    elif variant.startswith("b"):
        kw["buckets"] = int(variant[1:])
    elif variant == "noprune":
        kw["prune"] = 0
    eng = OracleEngine(seed=seed, sigma=orc.device_sigma(N, seed), **kw)
    if variant == "seqclo":
        def closure_sample(attempts, iteration, eng=eng):
            pairs = orc.closure_sequential_pairs(eng.kept, attempts, eng.seed * 7919 + iteration)
            dummy = np.zeros((1, eng.g.N), np.int32)
            cu, cv, _, cf = orc.closure_from_pairs(1, eng.kept, pairs, dummy, 1)
            order = np.lexsort((cv, cu))
            eng.cand = (cu[order], cv[order], cf[order])
            return len(cu)
        eng.closure_sample = closure_sample
    if variant.startswith("clo"):                 # clo<k>: the blocked sampler in k blocks
        k = int(variant[3:])

        def closure_sample(attempts, iteration, eng=eng, k=k):
            pairs = orc.closure_sample_pairs(eng.kept, attempts, eng.seed, iteration, rounds=k)
            dummy = np.zeros((1, eng.g.N), np.int32)
            cu, cv, _, cf = orc.closure_from_pairs(1, eng.kept, pairs, dummy, 1)
            order = np.lexsort((cv, cu))
            eng.cand = (cu[order], cv[order], cf[order])
            return len(cu)
        eng.closure_sample = closure_sample
    if variant == "seqcd":
        def cd(algo, r0, count, n_p, iteration, eng=eng):
            eng.lab, _ = orc.cd_batch(algo, count, eng.g, seed=eng.seed * 1000003 + iteration)
            eng.r0 = r0
        eng.cd = cd
    return eng


def one(args):
    variant, seed = args
    from fastconsensus_amd.distributed import run_sharded
    from oracle import oracle as orc
    from tests import dist_gates
    e, planted = graph()
    t = time.time()
    if variant == "refsem":
        g = orc.EdgeGraph.from_lines(N, e)
        lab, it = orc.refsem_run(1, g, 64, 0.8, 0.02, seed=seed)
    else:
        eng = make_engine(variant, seed)
        eng.load_graph(N, e[:, 0], e[:, 1])
        lab, st = run_sharded(eng, 1, 64, 0.8, 0.02, device="cpu", max_iters=1000)
        it = st["iterations"]
    return float(np.mean([dist_gates.nmi(planted, x) for x in lab])), int(it), time.time() - t


def main():
    from tests import dist_gates
    n = int(sys.argv[1])
    names = sys.argv[2:] or ["model"]
    s0 = int(os.environ.get("ABL_SEED0", "300"))
    with open(os.path.join(ROOT, "tests/golden/refsem_lfr100k_sparse_lpm_np64.json")) as f:
        ref = np.array(json.load(f)["nmi"])
    print("reference loop (%d seeds): %s" % (len(ref), dist_gates.describe(ref)), flush=True)
    graph()
    out = {}
    with mp.get_context("fork").Pool(int(os.environ.get("ABL_WORKERS", "8")), initializer=_init) as pool:
        for name in names:
            res = pool.map(one, [(name, s) for s in range(s0, s0 + n)], chunksize=1)
            got = np.array([r[0] for r in res])
            out[name] = got.tolist()
            print("%-8s %s | iters %s | %.0f s/run" % (name, dist_gates.describe(got),
                                                     sorted(set(r[1] for r in res)), np.mean([r[2] for r in res])),
                  flush=True)
    if os.environ.get("ABL_SAVE"):
        with open(os.environ["ABL_SAVE"], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
