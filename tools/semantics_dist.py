#!/usr/bin/env python3
"""Consensus-NMI DISTRIBUTION of the engine's CD semantics variants on the CPU model (C2).

Runs tests/cpu_engine.py's OracleEngine (bit-exact CPU model of the device engine) through the
sharded loop on LFR-1k mu=0.4 (BASELINE configs[1]: louvain n_p=20, tau 0.2, delta 0.02) over
many seeds per variant and prints mean / sd / 10th percentile / min, with a two-sample KS test
against the reference loop's distribution (tests/golden/refsem_lfr1k_louvain_np20.json, the
unmodified fast_consensus.py with the restated CD; make_refsem.py c2 N).

    python tools/semantics_dist.py [nseeds] [variant ...]

Variants: classic (shared=0), hybrid (2, the default engine), hyb_s0 (3: sweep 0 per replica,
then as hybrid), g<k> (replicas grouped by k, one shared order per group).
"""
import json
import multiprocessing as mp
import os
import sys

os.environ.setdefault("OMP_NUM_THREADS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

VARIANTS = {"classic": 0, "hybrid": 2, "hyb_s0": 3}


def shared_of(name):
    if name in VARIANTS:
        return VARIANTS[name]
    if name.startswith("g"):
        return 0x100 | int(name[1:])
    raise SystemExit("unknown variant " + name)


def _one(args):
    shared, seed, buckets = args
    from sklearn.metrics import normalized_mutual_info_score as nmi
    from fastconsensus_amd.distributed import run_sharded
    from tests import golden_io
    from tests.cpu_engine import OracleEngine
    case = golden_io.load("lfr1k_louvain_np20")
    planted = np.load(golden_io.GOLDEN + "/lfr1k_mu04_planted.npy")[case.z["nodes"]]
    if os.environ.get("SEM_DEVSIGMA"):      # the device's own numbering: predicts a device run of this seed
        from oracle import oracle as orc
        sigma = orc.device_sigma(case.N, seed)
    else:
        sigma = np.random.default_rng(seed + 1000).permutation(case.N).astype(np.int32)
    eng = OracleEngine(seed=seed, sigma=sigma, shared=shared, buckets=buckets)
    eng.load_graph(case.N, case.edges_file[:, 0], case.edges_file[:, 1])
    lab, st = run_sharded(eng, 0, 20, 0.2, 0.02, device="cpu", max_iters=1000)
    return float(np.mean([nmi(planted, x) for x in lab]))


def stats(x):
    x = np.asarray(x)
    q = np.percentile(x, [5, 10, 25, 50, 75])
    return "mean %.4f sd %.4f min %.4f q5/10/25/50/75 %s" % (x.mean(), x.std(), x.min(), " ".join("%.3f" % v for v in q))


def main():
    from scipy.stats import ks_2samp
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    names = sys.argv[2:] or ["classic", "hybrid", "hyb_s0"]
    buckets = int(os.environ.get("SEM_BUCKETS", "0")) or None
    with open(os.path.join(ROOT, "tests/golden/refsem_lfr1k_louvain_np20.json")) as f:
        ref = np.array(json.load(f)["nmi"])
    print("reference loop (%d seeds): %s" % (len(ref), stats(ref)), flush=True)
    with mp.get_context("fork").Pool(int(os.environ.get("SEM_WORKERS", "8"))) as pool:
        for name in names:
            s0 = int(os.environ.get("SEM_SEED0", "0"))
            got = np.array(pool.map(_one, [(shared_of(name), s, buckets) for s in range(s0, s0 + n)]))
            if os.environ.get("SEM_SAVE"):
                with open(os.path.join(os.environ["SEM_SAVE"], "sem_%s.json" % name), "w") as f:
                    json.dump(got.tolist(), f)
            ks = ks_2samp(got, ref)
            ks1 = ks_2samp(got, ref, alternative="greater")   # H1: the device's CDF lies above (values smaller)
            print("%-8s (%d seeds): %s | sd ratio %.2f | KS D %.3f p %.4f | one-sided p %.4f" % (
                name, n, stats(got), got.std() / ref.std(), ks.statistic, ks.pvalue, ks1.pvalue), flush=True)


if __name__ == "__main__":
    main()
