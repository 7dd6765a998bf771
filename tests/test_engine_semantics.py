"""The device's semantics, end to end, against the reference loop's -- on the CPU.

tests/cpu_engine.py's OracleEngine is the bit-exact CPU model of the HIP engine (bucketed
CD twin, parallel closure sampler, repair, ages; tests/test_gpu_parity.py holds the device
to it bit for bit).  Driven through the same sharded loop as the device, its consensus NMI
distribution over 30 seeds is compared with the reference loop's own distribution (the
unmodified fast_consensus.py with the restated CD, tests/golden/make_refsem.py).  This
isolates the statistical effect of every deliberate deviation together (bucketed rounds,
pruning, predicted-dQ stopping, parallel closure) from device arithmetic.  Tolerances:
louvain mean NMI >= reference - 0.02 (about 2 standard errors of the difference at 30 + 30
runs); lpm recovery rate >= reference - 0.25, NMI of recovering runs >= reference - 0.03.
"""
import json

import numpy as np

from tests import golden_io


def _refsem(name):
    with open(golden_io.GOLDEN + "/refsem_%s.json" % name) as f:
        return json.load(f)


def _model_runs(algo, N, e, n_p, tau, delta, planted, seeds):
    from sklearn.metrics import normalized_mutual_info_score as nmi

    from fastconsensus_amd.distributed import run_sharded
    from tests.cpu_engine import OracleEngine
    out = []
    for seed in seeds:
        sigma = np.random.default_rng(seed + 1000).permutation(N).astype(np.int32)   # like FC_OPT_RELABEL
        eng = OracleEngine(seed=seed, sigma=sigma)
        eng.load_graph(N, e[:, 0], e[:, 1])
        lab, st = run_sharded(eng, algo, n_p, tau, delta, device="cpu", max_iters=200)
        assert not st["hit_iter_cap"]
        out.append(float(np.mean([nmi(planted, l) for l in lab])))
    return np.array(out)


def test_louvain_engine_model_vs_reference_loop():
    case = golden_io.load("lfr1k_louvain_np20")
    planted = np.load(golden_io.GOLDEN + "/lfr1k_mu04_planted.npy")[case.z["nodes"]]
    ref = _refsem("lfr1k_louvain_np20")
    got = _model_runs(0, case.N, case.edges_file, 20, 0.2, 0.02, planted, range(30))
    print("louvain engine model mean %.4f sd %.4f min %.4f | reference loop mean %.4f sd %.4f min %.4f"
          % (got.mean(), got.std(), got.min(), ref["nmi_mean"], ref["nmi_sd"], min(ref["nmi"])))
    assert got.mean() >= ref["nmi_mean"] - 0.02


def test_lpm_engine_model_vs_reference_loop():
    ref = _refsem("lfr1k_mu055_lpm_np20")
    e = np.loadtxt(golden_io.GOLDEN + "/lfr1k_mu055_synth.txt", dtype=np.int32).reshape(-1, 2)
    planted = np.load(golden_io.GOLDEN + "/lfr1k_mu055_synth_planted.npy")
    got = _model_runs(1, len(planted), e, 20, 0.8, 0.02, planted, range(30))
    r = np.array(ref["nmi"])
    print("lpm engine model recovery %d/30 (NMI %.4f) | reference loop recovery %d/30 (NMI %.4f)"
          % ((got > 0.5).sum(), got[got > 0.5].mean() if (got > 0.5).any() else 0, (r > 0.5).sum(),
             r[r > 0.5].mean()))
    assert (got > 0.5).mean() >= (r > 0.5).mean() - 0.25
    assert (got > 0.5).any() and got[got > 0.5].mean() >= r[r > 0.5].mean() - 0.03
