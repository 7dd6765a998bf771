"""Distribution gates for the consensus NMI (TEST INFRASTRUCTURE ONLY).

The reference loop's consensus NMI varies from run to run (LFR-1k: a top mode near 0.91 and
about one run in ten in a low mode near 0.80, tests/golden/refsem_lfr1k_louvain_np20.json), so a
device engine is held to the reference's DISTRIBUTION, not only to its mean:

* mean            >= reference mean - tol_mean
* spread          sd <= 1.3 x the reference's sd
* lower tail      10th percentile >= the reference's - 0.03
* stochastic order  one-sided two-sample KS test (H1: the device's values are smaller) at
                  alpha = 0.01 -- a device distribution that is only shifted UP (better NMI)
                  passes; the two-sided p-value is printed beside it.  Asserted at C2 (sd
                  ~0.03) and, since round 6, at C3 too (sd ~0.0005, 40 device vs 64 reference
                  runs), where it resolves offsets of ~0.0003 NMI: round 5's C3 lpm shift of
                  0.0008 (p ~ 0) came from the closure's block count (DESIGN, "Triadic
                  closure").  C3 also tightens the lower tail to p10 >= reference - 0.0005.

nmi() is sklearn's normalized_mutual_info_score (arithmetic mean of the entropies) computed
from a bincount contingency table: the same value (tests/test_dist_gates.py), ~20x faster on
100k-node labelings.
"""
import numpy as np

SD_RATIO_MAX = 1.3
P10_SLACK = 0.03
KS_ALPHA = 0.01


def nmi(a, b):
    a = np.unique(np.asarray(a), return_inverse=True)[1].ravel()
    b = np.unique(np.asarray(b), return_inverse=True)[1].ravel()
    ka, kb = int(a.max()) + 1 if a.size else 0, int(b.max()) + 1 if b.size else 0
    if ka == kb and ka <= 1:
        return 1.0
    n = a.size
    cont = np.bincount(a.astype(np.int64) * kb + b, minlength=ka * kb).reshape(ka, kb) if ka * kb < 50_000_000 else None
    if cont is not None:
        nz = cont[cont > 0].astype(np.float64)
        ia, ib = np.nonzero(cont)
    else:                                        # sparse contingency for many clusters
        key, nzc = np.unique(a.astype(np.int64) * kb + b, return_counts=True)
        nz = nzc.astype(np.float64)
        ia, ib = key // kb, key % kb
    pa = np.bincount(a, minlength=ka).astype(np.float64)
    pb = np.bincount(b, minlength=kb).astype(np.float64)
    mi = float(np.sum(nz / n * (np.log(nz) + np.log(n) - np.log(pa[ia]) - np.log(pb[ib]))))
    if mi <= 0:
        return 0.0
    ha = -float(np.sum(pa / n * np.log(pa / n)))
    hb = -float(np.sum(pb / n * np.log(pb / n)))
    return mi / max((ha + hb) / 2, np.finfo(np.float64).eps)


def describe(x):
    x = np.asarray(x, np.float64)
    return "mean %.4f sd %.4f p10 %.4f min %.4f (%d runs)" % (x.mean(), x.std(), np.percentile(x, 10), x.min(), x.size)


def check(got, ref, tol_mean, label="", ks=True, p10_slack=P10_SLACK):
    """Returns the printed summary; raises AssertionError naming the failed gate."""
    from scipy.stats import ks_2samp
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    ks1 = ks_2samp(got, ref, alternative="greater").pvalue
    ks2 = ks_2samp(got, ref).pvalue
    ratio = got.std() / ref.std() if ref.std() > 0 else (0.0 if got.std() == 0 else np.inf)
    msg = "%s device %s | reference %s | sd ratio %.2f | KS one-sided p %.4f (two-sided %.4f)" % (
        label, describe(got), describe(ref), ratio, ks1, ks2)
    print(msg)
    assert got.mean() >= ref.mean() - tol_mean, "mean gate: " + msg
    assert ratio <= SD_RATIO_MAX, "spread gate: " + msg
    assert np.percentile(got, 10) >= np.percentile(ref, 10) - p10_slack, "lower-tail gate: " + msg
    if ks:
        assert ks1 >= KS_ALPHA, "KS gate: " + msg
    return msg
