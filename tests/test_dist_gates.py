"""tests/dist_gates.py: the fast NMI equals sklearn's, and the gates accept the reference's own
distribution while rejecting a heavier lower tail or a wider spread."""
import numpy as np
import pytest

from tests import dist_gates


@pytest.mark.parametrize("n,ka,kb", [(50, 3, 4), (1000, 40, 25), (20000, 700, 900), (10, 1, 1), (10, 1, 3)])
def test_nmi_matches_sklearn(n, ka, kb):
    from sklearn.metrics import normalized_mutual_info_score
    rng = np.random.default_rng(n + ka)
    a = rng.integers(0, ka, n) * 7 + 3
    b = np.where(rng.random(n) < 0.7, a // 7, rng.integers(0, kb, n))
    assert abs(dist_gates.nmi(a, b) - normalized_mutual_info_score(a, b)) < 1e-12


def test_gates_accept_reference_and_reject_worse():
    import json
    from tests import golden_io
    with open(golden_io.GOLDEN + "/refsem_lfr1k_louvain_np20.json") as f:
        ref = np.array(json.load(f)["nmi"])
    assert len(ref) >= 64
    rng = np.random.default_rng(0)
    half = rng.permutation(ref)
    dist_gates.check(half[:80], half[80:], 0.015, "reference vs itself")
    with pytest.raises(AssertionError, match="lower-tail|KS|spread"):
        dist_gates.check(np.where(ref < 0.89, ref - 0.06, ref), ref, 0.015)   # heavier low mode
    with pytest.raises(AssertionError, match="spread|KS"):
        dist_gates.check(ref.mean() + 1.6 * (ref - ref.mean()), ref, 0.015)
