"""K10 metrics on CPU: exact AUC == sklearn, histogram AUC close to it and mergeable by summation
(the data-parallel collective C6), ROC points, confusion counts."""
import numpy as np
import pytest
import torch
from sklearn.metrics import confusion_matrix, roc_auc_score

from fraud_detection_amd.ops import metrics as M


def _scores(n=50_000, rate=0.02, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = (torch.rand(n, generator=g) < rate).to(torch.uint8)
    s = torch.randn(n, generator=g) + 2.0 * y.float()
    s[:500] = torch.round(s[:500])  # ties
    return s.contiguous(), y


def test_exact_auc_equals_sklearn():
    s, y = _scores()
    assert M.roc_auc(s, y) == pytest.approx(roc_auc_score(y.numpy(), s.numpy()), abs=1e-12)


def test_hist_auc_close_and_exact_when_bins_resolve_ties():
    s, y = _scores()
    assert abs(M.roc_auc_hist(s, y, bits=20) - M.roc_auc(s, y)) < 2e-4
    # scores on a coarse grid: every distinct value has its own bin -> hist AUC is exact
    q = torch.round(s * 8) / 8
    assert M.roc_auc_hist(q, y, bits=20) == pytest.approx(M.roc_auc(q, y), abs=1e-12)


def test_hist_merges_across_shards():
    s, y = _scores(40_001)
    full = M.score_histogram(s, y)
    parts = sum(M.score_histogram(s[i::3].contiguous(), y[i::3].contiguous()) for i in range(3))
    assert torch.equal(full, parts)


def test_order_key_is_monotone():
    v = np.array([-np.inf, -3.5, -1e-30, -0.0, 0.0, 1e-30, 2.0, np.inf], np.float32)
    k = M._order_key_np(v)
    assert np.all(np.diff(k.astype(np.int64)) >= 0)


def test_roc_curve_hist_endpoints():
    s, y = _scores()
    fpr, tpr = M.roc_curve_hist(s, y)
    assert fpr[0] == 0 and tpr[0] == 0 and fpr[-1] == pytest.approx(1) and tpr[-1] == pytest.approx(1)
    assert np.all(np.diff(fpr) >= 0) and np.all(np.diff(tpr) >= 0)
    assert np.trapz(tpr, fpr) == pytest.approx(M.roc_auc(s, y), abs=5e-3)


def test_confusion_counts_match_sklearn():
    s, y = _scores()
    tn, fp, fn, tp = M.confusion_counts(s, y, 0.5)
    ref = confusion_matrix(y.numpy(), (s.numpy() > 0.5).astype(int)).ravel()
    assert [tn, fp, fn, tp] == list(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,rate,ties", [(20_000_000, 0.5, False), (3_000_001, 0.3, True), (9_000_000, 0.01, True)])
def test_exact_auc_sort_path_large_p(dev, n, rate, ties):
    """a 20M-row 50%-positive AUC through the native radix-sort path is exact
    (== sklearn) with no host synchronisation inside; the auto-selection takes that path above
    SORT_PATH_POSITIVES positives or RADIX_ROWS scores."""
    import time

    from sklearn.metrics import roc_auc_score

    from fraud_detection_amd.ops import metrics as M

    g = torch.Generator().manual_seed(n)
    y = (torch.rand(n, generator=g) < rate).to(torch.uint8)
    s = torch.randn(n, generator=g) + 0.8 * y.float()
    if ties:
        s = torch.round(s * 64) / 64          # heavy ties
    sd, yd = s.to(dev), y.to(dev)
    M.roc_auc(sd, yd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = M.roc_auc(sd, yd)
    dt = time.perf_counter() - t0
    exp = roc_auc_score(y.numpy(), s.numpy())
    assert got == pytest.approx(exp, abs=1e-12)
    auc_d, res = M.auc_radix(sd, yd)
    twice, P, N = (int(v) for v in res.cpu())
    assert P == int(y.sum()) and N == n - P
    assert twice == round(exp * 2 * P * (n - P))
    assert float(auc_d) == got
    assert dt < 0.05, f"{dt:.3f}s"          # 5 radix passes + one counting pass
    print(f"[auc] n={n} rate={rate} ties={ties}: {dt * 1e3:.2f} ms")


@pytest.mark.gpu
def test_radix_auc_small_and_degenerate(dev):
    """The radix path on small inputs (one block, partial sub-chunks), all-tied scores, -0 / +0,
    and single-class inputs (NaN AUC, no fault)."""
    from sklearn.metrics import roc_auc_score

    from fraud_detection_amd.ops import metrics as M

    rng = np.random.default_rng(5)
    for n in (1, 2, 7, 255, 256, 257, 1000, 70_001):
        y = (rng.random(n) < 0.4).astype(np.uint8)
        s = np.round(rng.normal(size=n) * 4) / 4
        s[: n // 3] = -0.0 if n > 3 else s[: n // 3]
        sd, yd = torch.from_numpy(s.astype(np.float32)).to(dev), torch.from_numpy(y).to(dev)
        auc, res = M.auc_radix(sd, yd)
        if 0 < y.sum() < n:
            assert float(auc) == pytest.approx(roc_auc_score(y, s.astype(np.float32)), abs=1e-12), n
        else:
            assert np.isnan(float(auc))
    y = torch.zeros(1000, dtype=torch.uint8, device=dev)
    y[::3] = 1
    auc, _ = M.auc_radix(torch.zeros(1000, device=dev), y)
    assert float(auc) == 0.5  # every pair tied


@pytest.mark.gpu
@pytest.mark.parametrize("n,rate", [(2_000_003, 0.0017), (300_000, 0.05), (50_000, 0.5), (1000, 0.0)])
def test_auc_known_positives_exact(dev, n, rate):
    """The sync-free sorted-positives AUC (CV folds know their positive count) == sklearn, and the
    radix path's pair count; above SORT_PATH_POSITIVES it delegates to the radix path."""
    from sklearn.metrics import roc_auc_score

    from fraud_detection_amd.ops import metrics as M

    g = torch.Generator().manual_seed(n)
    y = (torch.rand(n, generator=g) < rate).to(torch.uint8)
    s = torch.round((torch.randn(n, generator=g) + 1.1 * y.float()) * 32) / 32  # ties
    sd, yd = s.to(dev), y.to(dev)
    auc, twice = M.auc_known_positives(sd, yd, int(y.sum()))
    if 0 < int(y.sum()) < n:
        assert float(auc) == pytest.approx(roc_auc_score(y.numpy(), s.numpy()), abs=1e-12)
        assert int(twice) == int(M.auc_radix(sd, yd)[1][0])
    else:
        assert np.isnan(float(auc))
