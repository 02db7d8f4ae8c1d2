"""Property-based tests (hypothesis) of the HIP kernels against their oracles on MI355X: random
shapes (N not a multiple of a tile, N < 64), constant columns, large offsets, heavy score ties,
duplicate points.  Each example is one small kernel launch; the example count is bounded so the
module stays within a few seconds."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from fraud_detection_amd.ops import knn as K
from fraud_detection_amd.ops import metrics as M
from fraud_detection_amd.ops import predict as P
from fraud_detection_amd.ops import reference as ref
from fraud_detection_amd.ops import scaler as S

pytestmark = pytest.mark.gpu
SETTINGS = settings(max_examples=25, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


def _table(n, d, seed, offsets=True):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) * rng.uniform(0.01, 50, d)
    if offsets:  # large column offsets (creditcard Time ~ 1e5): the scaler's pivot-shifted sums
        X += rng.uniform(-1e5, 1e5, d) * (rng.random(d) < 0.3)
    const = rng.random(d) < 0.2
    X[:, const] = rng.normal(size=int(const.sum()))
    return X.astype(np.float32)


@SETTINGS
@given(st.integers(1, 5000), st.integers(1, 30), st.integers(0, 2**31 - 1))
def test_scaler_kernel_matches_oracle(dev, n, d, seed):
    X = _table(n, d, seed)
    g = S.scaler_fit(torch.from_numpy(X).to(dev))
    c = S.scaler_fit(torch.from_numpy(X))
    for a, b in zip(g.numpy(), c.numpy()):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9 * (1 + np.abs(b).max()))


@SETTINGS
@given(st.integers(2, 20000), st.integers(1, 16), st.floats(0.01, 0.99), st.integers(0, 2**31 - 1))
def test_auc_and_confusion_kernels_exact_with_ties(dev, n, levels, rate, seed):
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < rate).astype(np.uint8)
    y[0], y[-1] = 0, 1
    s = (rng.integers(0, levels, n) - levels / 2).astype(np.float32)
    st_, yt = torch.from_numpy(s), torch.from_numpy(y)
    assert M.auc_pair_counts(st_.to(dev), yt.to(dev)) == M.auc_pair_counts(st_, yt)
    assert np.array_equal(M.confusion_counts(st_.to(dev), yt.to(dev), 0.0), ref.confusion(s, y, 0.0))


@SETTINGS
@given(st.integers(6, 700), st.integers(1, 8), st.integers(0, 60), st.integers(0, 2**31 - 1))
def test_knn_kernel_exact_lists_with_duplicates(dev, m, k, dups, seed):
    rng = np.random.default_rng(seed)
    C = np.zeros((m, 32), np.float32)
    C[:, :30] = np.round(rng.normal(size=(m, 30)) * 2) / 2  # exact fp32 arithmetic on this grid
    nd = min(dups, m // 2)
    if nd:
        C[m - nd:] = C[:nd]
    k = min(k, m - 1)
    Ct = torch.from_numpy(C)
    got = K.knn_topk(Ct.to(dev), Ct.to(dev), k=k, self_offset=0).cpu()
    want = K.knn_topk(Ct, Ct, k=k, self_offset=0)
    assert torch.equal(got, want)  # same neighbours in the same (distance, index) order


@SETTINGS
@given(st.integers(1, 3000), st.integers(0, 2**31 - 1))
def test_predict_shap_kernel_matches_oracle(dev, n, seed):
    rng = np.random.default_rng(seed)
    X = _table(n, 30, seed, offsets=False)  # fp32 x - mean: same arithmetic, not a conditioning test
    mean, _, scale = S.scaler_fit(torch.from_numpy(X)).numpy()  # constant columns -> scale 1 (sklearn)
    w = np.zeros(32)
    w[:30] = rng.normal(0, 0.5, 30)
    w[30] = rng.normal()
    a, c, b = P.fold_scaler(w, mean, scale)
    at, ct = torch.from_numpy(a), torch.from_numpy(c)
    pg, phg = P.predict_shap_raw(torch.from_numpy(X).to(dev), at.to(dev), ct.to(dev), b)
    pc, phc = P.predict_shap_raw(torch.from_numpy(X), at, ct, b)
    np.testing.assert_allclose(pg.cpu().numpy(), pc.numpy(), atol=2e-5)
    np.testing.assert_allclose(phg.cpu().numpy(), phc.numpy(), rtol=1e-4, atol=1e-3)
