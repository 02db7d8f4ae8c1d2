"""Property-based tests (hypothesis) of the numeric contracts every kernel is held to, on the CPU
paths (the numpy oracles the GPU kernels are compared against in tests/test_properties_gpu.py).
SURVEY.md §7.5: N not a multiple of a tile, N < 64, constant columns (scale -> 1), ties in AUC,
duplicate points in k-NN."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
from hypothesis.extra.numpy import arrays

from fraud_detection_amd.models.explainers import KernelExplainer, cached_design, kernelshap_reference
from fraud_detection_amd.ops import knn as K
from fraud_detection_amd.ops import metrics as M
from fraud_detection_amd.ops import reference as ref
from fraud_detection_amd.ops import scaler as S

SETTINGS = settings(max_examples=40, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


@st.composite
def tables(draw, max_n=300):
    n = draw(st.integers(1, max_n))
    d = draw(st.integers(1, 30))
    seed = draw(st.integers(0, 2**31 - 1))
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)) * rng.uniform(0.01, 50, d) + rng.uniform(-1e5, 1e5, d) * (rng.random(d) < 0.3)
    const = rng.random(d) < 0.2
    X[:, const] = rng.normal(size=int(const.sum()))  # constant columns: scale must become 1
    return X.astype(np.float32)


@SETTINGS
@given(tables())
def test_scaler_matches_sklearn(X):
    from sklearn.preprocessing import StandardScaler

    st_ = S.scaler_fit(torch.from_numpy(X))
    mean, var, scale = st_.numpy()
    sk = StandardScaler().fit(X.astype(np.float64))
    np.testing.assert_allclose(mean, sk.mean_, rtol=1e-9, atol=1e-9 * (1 + np.abs(sk.mean_).max()))
    np.testing.assert_allclose(var, sk.var_, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(scale, sk.scale_, rtol=1e-6)


@SETTINGS
@given(st.integers(2, 500), st.integers(1, 12), st.floats(0.02, 0.98), st.integers(0, 2**31 - 1))
def test_exact_auc_with_ties_equals_sklearn(n, levels, rate, seed):
    from sklearn.metrics import roc_auc_score

    rng = np.random.default_rng(seed)
    y = (rng.random(n) < rate).astype(np.uint8)
    y[0], y[-1] = 0, 1  # both classes present
    s = rng.integers(0, levels, n).astype(np.float32)  # few levels: many ties
    auc = M.roc_auc(torch.from_numpy(s), torch.from_numpy(y))
    assert abs(auc - roc_auc_score(y, s)) < 1e-12
    tn, fp, fn, tp = M.confusion_counts(torch.from_numpy(s), torch.from_numpy(y), float(levels) / 2)
    assert tn + fp + fn + tp == n and tp + fn == int(y.sum())


@SETTINGS
@given(st.integers(6, 150), st.integers(1, 8), st.integers(0, 40), st.integers(0, 2**31 - 1))
def test_knn_oracle_is_the_exact_brute_force(m, k, dups, seed):
    rng = np.random.default_rng(seed)
    C = np.zeros((m, 32), np.float32)
    C[:, :30] = np.round(rng.normal(size=(m, 30)) * 2) / 2  # coarse grid: exact distance ties
    nd = min(dups, m // 2)
    if nd:
        C[m - nd:] = C[:nd]  # duplicate rows
    k = min(k, m - 1)
    idx = K.knn_topk(torch.from_numpy(C), torch.from_numpy(C), k=k, self_offset=0).numpy()
    d2 = ((C[:, None, :30].astype(np.float64) - C[None, :, :30]) ** 2).sum(-1)
    np.fill_diagonal(d2, np.inf)
    for q in range(m):
        assert q not in idx[q]
        got = np.sort(d2[q, idx[q]])
        want = np.sort(d2[q])[:k]
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-4)
        # ties resolve to the smaller index: the list is ordered by (distance, index)
        key = [(round(d2[q, j], 4), j) for j in idx[q]]
        assert key == sorted(key)


@SETTINGS
@given(arrays(np.float32, st.integers(1, 200), elements=st.floats(-500, 500, width=32)))
def test_fp8_e4m3_round_trip(x):
    dec = ref.fp8_decode(ref.fp8_encode(x))
    ax = np.abs(x.astype(np.float64))
    sat = ax >= 448.0
    assert np.all(np.abs(dec[sat]) == 448.0)  # satfinite
    ok = ~sat & (ax >= 2.0 ** -6)  # normal range: 3 mantissa bits -> |rel err| <= 2^-4
    assert np.all(np.abs(dec[ok] - x[ok]) <= ax[ok] * 2.0 ** -4 + 1e-12)
    sub = ax < 2.0 ** -6  # subnormals: absolute step 2^-9
    assert np.all(np.abs(dec[sub] - x[sub]) <= 2.0 ** -10 + 1e-12)


@SETTINGS
@given(st.integers(2, 60), st.integers(1, 6), st.integers(0, 3000), st.integers(0, 2**31 - 1))
def test_smote_draws_stay_on_neighbour_segments(mq, k, n_new, seed):
    k = min(k, mq - 1)
    rng = np.random.default_rng(seed)
    nbr = np.stack([rng.choice(np.delete(np.arange(mq), q), k, replace=False) for q in range(mq)]).astype(np.int32)
    plan = ref.smote_plan(nbr, n_new, seed, 0)
    i, j, lam = ref.smote_draws_decode(plan)
    assert len(i) == n_new
    if n_new:
        assert i.min() >= 0 and i.max() < mq
        assert np.all([j[s] in nbr[i[s]] for s in range(min(n_new, 500))])
        assert lam.min() >= 0.0 and lam.max() < 1.0


@settings(max_examples=15, deadline=None, derandomize=True)
@given(st.integers(2, 12), st.integers(1, 6), st.integers(0, 2**31 - 1))
def test_kernelshap_efficiency_and_linear_limit(d, n_expl, seed):
    """phi sums to f(x) - f0 for any model (efficiency, identity link), and on the model's
    log-odds KernelSHAP equals LinearSHAP exactly (the interventional linear closed form)."""
    rng = np.random.default_rng(seed)
    a = rng.normal(0, 0.5, d)
    bias = float(rng.normal())
    B = rng.normal(size=(20, d))
    X = rng.normal(size=(n_expl, d))
    Z, _, A, zM = cached_design(d, None, 0)
    phi, fx, f0 = kernelshap_reference(X, a, bias, B, Z, A, zM, "identity")
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-9)
    phi_l, _, _ = kernelshap_reference(X, a, bias, B, Z, A, zM, "logit_model")
    np.testing.assert_allclose(phi_l, a[None, :] * (X - B.mean(0)[None, :]), atol=1e-8)
    ke = KernelExplainer(a, bias, B, device="cpu")
    np.testing.assert_allclose(ke.shap_values(X), phi, atol=1e-9)
