"""Scaler folded into the solver (ops/scaler.scaler_fit_cast + newton_fit(affine=...)): CPU oracle
semantics -- identical statistics, pivot-shifted rows, and the same standardized-space model."""
import numpy as np
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import scaler as S


def _data(n=40_000, seed=3):
    return separable(n, seed=seed, device="cpu")  # col 0 Time-like (0..172800), col 29 Amount-like


def test_stats_and_rows_match_unfused():
    X, y = _data()
    out = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, out)
    ref = S.scaler_fit(X)
    for a, b in zip(st.numpy(), ref.numpy()):
        assert np.array_equal(a, b)
    expect = (X - X[0]).to(torch.bfloat16)
    assert torch.equal(out[:, :30], expect)
    assert torch.all(out[:, 30] == 1) and torch.equal(out[:, 31], y.to(torch.bfloat16))
    a = st.aff.numpy()
    assert np.allclose(a[:30], st.mean64[:30].numpy() - X[0].double().numpy(), rtol=0, atol=1e-6)
    assert np.allclose(a[32:62], 1.0 / st.scale64[:30].numpy()) and np.all(a[30:32] == 0) and np.all(a[62:] == 1)


def test_affine_fit_equals_standardized_fit():
    X, y = _data()
    shifted = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, shifted)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    f_ref = L.newton_fit(z, C=1.0, tol=1e-8)
    f_aff = L.newton_fit(shifted, C=1.0, tol=1e-8, affine=st.aff)
    assert f_aff.converged and f_ref.converged
    # only the bf16 rounding of the shifted rows separates the two fits
    assert np.allclose(f_aff.w, f_ref.w, rtol=0, atol=3e-3)
    assert abs(f_aff.objective - f_ref.objective) < 1e-3 * abs(f_ref.objective)


def test_shift_roundtrip():
    X, y = _data(5000)
    out = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, out)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    s = st.standard_to_shifted(z)
    assert torch.allclose(s[:, :30], (X - X[0]), rtol=1e-5, atol=5e-2)
    assert torch.equal(s[:, 30:], z[:, 30:])
    assert torch.allclose(st.shifted_to_standard(s), z, rtol=1e-4, atol=1e-4)


def test_affine_sgd_equals_standardized_sgd():
    """SGD on pivot-shifted rows with the affine map (the fused scaler path) follows the same
    standardized-space trajectory as SGD on standardized rows."""
    X, y = _data()
    shifted = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, shifted)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    kw = dict(C=1.0, epochs=3, batches=4)
    f_ref = L.sgd_fit(z, **kw)
    f_aff = L.sgd_fit(shifted, affine=st.aff, **kw)
    assert np.allclose(f_aff.w, f_ref.w, rtol=0, atol=3e-3)
