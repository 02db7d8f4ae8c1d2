"""Virtual SMOTE (ops/logreg.VirtualRows): the solver passes rebuild the synthetic rows from their
Philox draws instead of reading them from HBM.  The rebuilt rows must be bit-identical to the
ones ops/knn.smote_generate writes, so every pass -- and therefore every fit -- is bit-identical to
the materialized pipeline."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.ops import knn as K
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import scaler as S
from fraud_detection_amd.ops.native import native, stream_of


def _setup(dev, n, kind, affine, seed=5):
    X, y = separable(n, fraud_rate=0.02, seed=seed)
    X, y = X.to(dev), y.to(dev)
    if affine:
        rows = torch.empty((n, 32), dtype=torch.bfloat16, device=dev)
        st = S.scaler_fit_cast(X, y, rows)
    else:
        st = S.scaler_fit(X)
        rows = S.scale_cast(X, st, labels=y, out_dtype=kind)
    idx = torch.nonzero(y == 1).reshape(-1).to(torch.int64)
    xmin = S.scale_cast(X, st, labels=y, out_dtype="f32", idx=idx)
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0)
    n_new = n - 2 * int(idx.numel())
    v = L.VirtualRows(K.smote_parents(xmin, st.aff if affine else None), nbr, 0, n_new, seed=11, counter_base=2)
    return rows, v


def _reduced(rows, ws, h, begin, end, sub, vrows, n_split=None):
    m = native()
    L._pass(m, rows, ws, h, begin, end, L.DEFAULT_FP8_SCALE, stream_of(rows), done=False, sub=sub, vrows=vrows,
            n_split=n_split)
    torch.cuda.synchronize()
    return ws.red.clone().cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,affine", [("bf16", False), ("bf16", True), ("fp8", False)])
@pytest.mark.parametrize("h,sub", [(1, 1), (3, 1), (0, 1), (1, 4)])
def test_virtual_pass_bit_identical(dev, kind, affine, h, sub):
    rows, v = _setup(dev, 200_037, kind, affine)   # n_real not a multiple of the 64-row tile
    full = v.materialize(rows)
    assert full.shape[0] == rows.shape[0] + v.n_new
    ws = L.LRWorkspace(dev)
    w0 = np.r_[np.random.default_rng(1).normal(0, 0.2, 30), -1.0, 0.0]
    n_tot = full.shape[0]
    for begin, end in ((0, n_tot), (rows.shape[0] - 100, n_tot - 7), (rows.shape[0] + 5, n_tot)):
        ws.reset(w0)
        a = _reduced(full, ws, h, begin, end, sub, None, n_split=rows.shape[0])
        ws.reset(w0)
        b = _reduced(rows, ws, h, begin, end, sub, v)
        assert np.array_equal(a, b), (begin, end, np.abs(a - b).max())


@pytest.mark.gpu
@pytest.mark.parametrize("solver,storage", [("newton", "bf16"), ("newton", "fp8"), ("sgd", "bf16")])
def test_pipeline_virtual_equals_materialized(dev, solver, storage):
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig

    X, y = separable(2_500_000, seed=77, device=dev)
    fits = {}
    for mode in ("virtual", "materialize"):
        cfg = TrainConfig(solver=solver, storage=storage, smote_mode=mode, sgd_epochs=2, sgd_batch_rows=1 << 20)
        r = DevicePipeline(cfg).fit(X, y)
        fits[mode] = (r.w.copy(), r.n_train_rows, r.fit.n_iter)
    (wv, nv, iv), (wm, nm, im) = fits["virtual"], fits["materialize"]
    assert nv == nm and iv == im
    assert np.array_equal(wv, wm), np.abs(wv - wm).max()


@pytest.mark.gpu
def test_smote_plan_matches_oracle(dev):
    rng = np.random.default_rng(2)
    nbr = torch.from_numpy(rng.integers(0, 5000, size=(4000, 5)).astype(np.int32))
    got = K.smote_plan(nbr.to(dev), 300_001, seed=123456789012, counter_base=7).cpu()
    exp = K.smote_plan(nbr, 300_001, seed=123456789012, counter_base=7)
    assert torch.equal(got, exp)


@pytest.mark.gpu
def test_zipped_stored_pass_matches_oracle(dev):
    """The zipped tile order only regroups the sums: same gradient/Hessian as the plain pass."""
    rows, v = _setup(dev, 100_000, "bf16", False)
    full = v.materialize(rows)
    w = torch.from_numpy(np.r_[np.random.default_rng(3).normal(0, 0.2, 30), -1.0, 0.0])
    g0, l0, s0, H0 = L.logreg_pass(full, w)
    ws = L.LRWorkspace(dev)
    ws.reset(w.numpy())
    red = _reduced(full, ws, 1, 0, full.shape[0], 1, None, n_split=rows.shape[0])
    np.testing.assert_allclose(red[:32], g0, rtol=1e-5, atol=1e-3)
    assert abs(red[32] - l0) / l0 < 1e-6 and red[33] == s0
    np.testing.assert_allclose(red[64:].reshape(32, 32), H0, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
def test_smote_parents_match_cpu(dev):
    X, y = separable(50_000, fraud_rate=0.05, seed=8)
    rows = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, rows)
    idx = torch.nonzero(y == 1).reshape(-1)
    xmin = S.scale_cast(X[idx].contiguous(), st, labels=y[idx].contiguous(), out_dtype="f32")
    for aff in (None, st.aff):
        cpu = K.smote_parents(xmin, aff)
        gpu = K.smote_parents(xmin.to(dev), aff.to(dev) if aff is not None else None).cpu()
        assert torch.equal(cpu, gpu)


def test_virtual_rows_materialize_cpu():
    """CPU path: a fit given VirtualRows materializes them and equals the explicit concatenation."""
    X, y = separable(20_000, fraud_rate=0.05, seed=3)
    st = S.scaler_fit(X)
    rows = S.scale_cast(X, st, labels=y, out_dtype="bf16")
    idx = torch.nonzero(y == 1).reshape(-1)
    xmin = S.scale_cast(X[idx].contiguous(), st, labels=y[idx].contiguous(), out_dtype="f32")
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0)
    v = L.VirtualRows(K.smote_parents(xmin), nbr, 0, 5_000, seed=9)
    full = v.materialize(rows)
    a = L.newton_fit(rows, tol=1e-6, vrows=v)
    b = L.newton_fit(full, tol=1e-6)
    assert np.array_equal(a.w, b.w)
