"""Virtual SMOTE samples (ops/logreg.VirtualSmote, logreg.hip pick_terms): a logistic pass over
stored rows plus SMOTE samples folded in through per-pick sums must match the fp64 oracle pass
over the stored rows followed by the samples' fp32 interpolants (ops/reference.py); the
lambda buckets must hold exactly the oracle's draws; fits must be bitwise reproducible and agree
with the stored-SMOTE fit (which rounds each interpolant to bf16 / e4m3)."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import reference as ref


def _case(n_real, m, mq, k, seed, device):
    """bf16 real rows (labels 0/1 in col 31, 1 in col 30), bf16 parents [m, 32] and distinct
    neighbour slots per query row."""
    g = torch.Generator().manual_seed(seed)
    real = torch.randn(n_real, 32, generator=g) * 1.5
    real[:, 30] = 1.0
    real[:, 31] = (torch.rand(n_real, generator=g) < 0.3).float()
    par = torch.randn(m, 32, generator=g) + 0.7
    par[:, 30] = 1.0
    par[:, 31] = 1.0
    nbr = torch.stack([torch.randperm(m, generator=g)[:k] for _ in range(mq)]).to(torch.int32)
    return real.to(torch.bfloat16).to(device), par.to(torch.bfloat16).to(device), nbr.to(device)


def _fp8_rows(real_bf16, scale):
    r = real_bf16.float().cpu().numpy().copy()
    r[:, :30] *= scale
    return torch.from_numpy(ref.fp8_encode(r)).to(real_bf16.device)


def test_virtual_newton_cpu_fallback():
    real, par, nbr = _case(3000, 40, 30, 5, 1, "cpu")
    v = L.VirtualSmote(par, nbr, 2500, q_offset=7, sample_offset=256, seed=9, counter_base=2)
    a = L.newton_fit(real, tol=1e-6, virtual=v)
    b = L.newton_fit(torch.cat([real.float(), v.rows_f32()]), tol=1e-6)
    np.testing.assert_array_equal(np.asarray(a.w), np.asarray(b.w))


def test_pick_draws_match_plan():
    nbr = np.arange(30 * 5).reshape(30, 5) % 40
    pick, lam = ref.smote_pick_draws(30, 5, 1000, 42, 3, 128)
    plan = ref.smote_plan(nbr, 1000, 42, 3, 128)
    i, j, lf = ref.smote_draws_decode(plan)
    np.testing.assert_array_equal(i, pick // 5)
    np.testing.assert_array_equal(j, nbr[pick // 5, pick % 5])
    np.testing.assert_array_equal(lf, lam.astype(np.float32) / 65536)


@pytest.mark.gpu
def test_buckets_hold_the_draws(dev):
    _, par, nbr = _case(10, 500, 300, 5, 2, dev)
    v = L.VirtualSmote(par, nbr, 123_457, q_offset=11, sample_offset=384, seed=5, counter_base=7).prepare()
    pick, lam = ref.smote_pick_draws(300, 5, 123_457, 5, 7, 384)
    off, cnt = v.off.cpu().numpy(), v.cnt.cpu().numpy()
    np.testing.assert_array_equal(cnt, np.bincount(pick, minlength=1500))
    got = v.lam.cpu().numpy().view(np.uint16)
    runs = sorted((int(o), int(c)) for o, c in zip(off, cnt) if c)
    pos = 0
    for o, c in runs:  # the runs tile lam exactly
        assert o == pos
        pos += c
    assert pos == 123_457
    for p in range(0, 1500, 37):  # each run holds its pick's lambdas (any order)
        np.testing.assert_array_equal(np.sort(got[off[p]:off[p] + cnt[p]]), np.sort(lam[pick == p].astype(np.uint16)))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bf16", "fp8"])
@pytest.mark.parametrize("n_real,n_new,q_off,s_off", [(100_003, 77_777, 0, 0), (5, 300_001, 3, 128)])
def test_virtual_pass_matches_oracle(dev, kind, n_real, n_new, q_off, s_off):
    real, par, nbr = _case(n_real, 200, 150, 5, n_real, dev)
    v = L.VirtualSmote(par, nbr, n_new, q_offset=q_off, sample_offset=s_off, seed=42, counter_base=5)
    rows = real if kind == "bf16" else _fp8_rows(real, 4.0)
    R = np.concatenate([ref.rows_to_f32(rows.cpu(), 4.0).numpy(), v.rows_f32().numpy()])
    w = np.r_[np.random.default_rng(3).normal(0, 0.3, 30), -0.5, 0.0]
    g_r, loss_r, ws_r, H_r = ref.logreg_pass(R, w, (1.0, 3.0), True)
    for hess in (True, False):
        g, loss, ws, H = L.logreg_pass(rows, torch.from_numpy(w), (1.0, 3.0), hessian=hess, fp8_scale=4.0, virtual=v)
        np.testing.assert_allclose(g, g_r, rtol=1e-4, atol=1e-2)
        assert abs(loss - loss_r) / loss_r < 1e-5
        assert ws == pytest.approx(ws_r)
        if hess:
            rel = np.linalg.norm(H - H_r) / np.linalg.norm(H_r)
            assert rel < 5e-3, rel
            np.testing.assert_allclose(H, H.T, atol=1e-6 * np.abs(H).max())


@pytest.mark.gpu
def test_virtual_newton_fit_reproducible_and_close(dev):
    """Progressive warm-up (pick-tile subsets), sub-sampled Hessian: the virtual fit is bitwise
    reproducible and lands on the fit over the stored bf16 rows (which round each interpolant)."""
    real, par, nbr = _case(8_500_001, 3000, 3000, 5, 8, dev)
    v = L.VirtualSmote(par, nbr, 8_400_000, seed=42)
    a = L.newton_fit(real, tol=1e-5, virtual=v)
    a2 = L.newton_fit(real, tol=1e-5, virtual=L.VirtualSmote(par, nbr, 8_400_000, seed=42))
    np.testing.assert_array_equal(np.asarray(a.w), np.asarray(a2.w))
    full = torch.empty((real.shape[0] + v.n_new, 32), dtype=real.dtype, device=dev)
    full[: real.shape[0]] = real
    v.materialize(full[real.shape[0]:])
    b = L.newton_fit(full, tol=1e-5)
    assert a.converged and b.converged
    np.testing.assert_allclose(np.asarray(a.w), np.asarray(b.w), rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("storage", ["bf16"])  # fp8 fits keep stored SMOTE rows (pipeline.py virt_ok)
def test_pipeline_virtual_vs_stored_smote(dev, storage):
    X, y = separable(600_000, fraud_rate=0.01, seed=12)
    Xt, yt = separable(200_000, fraud_rate=0.01, seed=13)
    Xd, yd = X.to(dev), y.to(dev)
    rv = DevicePipeline(TrainConfig(virtual_smote=True, storage=storage)).fit(Xd, yd)
    rv2 = DevicePipeline(TrainConfig(virtual_smote=True, storage=storage)).fit(Xd, yd)
    rs = DevicePipeline(TrainConfig(virtual_smote=False, storage=storage)).fit(Xd, yd)
    assert rv.n_train_rows == rs.n_train_rows and rv.n_synthetic > 0
    np.testing.assert_array_equal(np.asarray(rv.w), np.asarray(rv2.w))
    np.testing.assert_allclose(np.asarray(rv.w), np.asarray(rs.w), rtol=2e-2, atol=5e-3)
    av = evaluate(rv, Xt.to(dev), yt.to(dev))["auc"]
    as_ = evaluate(rs, Xt.to(dev), yt.to(dev))["auc"]
    assert abs(av - as_) < 1e-3, (av, as_)


@pytest.mark.gpu
@pytest.mark.parametrize("solver", ["sgd", "newton"])
def test_bucket_sort_placement_does_not_change_the_fit(dev, solver, monkeypatch):
    """FDX_SMOTE_OVERLAP: the virtual-SMOTE bucket sort in line, on a side stream beside the k-NN
    (default) or beside the scaler pass (staged) -- the same draw, so bitwise the same model, fit
    after fit with nothing synchronising the host in between (a cross-stream race on the bucket
    buffers would show as a changed model).  The CV job's up-front side-stream sorts likewise."""
    from fraud_detection_amd.models.cv import DeviceCV

    X, y = separable(1_500_000, seed=31, device=dev)
    got = {}
    for mode in ("0", "knn", "scaler"):
        monkeypatch.setenv("FDX_SMOTE_OVERLAP", mode)
        pipe = DevicePipeline(TrainConfig(seed=42, solver=solver))
        runs = [pipe.fit(X, y) for _ in range(3)]
        torch.cuda.synchronize()
        got[mode] = [np.asarray(r.w).copy() for r in runs]
    for mode in ("knn", "scaler"):
        for a, b in zip(got["0"], got[mode]):
            assert np.array_equal(a, b), mode
    cv = {}
    for mode in ("0", "scaler"):
        monkeypatch.setenv("FDX_SMOTE_OVERLAP", mode)
        r = DeviceCV(TrainConfig(seed=42, solver=solver)).run(X, y)
        cv[mode] = (list(r.fold_aucs), np.asarray(r.final.w).copy())
    assert cv["0"][0] == cv["scaler"][0] and np.array_equal(cv["0"][1], cv["scaler"][1])
