"""Minibatch SGD (BASELINE config 3) on CPU: the minibatch partition of the device pass
(logreg.hip row_phase walk) and the fp64 mirror of the device update (ops/reference.SgdStateRef):
every row and SMOTE sample lands in exactly one minibatch, every minibatch holds both classes, and
the solver reaches the Newton optimum with a converged state."""
import numpy as np
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import reference as ref
from fraud_detection_amd.ops import scaler as S


def test_row_partition_covers_each_row_once():
    for n, nb, full in ((10_000_000, 8, 768), (200_000, 8, 768), (5000, 3, 768), (64, 4, 768)):
        blocks = ref.sgd_grid_blocks(n, nb, full)
        b = ref.sgd_row_batches(n, nb, blocks)
        assert b.shape == (n,) and b.min() >= 0 and b.max() < nb
        if n >= 64 * 4 * nb * 4:  # large enough: every minibatch strides over the whole shard
            counts = np.bincount(b, minlength=nb)
            assert counts.min() > 0.7 * n / nb
            for k in range(nb):
                idx = np.nonzero(b == k)[0]
                assert idx.min() < n // 4 and idx.max() > 3 * n // 4


def test_pick_partition():
    b = ref.sgd_pick_batches(1000, 8)
    assert np.array_equal(np.bincount(b, minlength=8), np.bincount(np.arange(1000) // 16 % 8, minlength=8))
    assert set(b[:16]) == {0} and set(b[16:32]) == {1}


def _objective(R, w, C=1.0):
    g, loss, wsum, _ = ref.logreg_pass(R, w, (1.0, 1.0), False)
    return loss / wsum + 0.5 * float(w[:30] @ w[:30]) / (C * wsum)


def test_sgd_reaches_newton_optimum_cpu():
    X, y = separable(120_000, fraud_rate=0.3, seed=5)
    st = S.scaler_fit(X)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    newton = L.newton_fit(z, tol=1e-9, max_iter=40)
    sgd = L.sgd_fit(z, batches=4, epochs=4)
    R = z.double().numpy()
    f_n, f_s = _objective(R, newton.w), _objective(R, sgd.w)
    assert f_s >= f_n - 1e-12
    assert (f_s - f_n) / f_n < 1e-3, (f_s, f_n)
    assert sgd.n_iter == 16 and sgd.n_newton_steps == 0
    assert np.isfinite(sgd.grad_max) and np.isfinite(sgd.objective)
    assert sgd.converged == (sgd.grad_max <= L.SGD_TOL)


def test_sgd_virtual_cpu_matches_stored_samples():
    """CPU SGD over virtual SMOTE samples equals SGD over the same samples appended as rows when
    the samples are assigned the minibatches their pick tiles give them."""
    g = torch.Generator().manual_seed(3)
    real = torch.randn(6000, 32, generator=g)
    real[:, 30] = 1.0
    real[:, 31] = (torch.rand(6000, generator=g) < 0.05).float()
    par = torch.randn(80, 32, generator=g) + 0.8
    par[:, 30] = 1.0
    par[:, 31] = 1.0
    nbr = torch.stack([torch.randperm(80, generator=g)[:5] for _ in range(80)]).to(torch.int32)
    v = L.VirtualSmote(par.to(torch.bfloat16), nbr, 5000, seed=4)
    a = L.sgd_fit(real, batches=3, epochs=2, virtual=v)
    assert a.n_iter == 6 and np.all(np.isfinite(a.w))
    # every minibatch of the combined partition holds both classes
    rb = ref.sgd_row_batches(6000, 3, ref.sgd_grid_blocks(6000, 3, 768))
    pick, _ = ref.smote_pick_draws(80, 5, 5000, 4, 0, 0)
    pb = ref.sgd_pick_batches(400, 3)[pick.astype(np.int64)]
    for b in range(3):
        assert (real[rb == b, 31] == 0).any() and (pb == b).any()


def test_extra_epochs_run_only_until_converged_cpu():
    """extra_epochs: a converged fit never runs them (same model as without), an unconverged one
    runs them, each averaged like the last nominal epoch."""
    X, y = separable(60_000, fraud_rate=0.3, seed=9)
    st = S.scaler_fit(X)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    base = L.sgd_fit(z, batches=4, epochs=2, tol=1.0)  # loose tol: converged at the first full epoch end
    more = L.sgd_fit(z, batches=4, epochs=2, tol=1.0, extra_epochs=2)
    assert base.converged and more.converged and more.n_iter == base.n_iter <= 8
    assert np.array_equal(base.w, more.w)
    a = L.sgd_fit(z, batches=4, epochs=2, tol=0.0)  # never converges: every extra epoch runs
    b = L.sgd_fit(z, batches=4, epochs=2, tol=0.0, extra_epochs=1)
    assert a.n_iter == 8 and b.n_iter == 12 and not b.converged
    R = z.double().numpy()
    assert _objective(R, b.w) <= _objective(R, a.w) + 1e-12


def test_per_epoch_minibatch_counts_cpu():
    """epoch_batches: an epoch of 2 minibatches then one of 4 -- 6 steps; with 4 and 4 it is the
    uniform schedule exactly."""
    X, y = separable(40_000, fraud_rate=0.3, seed=12)
    st = S.scaler_fit(X)
    z = S.scale_cast(X, st, labels=y, out_dtype="f32")
    a = L.sgd_fit(z, batches=4, epochs=2, tol=0.0, subsample=None, epoch_batches=(2, 4))
    assert a.n_iter == 6 and np.all(np.isfinite(a.w))
    b = L.sgd_fit(z, batches=4, epochs=2, tol=0.0, subsample=None, epoch_batches=(4, 4))
    c = L.sgd_fit(z, batches=4, epochs=2, tol=0.0, subsample=None)
    assert np.array_equal(b.w, c.w) and b.n_iter == c.n_iter == 8
