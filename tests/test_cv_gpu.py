"""Device cross-validation (models/cv.py, K12): the reference's train_model.py job -- one scaler
on the training split, 5 stratified folds with SMOTE inside each, the final fit and 6 exact AUCs --
on one fold-sorted device table, with no per-fold copy.  A fold's fit that steps over its
validation block equals the fit on an explicit copy of the other blocks (bitwise: the passes see
the same logical rows), and each fold AUC equals the host AUC of that fold's model."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models.cv import DeviceCV
from fraud_detection_amd.models.pipeline import TrainConfig
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import reference as ref
from fraud_detection_amd.ops import split as SP

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("solver,storage", [("newton", "bf16"), ("sgd", "bf16"), ("sgd", "fp8")])
def test_device_cv_job(dev, solver, storage):
    X, y = separable(1_200_000, fraud_rate=0.004, seed=31, device=dev)
    Xt, yt = separable(200_000, fraud_rate=0.004, seed=32, device=dev)
    cv = DeviceCV(TrainConfig(solver=solver, storage=storage, seed=42))
    r = cv.run(X, y, Xt, yt)
    assert len(r.fold_aucs) == 5 and all(a > 0.9 for a in r.fold_aucs) and r.test_auc > 0.9
    # the permutation is a permutation, sorted by fold code, rows in their order inside a fold
    perm = cv.perm.cpu().numpy()
    assert np.array_equal(np.sort(perm), np.arange(X.shape[0]))
    codes = SP.assign_numpy(y.cpu().numpy(), 0.0, 5, 42)
    yp = y.cpu().numpy()[perm]
    cp = codes[perm].astype(int)
    assert np.all(np.diff(cp) >= 0)
    assert np.all(np.diff(perm)[np.diff(cp) == 0] > 0)
    b = cv.bounds
    assert b[-1] == X.shape[0] and np.all(np.diff(b) > 0)
    # fold 2's fit == the same solver on an explicit copy of the other blocks (same samples)
    k = 2
    f = cv.fits[k]
    part = torch.cat([cv.rows[: b[k]], cv.rows[b[k + 1]:]])
    v = cv.virtuals[k]
    w0 = np.zeros(32)
    w0[:30] = np.random.default_rng(42).normal(0.0, 0.01, 30)
    if solver == "newton":  # fold 2 warm-starts from fold 1's weights, without the warm-up phase
        g = L.newton_fit(part, tol=1e-4, max_iter=25, w0=w0, affine=cv.stats.aff, virtual=v,
                         fp8_scale=4.0, progressive=[], w0_from=cv._ws[1].state).as_fit_info()
        assert g.n_iter == f.n_iter
    else:
        g = L.sgd_fit(part, w0=w0, affine=cv.stats.aff, virtual=v,
                          extra_epochs=L.SGD_EXTRA_EPOCHS, avg_from=L.SGD_AVG_FROM,
                          epoch_batches=L.SGD_EPOCH_BATCHES).as_fit_info()
    assert np.array_equal(g.w, f.w)
    # the fold AUC is the exact AUC of the fold model on the fold's raw validation rows
    mean, _, scale = cv.stats.numpy()
    Xv = X.cpu().numpy()[perm[b[k]:b[k + 1]]].astype(np.float64)
    z = ((Xv - mean) / scale) @ f.w[:30] + f.w[30]
    assert abs(r.fold_aucs[k] - ref.roc_auc(z, yp[b[k]:b[k + 1]].astype(bool))) < 2e-6
    assert len(r.fold_ms) == 5 and r.final_ms > 0 and r.prep_ms > 0


def test_device_cv_warm_start_same_models(dev):
    """Warm-started folds (each Newton fit starts from the previous fit's weights) converge to the
    same tolerance as cold ones: fold 0 (cold in both) is bitwise the same fit; the warm folds'
    models differ from the cold ones only within the solver tolerance (weights ~1e-2 at tol 1e-4 on
    a weakly curved direction), so the fold AUCs agree to 1e-4 with fewer iterations."""
    X, y = separable(1_200_000, fraud_rate=0.004, seed=33, device=dev)
    cold = DeviceCV(TrainConfig(seed=42), warm_start=False)
    rc = cold.run(X, y)
    warm = DeviceCV(TrainConfig(seed=42), warm_start=True)
    rw = warm.run(X, y)
    assert np.array_equal(warm.fits[0].w, cold.fits[0].w)
    for fc, fw in zip(cold.fits, warm.fits):
        assert fc.converged and fw.converged and fw.grad_max <= 1e-4
    np.testing.assert_allclose(rw.fold_aucs, rc.fold_aucs, atol=1e-4)
    assert sum(rw.fold_iters[1:]) < sum(rc.fold_iters[1:])  # fewer iterations from a warm start


@pytest.mark.parametrize("solver", ["newton", "sgd"])
def test_device_cv_sklearn_folds(dev, solver):
    """With sklearn's StratifiedKFold(5, shuffle=True, random_state=42) codes (train.py split=sklearn,
    train_model.py:49,58) the job's fold blocks are exactly sklearn's validation folds, and every fold
    AUC agrees within 1e-3 with the per-fold path (scaler + SMOTE + fit on a copy of the fold's
    training rows, AUC of its validation rows) on the same folds."""
    from sklearn.model_selection import StratifiedKFold

    from fraud_detection_amd.models.cv import fold_codes_from_splits
    from fraud_detection_amd.models.pipeline import DevicePipeline, evaluate

    X, y = separable(1_200_000, fraud_rate=0.004, seed=35, device=dev)
    yh = y.cpu().numpy()
    sk = list(StratifiedKFold(n_splits=5, shuffle=True, random_state=42).split(np.zeros(len(yh)), yh))
    cfg = TrainConfig(solver=solver, seed=42)
    cv = DeviceCV(cfg)
    r = cv.run(X, y, fold_codes=fold_codes_from_splits(sk, len(yh)))
    perm, b = cv.perm.cpu().numpy(), cv.bounds
    for k, (tr, va) in enumerate(sk):
        assert np.array_equal(perm[b[k]:b[k + 1]], np.sort(va)), k  # exactly sklearn's fold k, in row order
        t = torch.from_numpy(tr).to(dev)
        v = torch.from_numpy(va).to(dev)
        res = DevicePipeline(cfg).fit(X.index_select(0, t), y.index_select(0, t))
        auc = evaluate(res, X.index_select(0, v), y.index_select(0, v))["auc"]
        assert abs(r.fold_aucs[k] - auc) < 1e-3, (k, r.fold_aucs[k], auc)
