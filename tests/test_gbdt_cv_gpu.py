"""The GBDT family's device CV job (models/gbdt_cv.DeviceGBDTCV, train_model.py:49-110): the
folds fit the binned fold-sorted table around their own block (gbdt.hip row hole), and a fold's
trees are bit-identical to the same fit on an explicit copy of its rows."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models.gbdt_cv import DeviceGBDTCV
from fraud_detection_amd.models.pipeline import TrainConfig
from fraud_detection_amd.ops import gbdt as gb
from fraud_detection_amd.ops import metrics as M

pytestmark = pytest.mark.gpu


def _job(dev, n=400_000, trees=12):
    X, y = separable(n, seed=61, device=dev)
    Xt, yt = separable(100_000, seed=62, device=dev)
    cv = DeviceGBDTCV(TrainConfig(), gb.GBDTParams(n_estimators=trees, max_depth=5))
    return cv, cv.run(X, y, Xt, yt), (X, y)


def test_gbdt_cv_job(dev):
    cv, r, _ = _job(dev)
    assert len(r.fold_aucs) == 5 and min(r.fold_aucs) > 0.9, r.fold_aucs
    assert r.test_auc is not None and r.test_auc > 0.9
    assert r.final.n_synthetic > 0 and r.final.scale_pos_weight == pytest.approx(1.0)
    # each fold's margins over its block are its validation scores: the radix AUC agrees
    ens, margin, *_ = cv._one_fit(2)
    b0, b1 = int(cv.bounds[2]), int(cv.bounds[3])
    assert M.roc_auc(margin[b0:b1].contiguous(), cv.labels[b0:b1]) == pytest.approx(r.fold_aucs[2], abs=1e-12)


def test_fold_trees_bit_identical_to_an_explicit_copy(dev):
    cv, r, _ = _job(dev, n=300_000, trees=8)
    k = 1
    ens_h, margin_h, n_fit, n_min, n_new, spw = cv._one_fit(k)
    n = int(cv.bounds[-1])
    b0, b1 = int(cv.bounds[k]), int(cv.bounds[k + 1])
    keep = torch.cat([torch.arange(0, b0, device=dev), torch.arange(b1, n + n_new, device=dev)])
    bins_c = cv.bins[: n + n_new].index_select(0, keep).contiguous()
    lab_c = cv.labels[: n + n_new].index_select(0, keep).contiguous()
    params = gb.GBDTParams(n_estimators=8, max_depth=5, scale_pos_weight=spw)
    ens_c, margin_c = gb.fit_binned(bins_c, lab_c, cv.cuts, params, return_margin=True)
    for a in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(ens_h, a), getattr(ens_c, a)), a
    assert torch.equal(margin_h.index_select(0, keep), margin_c)
    # the hole's margins = the copy's ensemble walked over the block's bins
    ref = gb.R.predict_margin_bins(cv.bins[b0:b1].cpu().numpy(), ens_c.feat, ens_c.bin, ens_c.leaf, 5,
                                   ens_c.base_margin)
    np.testing.assert_array_equal(margin_h[b0:b1].cpu().numpy(), ref)


def test_train_entry_point_runs_the_device_gbdt_cv_job(tmp_path, monkeypatch):
    """train.run(model_type="gbdt") on a GPU takes the device CV job (no per-fold copies) and
    ships its final fit with the reference's artifact layout."""
    import os

    from fraud_detection_amd import train
    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.data.synthetic import reference_frame

    df = reference_frame(20000, seed=5)
    csv = tmp_path / "cc.csv"
    df.to_csv(csv, index=False)
    monkeypatch.setenv("DATA_CSV", str(csv))
    monkeypatch.setenv("FDX_DEVICE", "cuda")
    monkeypatch.setenv("MLFLOW_TRACKING_URI", str(tmp_path / "mlruns"))
    monkeypatch.setenv("MLFLOW_AUC_THRESHOLD", "0.0")
    orig = gb.GBDTParams
    monkeypatch.setattr(gb, "GBDTParams", lambda **kw: orig(**{"n_estimators": 5, "max_depth": 3, **kw}))
    out = train.run(Settings.load(), model_type="gbdt", cv_folds=3, model_dir=str(tmp_path / "models"), verbose=False)
    assert out["cv_engine"] == "device", out["cv_engine"]
    assert len(out["cv_scores"]) == 3 and all(0.0 <= a <= 1.0 for a in out["cv_scores"])
    assert os.path.exists(tmp_path / "models" / "xgb_model.json")


def test_gbdt_cv_sklearn_folds(dev):
    """sklearn StratifiedKFold(5, shuffle, 42) codes: the GBDT job's fold blocks are sklearn's
    validation folds; fold AUCs agree with the per-fold GBDT pipeline on the same folds (its own
    scaler, cuts and SMOTE draws on the fold copy, so a looser bound than the logistic job's)."""
    from sklearn.model_selection import StratifiedKFold

    from fraud_detection_amd.models.cv import fold_codes_from_splits
    from fraud_detection_amd.models.gbdt import GBDTPipeline

    X, y = separable(400_000, fraud_rate=0.004, seed=63, device=dev)
    yh = y.cpu().numpy()
    sk = list(StratifiedKFold(n_splits=5, shuffle=True, random_state=42).split(np.zeros(len(yh)), yh))
    params = gb.GBDTParams(n_estimators=20, max_depth=5)
    cv = DeviceGBDTCV(TrainConfig(), params)
    r = cv.run(X, y, fold_codes=fold_codes_from_splits(sk, len(yh)))
    perm, b = cv.perm.cpu().numpy(), cv.bounds
    for k, (tr, va) in enumerate(sk):
        assert np.array_equal(perm[b[k]:b[k + 1]], np.sort(va)), k
    for k in (0, 3):
        t, v = torch.from_numpy(sk[k][0]).to(dev), torch.from_numpy(sk[k][1]).to(dev)
        res = GBDTPipeline(TrainConfig(), params).fit(X.index_select(0, t), y.index_select(0, t))
        auc = res.evaluate(X.index_select(0, v), y.index_select(0, v))["auc"]
        assert abs(r.fold_aucs[k] - auc) < 5e-3, (k, r.fold_aucs[k], auc)
