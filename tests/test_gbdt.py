"""GBDT family on CPU (the numpy oracle of csrc/kernels/gbdt.hip), SURVEY.md §2.3 K11.

The oracle's split search is checked against an independent brute-force search over raw
(unbinned) thresholds; the estimator, JSON round trip, pipeline and DP (gloo) paths run on it.
xgboost is not installed in this image: parity with xgboost itself is unpinned, so quality is
pinned against sklearn's HistGradientBoostingClassifier on the same data instead."""
import json
import os

import numpy as np
import pytest
import torch

from fraud_detection_amd.ops import gbdt as gb
from fraud_detection_amd.ops import reference_gbdt as R


def _data(n=4000, d=6, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, max(d, 4))).astype(np.float32)
    logit = 1.5 * X[:, 0] - 2.0 * (X[:, 1] > 0.3) + X[:, 2] * X[:, 3] - 2.5
    X = np.ascontiguousarray(X[:, :d])
    y = (rng.random(n) < 1.0 / (1.0 + np.exp(-logit))).astype(np.uint8)
    return X, y


def test_cuts_and_bins_are_consistent():
    X, _ = _data()
    cuts, nb = R.quantile_cuts(X, 256)
    bins = R.bin_rows(X, cuts, nb)
    for f in range(X.shape[1]):
        assert np.isinf(cuts[f, nb[f] - 1]) and np.all(np.diff(cuts[f, : nb[f] - 1]) > 0)
        for b in (0, 7, nb[f] // 2, nb[f] - 2):
            # "bins <= b go left" must equal "x < cuts[b]"
            assert np.array_equal(bins[:, f] <= b, X[:, f] < cuts[f, b])
    assert bins[:, : X.shape[1]].max() < 256


def test_few_unique_values_get_few_bins():
    X = np.repeat(np.arange(5, dtype=np.float32), 100)[:, None]
    cuts, nb = R.quantile_cuts(X, 256)
    assert nb[0] == 5 and list(cuts[0, :4]) == [1, 2, 3, 4]


def _brute_best(X, g, h, lam, mcw):
    """Exhaustive search over raw thresholds from the cut set, float64 straight from g/h."""
    best = (-np.inf, None, None)
    G, H = g.sum(), h.sum()
    root = G * G / (H + lam)
    cuts, nb = R.quantile_cuts(X, 256)
    for f in range(X.shape[1]):
        for b in range(nb[f] - 1):
            left = X[:, f] < cuts[f, b]
            GL, HL = g[left].sum(), h[left].sum()
            GR, HR = G - GL, H - HL
            if HL < mcw or HR < mcw:
                continue
            gain = GL * GL / (HL + lam) + GR * GR / (HR + lam) - root
            if gain > best[0] + 1e-9:
                best = (gain, f, b)
    return best


def test_oracle_root_split_matches_brute_force():
    X, y = _data(3000, 4)
    cuts, nb = R.quantile_cuts(X, 256)
    bins = R.bin_rows(X, cuts, nb)
    gs, hs = R.grad_scales(3.0)
    q = R.gradients(np.zeros(len(y), np.float32), y, 3.0, gs, hs)
    tree, _ = R.build_tree(bins, q, cuts, nb, 1, 1.0, 1.0, 0.0, 0.1, gs, hs)
    g, h = q[:, 0] / gs, q[:, 1] / hs
    gain, f, b = _brute_best(X, g, h, 1.0, 1.0)
    assert (tree.feat[0], tree.bin[0]) == (f, b)
    assert tree.gain[0] == pytest.approx(gain, rel=1e-9)


def test_leaf_values_follow_xgboost_weight_rule():
    X, y = _data(2000, 3)
    cuts, nb = R.quantile_cuts(X, 256)
    bins = R.bin_rows(X, cuts, nb)
    gs, hs = R.grad_scales(1.0)
    q = R.gradients(np.zeros(len(y), np.float32), y, 1.0, gs, hs)
    tree, leaf_idx = R.build_tree(bins, q, cuts, nb, 3, 1.0, 1.0, 0.0, 0.3, gs, hs)
    for i in np.unique(leaf_idx):
        sel = leaf_idx == i
        G, H = q[sel, 0].sum() / gs, q[sel, 1].sum() / hs
        expect = 0.0 if H < 1.0 else -G / (H + 1.0) * 0.3
        assert tree.leaf[i] == pytest.approx(expect, rel=1e-6, abs=1e-9)


def test_min_child_weight_blocks_tiny_children():
    X, y = _data(400, 3)
    cuts, nb = R.quantile_cuts(X, 256)
    bins = R.bin_rows(X, cuts, nb)
    gs, hs = R.grad_scales(1.0)
    q = R.gradients(np.zeros(len(y), np.float32), y, 1.0, gs, hs)
    tree, leaf_idx = R.build_tree(bins, q, cuts, nb, 4, 1.0, 20.0, 0.0, 0.1, gs, hs)
    hsum = np.bincount(leaf_idx, weights=q[:, 1] / hs, minlength=16)
    assert np.all((hsum == 0) | (hsum >= 20.0 - 1e-9))


def test_classifier_cpu_quality_and_training_margins():
    from sklearn.ensemble import HistGradientBoostingClassifier
    from sklearn.metrics import roc_auc_score

    X, y = _data(6000, 6, seed=1)
    Xt, yt = _data(3000, 6, seed=2)
    Xs, ys = torch.from_numpy(X), torch.from_numpy(y)
    ens, margin = gb.fit(Xs, ys, gb.GBDTParams(n_estimators=30, max_depth=4), return_margin=True)
    # training margins (bins) == inference margins (float thresholds), bit for bit
    assert np.array_equal(margin.numpy(), gb.predict_margin(Xs, ens).numpy())
    auc = roc_auc_score(yt, gb.predict_margin(torch.from_numpy(Xt), ens).numpy())
    ref = HistGradientBoostingClassifier(max_iter=30, max_depth=4, learning_rate=0.1, random_state=0,
                                         early_stopping=False).fit(X, y)
    auc_ref = roc_auc_score(yt, ref.predict_proba(Xt)[:, 1])
    assert auc > auc_ref - 0.02, (auc, auc_ref)


def test_classifier_api_and_json_roundtrip(tmp_path):
    from fraud_detection_amd.models.gbdt import GBDTClassifier

    X, y = _data(2000, 5)
    m = GBDTClassifier(n_estimators=8, max_depth=3, scale_pos_weight=2.0, device="cpu", objective="binary:logistic",
                       eval_metric="logloss", random_state=42, n_jobs=-1).fit(X, y)
    p = m.predict_proba(X)
    assert p.shape == (2000, 2) and np.allclose(p.sum(1), 1.0)
    assert m.predict(X).shape == (2000,)
    imp = m.feature_importances_
    assert imp.shape == (5,) and imp.sum() == pytest.approx(1.0) and imp[0] > 0
    path = str(tmp_path / "m.json")
    m.save_model(path, [f"f{i}" for i in range(5)])
    json.load(open(path))
    m2 = GBDTClassifier.load_model(path, device="cpu")
    assert np.array_equal(m2.predict_margin(X), m.predict_margin(X))
    assert m2.feature_names_in_ == [f"f{i}" for i in range(5)]
    assert m2.get_params()["scale_pos_weight"] == 2.0


def test_pipeline_cpu_smote_and_artifacts(tmp_path):
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.gbdt import GBDTPipeline
    from fraud_detection_amd.models.pipeline import TrainConfig

    X, y = separable(20_000, fraud_rate=0.02, seed=3)
    Xt, yt = separable(5_000, fraud_rate=0.02, seed=4)
    res = GBDTPipeline(TrainConfig(), gb.GBDTParams(n_estimators=40, max_depth=4)).fit(X, y)
    n_min = int(y.sum())
    assert res.n_train_rows == 2 * (len(y) - n_min)
    assert res.scale_pos_weight == pytest.approx(1.0)  # the fitted (post-SMOTE) rows are balanced
    ev = res.evaluate(Xt, yt)
    assert ev["auc"] > 0.9
    ref = GBDTPipeline(TrainConfig(), gb.GBDTParams(n_estimators=2, max_depth=2), scale_pos_weight="reference").fit(X, y)
    assert ref.scale_pos_weight == pytest.approx((len(y) - n_min) / n_min)  # train_model.py:52-54
    paths = res.save(str(tmp_path), [f"f{i}" for i in range(30)])
    assert os.path.exists(paths["model"]) and os.path.exists(paths["scaler"])
    o = json.load(open(paths["model"]))
    assert o["format"] == "fdx-gbdt/1" and len(o["feat"]) == 40


def test_train_entry_point_gbdt(tmp_path, monkeypatch):
    from fraud_detection_amd import train
    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.data.synthetic import reference_frame

    df = reference_frame(6000, seed=5)
    csv = tmp_path / "cc.csv"
    df.to_csv(csv, index=False)
    monkeypatch.setenv("DATA_CSV", str(csv))
    monkeypatch.setenv("MLFLOW_TRACKING_URI", str(tmp_path / "mlruns"))
    monkeypatch.setenv("MLFLOW_AUC_THRESHOLD", "0.0")
    import fraud_detection_amd.models.gbdt as mg

    orig = gb.GBDTParams
    monkeypatch.setattr(mg.gb, "GBDTParams", lambda **kw: orig(**{"n_estimators": 5, "max_depth": 3, **kw}))
    out = train.run(Settings.load(), model_type="gbdt", cv_folds=2, model_dir=str(tmp_path / "models"), verbose=False)
    assert 0.0 <= out["test_auc"] <= 1.0 and len(out["cv_scores"]) == 2  # random labels: AUC ~ 0.5
    assert os.path.exists(tmp_path / "models" / "xgb_model.json")
    assert out["registered_version"] == 1
    # the reference's artifact contract: joblib.load(models/xgb_model.joblib).predict_proba(scaled X)
    import joblib
    import numpy as np

    from fraud_detection_amd.models.gbdt import GBDTClassifier

    clf = joblib.load(tmp_path / "models" / "xgb_model.joblib")
    assert isinstance(clf, GBDTClassifier)
    js = GBDTClassifier.load_model(str(tmp_path / "models" / "xgb_model.json"), device="cpu")
    sc = joblib.load(tmp_path / "models" / "scaler.joblib")
    Xs = sc.transform(df.drop(columns=["Class"]).to_numpy()[:50])
    clf.device = "cpu"
    np.testing.assert_array_equal(clf.predict_proba(Xs), js.predict_proba(Xs))
    assert clf.params.scale_pos_weight == pytest.approx(out["scale_pos_weight"])
    assert out["scale_pos_weight"] == pytest.approx(1.0, abs=0.01)  # post-SMOTE balance (App. D #11)


def test_fit_binned_hole_equals_explicit_copy_cpu():
    """CPU oracle: a fit over the table minus a block equals the fit on the copy without it, and the
    block's returned margins are the ensemble walked over its bins."""
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import gbdt as gb

    X, y = separable(6000, fraud_rate=0.1, seed=5)
    p = gb.GBDTParams(n_estimators=4, max_depth=3)
    cuts = gb.quantile_cuts(X, p.max_bin)
    bins = gb.bin_rows(X, *cuts)
    ens_h, m_h = gb.fit_binned(bins, y, cuts, p, hole=(1000, 1500), return_margin=True)
    keep = np.r_[0:1000, 2500:6000]
    ens_c, m_c = gb.fit_binned(bins[keep].contiguous(), y[keep].contiguous(), cuts, p, return_margin=True)
    for a in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(ens_h, a), getattr(ens_c, a)), a
    assert torch.equal(m_h[keep], m_c)
    ref = gb.R.predict_margin_bins(bins[1000:2500].numpy(), ens_c.feat, ens_c.bin, ens_c.leaf, 3, ens_c.base_margin)
    np.testing.assert_array_equal(m_h[1000:2500].numpy(), ref)
