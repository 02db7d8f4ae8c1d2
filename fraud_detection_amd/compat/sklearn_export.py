"""Artifact layout compatible with the reference:

    models/logistic_model.joblib   sklearn.linear_model.LogisticRegression (real object)
    models/scaler.joblib           sklearn.preprocessing.StandardScaler   (real object)
    models/columns.joblib          list[str] feature order
    models/feature_names.json      same list as JSON
    models/xgb_model.joblib        GBDT family (when trained): a models.gbdt.GBDTClassifier --
                                   predict / predict_proba on SCALED rows, like the reference's
                                   XGBClassifier dump (train_model.py:113); loading it needs this
                                   package importable, as the reference's needs xgboost
    models/xgb_model.json          the same trees as fdx-gbdt/1 JSON: what serving loads (no pickle)

The GPU-fitted parameters are written into genuine sklearn 1.7 estimator objects, so any tool
that loads the reference's artifacts (api/app.py, predict_single.py, evaluate_model.py, MLflow's
sklearn flavour) can load ours unchanged.  Loading goes the other way through
``load_artifacts``: our own files are loaded with joblib; foreign files (e.g. the reference's
shipped pickles) only through the non-executing decoder in compat/safe_joblib.py.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import joblib
import numpy as np
from sklearn.linear_model import LogisticRegression
from sklearn.preprocessing import StandardScaler

from . import safe_joblib

FEATURE_NAMES = ["Time"] + [f"V{i}" for i in range(1, 29)] + ["Amount"]
MARKER = "fraud_detection_amd"


def make_scaler(mean, var, scale, n_samples_seen, feature_names=None) -> StandardScaler:
    sc = StandardScaler()
    sc.mean_ = np.asarray(mean, dtype=np.float64)
    sc.var_ = np.asarray(var, dtype=np.float64)
    sc.scale_ = np.asarray(scale, dtype=np.float64)
    sc.n_samples_seen_ = int(n_samples_seen)
    sc.n_features_in_ = len(sc.mean_)
    if feature_names is not None:
        sc.feature_names_in_ = np.asarray(feature_names, dtype=object)
    return sc


def make_logistic(coef, intercept, n_iter=0, C=1.0, max_iter=1000, tol=1e-4, solver="lbfgs",
                  feature_names=None, random_state=42) -> LogisticRegression:
    lr = LogisticRegression(C=C, max_iter=max_iter, tol=tol, solver=solver, random_state=random_state)
    lr.coef_ = np.asarray(coef, dtype=np.float64).reshape(1, -1)
    lr.intercept_ = np.asarray([float(np.ravel(intercept)[0])], dtype=np.float64)
    lr.classes_ = np.array([0, 1])
    lr.n_features_in_ = lr.coef_.shape[1]
    lr.n_iter_ = np.asarray([int(n_iter)], dtype=np.int32)
    if feature_names is not None:
        lr.feature_names_in_ = np.asarray(feature_names, dtype=object)
    return lr


@dataclass
class LinearArtifacts:
    coef: np.ndarray        # [d] standardized-space coefficients
    intercept: float
    mean: np.ndarray
    var: np.ndarray
    scale: np.ndarray
    n_samples_seen: int
    feature_names: list
    n_iter: int = 0
    C: float = 1.0
    source: str = MARKER

    def padded_weights(self) -> np.ndarray:
        w = np.zeros(32)
        w[: len(self.coef)] = self.coef
        w[30] = self.intercept
        return w


def save_artifacts(art: LinearArtifacts, model_dir: str = "models", model_name: str = "logistic_model.joblib") -> dict:
    os.makedirs(model_dir, exist_ok=True)
    lr = make_logistic(art.coef, art.intercept, art.n_iter, art.C)
    sc = make_scaler(art.mean, art.var, art.scale, art.n_samples_seen, art.feature_names)
    paths = {
        "model": os.path.join(model_dir, model_name),
        "scaler": os.path.join(model_dir, "scaler.joblib"),
        "columns": os.path.join(model_dir, "columns.joblib"),
        "feature_names": os.path.join(model_dir, "feature_names.json"),
    }
    joblib.dump(lr, paths["model"])
    joblib.dump(sc, paths["scaler"])
    joblib.dump(list(art.feature_names), paths["columns"])
    with open(paths["feature_names"], "w") as f:
        json.dump(list(art.feature_names), f)
    with open(os.path.join(model_dir, ".fdx_provenance.json"), "w") as f:
        json.dump({"writer": MARKER, "model": model_name}, f)
    return paths


def _is_ours(model_dir: str) -> bool:
    return os.path.exists(os.path.join(model_dir, ".fdx_provenance.json"))


def load_artifacts(model_path: str = "models/logistic_model.joblib", scaler_path: str = "models/scaler.joblib",
                   features_path: str = "models/feature_names.json", trusted: bool | None = None) -> LinearArtifacts:
    """Load a linear model + scaler.  ``trusted=None`` trusts only directories this framework
    wrote (provenance marker); anything else is read with the non-executing decoder."""
    model_dir = os.path.dirname(os.path.abspath(model_path))
    if trusted is None:
        trusted = _is_ours(model_dir)
    names = None
    if features_path and os.path.exists(features_path):
        with open(features_path) as f:
            names = json.load(f)
    if trusted:
        lr = joblib.load(model_path)
        sc = joblib.load(scaler_path)
        coef, intercept = lr.coef_[0], float(lr.intercept_[0])
        n_iter = int(np.ravel(getattr(lr, "n_iter_", [0]))[0])
        C = float(getattr(lr, "C", 1.0))
        mean, var, scale, nss = sc.mean_, sc.var_, sc.scale_, int(np.ravel(sc.n_samples_seen_)[0])
        names = names or list(getattr(sc, "feature_names_in_", FEATURE_NAMES))
    else:
        m = safe_joblib.decode_logistic(model_path)
        s = safe_joblib.decode_scaler(scaler_path)
        coef, intercept = m["coef"][0], float(m["intercept"][0])
        n_iter, C = int(m["n_iter"][0]), m["C"]
        mean, var, scale, nss = s["mean_"], s["var_"], s["scale_"], s["n_samples_seen"]
        names = names or s.get("feature_names") or FEATURE_NAMES
    return LinearArtifacts(np.asarray(coef, np.float64), intercept, np.asarray(mean, np.float64),
                           np.asarray(var, np.float64), np.asarray(scale, np.float64), nss, list(names), n_iter, C,
                           MARKER if trusted else "foreign")
