"""Gradient-boosted trees family (the reference's XGBoost path, train_model.py:49-114).

* ``GBDTClassifier`` -- estimator with xgboost.XGBClassifier's parameter names
  (n_estimators, learning_rate, max_depth, reg_lambda, min_child_weight, gamma, max_bin,
  scale_pos_weight, base_score) over numpy arrays or torch tensors; device kernels on a GPU
  tensor, the numpy oracle on CPU.  Models serialise to JSON (no pickle).
* ``GBDTPipeline`` -- the reference's per-fold recipe on device: StandardScaler fit on the
  fold's rows -> SMOTE (MFMA k-NN + Philox interpolation, fp32 rows) -> boosting -> exact AUC.
  ``scale_pos_weight="auto"`` (default) is neg/pos of the rows the trees are fit on, i.e. AFTER
  SMOTE (= 1 at sampling_ratio 1): the reference computes neg/pos BEFORE SMOTE
  (train_model.py:52-54) and applies it to the SMOTE-balanced rows (:77), compensating the class
  imbalance twice (AUC 0.9467 < 0.95 on the bench data, profiles/r2_s4b).
  ``scale_pos_weight="reference"`` reproduces that pre-SMOTE value on purpose; a number is used
  as given.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import gbdt as gb
from ..ops import knn as knn_ops
from ..ops import metrics as metric_ops
from ..ops import scaler as scaler_ops
from ..ops.layout import NCOLS
from .pipeline import TrainConfig, global_smote_slices

MODEL_FILE = "xgb_model.json"
JOBLIB_FILE = "xgb_model.joblib"  # the reference's artifact name (train_model.py:113)
_PARAM_FIELDS = frozenset(gb.GBDTParams.__dataclass_fields__)


def _as_tensor(X, device=None, dtype=torch.float32) -> torch.Tensor:
    t = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(X, dtype=np.float32)))
    if device is not None:
        t = t.to(device)
    return t.to(dtype).contiguous() if t.dtype != dtype or not t.is_contiguous() else t


class GBDTClassifier:
    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.1, max_depth: int = 5,
                 reg_lambda: float = 1.0, min_child_weight: float = 1.0, gamma: float = 0.0, max_bin: int = 256,
                 scale_pos_weight: float = 1.0, base_score: float = 0.5, device: str = "auto", **_ignored):
        # xgboost-only knobs the reference passes (objective, eval_metric, random_state, n_jobs)
        # are accepted and ignored: the objective is binary:logistic, the fit is deterministic.
        self.params = gb.GBDTParams(n_estimators=n_estimators, learning_rate=learning_rate, max_depth=max_depth,
                                    reg_lambda=reg_lambda, min_child_weight=min_child_weight, gamma=gamma,
                                    max_bin=max_bin, scale_pos_weight=scale_pos_weight, base_score=base_score)
        self.device = device
        self.ensemble: gb.TreeEnsemble | None = None
        self._dens = None
        self.feature_names_in_ = None

    def _dev(self, X):
        if isinstance(X, torch.Tensor) and self.device == "auto":
            return X.device
        if self.device == "auto":
            return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        return torch.device(self.device)

    def get_params(self, deep: bool = True) -> dict:
        return dict(self.params.__dict__)

    def __getstate__(self):  # joblib/pickle: plain values and host arrays only (no device tensors)
        st = dict(self.__dict__)
        st["_dens"] = None
        st["params"] = dict(self.params.__dict__)
        return st

    def __setstate__(self, st):
        st = dict(st)
        st["params"] = gb.GBDTParams(**{k: v for k, v in st["params"].items() if k in _PARAM_FIELDS})
        self.__dict__.update(st)

    def fit(self, X, y, comm=None):
        dev = self._dev(X)
        Xt = _as_tensor(X, dev)
        yt = (y if isinstance(y, torch.Tensor) else torch.from_numpy(np.asarray(y))).to(dev).to(torch.uint8)
        self.ensemble = gb.fit(Xt, yt.contiguous(), self.params, comm=comm)
        self._dens = None
        return self

    def _check(self):
        if self.ensemble is None:
            raise RuntimeError("model is not fitted")

    def predict_margin(self, X) -> np.ndarray:
        self._check()
        dev = self._dev(X)
        Xt = _as_tensor(X, dev)
        if Xt.is_cuda and (self._dens is None or self._dens.device != Xt.device):
            self._dens = gb.DeviceEnsemble(self.ensemble, Xt.device)
        return gb.predict_margin(Xt, self.ensemble, self._dens).cpu().numpy()

    def predict_proba(self, X) -> np.ndarray:
        p = 1.0 / (1.0 + np.exp(-self.predict_margin(X).astype(np.float64)))
        return np.stack([1.0 - p, p], 1)

    def predict(self, X) -> np.ndarray:
        return (self.predict_margin(X) > 0.0).astype(np.int64)

    @property
    def feature_importances_(self) -> np.ndarray:
        self._check()
        imp = self.ensemble.feature_importance("gain")
        s = imp.sum()
        return imp / s if s > 0 else imp

    def save_model(self, path: str, feature_names=None):
        self._check()
        o = self.ensemble.to_dict()
        o["feature_names"] = list(feature_names) if feature_names is not None else self.feature_names_in_
        with open(path, "w") as f:
            json.dump(o, f)

    @classmethod
    def load_model(cls, path: str, device: str = "auto") -> "GBDTClassifier":
        with open(path) as f:
            o = json.load(f)
        ens = gb.TreeEnsemble.from_dict(o)
        m = cls(device=device, **{k: v for k, v in ens.params.items() if k in _PARAM_FIELDS})
        m.ensemble = ens
        m.feature_names_in_ = o.get("feature_names")
        return m


@dataclass
class GBDTResult:
    scaler: scaler_ops.ScalerStats
    ensemble: gb.TreeEnsemble
    n_rows: int
    n_train_rows: int
    n_minority: int
    n_synthetic: int
    scale_pos_weight: float
    timings: dict = field(default_factory=dict)
    _dens: object = None

    def standardize(self, X: torch.Tensor) -> torch.Tensor:
        rows = scaler_ops.scale_cast(X, self.scaler, out_dtype="f32")
        return rows[:, : self.scaler.d]

    def predict_margin(self, X: torch.Tensor) -> torch.Tensor:
        Xs = self.standardize(X)
        if Xs.is_cuda and (self._dens is None or self._dens.device != Xs.device):
            self._dens = gb.DeviceEnsemble(self.ensemble, Xs.device)
        return gb.predict_margin(Xs, self.ensemble, self._dens)

    def evaluate(self, X: torch.Tensor, y: torch.Tensor, comm=None) -> dict:
        margin = self.predict_margin(X)
        if comm is not None and comm.world_size > 1:
            margin, _ = comm.all_gather_rows(margin.reshape(-1, 1))
            y, _ = comm.all_gather_rows(y.reshape(-1, 1))
            margin, y = margin.reshape(-1).contiguous(), y.reshape(-1).contiguous()
        auc = metric_ops.roc_auc(margin, y)
        tn, fp, fn, tp = (int(v) for v in metric_ops.confusion_counts(margin, y, 0.0))
        return {"auc": auc, "tn": tn, "fp": fp, "fn": fn, "tp": tp, "recall": tp / max(tp + fn, 1),
                "precision": tp / max(tp + fp, 1), "accuracy": (tp + tn) / max(tn + fp + fn + tp, 1)}

    def save(self, model_dir: str, feature_names) -> dict:
        from ..compat.sklearn_export import MARKER, make_scaler
        import joblib

        os.makedirs(model_dir, exist_ok=True)
        mean, var, scale = self.scaler.numpy()
        paths = {"model": os.path.join(model_dir, MODEL_FILE), "joblib": os.path.join(model_dir, JOBLIB_FILE),
                 "scaler": os.path.join(model_dir, "scaler.joblib"),
                 "columns": os.path.join(model_dir, "columns.joblib"),
                 "feature_names": os.path.join(model_dir, "feature_names.json")}
        o = self.ensemble.to_dict()
        o["feature_names"] = list(feature_names)
        o["scale_pos_weight"] = self.scale_pos_weight
        with open(paths["model"], "w") as f:
            json.dump(o, f)
        clf = GBDTClassifier(**{k: v for k, v in self.ensemble.params.items() if k in _PARAM_FIELDS})
        clf.params.scale_pos_weight = float(self.scale_pos_weight)
        clf.ensemble, clf.feature_names_in_ = self.ensemble, list(feature_names)
        joblib.dump(clf, paths["joblib"])
        joblib.dump(make_scaler(mean, var, scale, int(self.scaler.n), feature_names), paths["scaler"])
        joblib.dump(list(feature_names), paths["columns"])
        with open(paths["feature_names"], "w") as f:
            json.dump(list(feature_names), f)
        prov = os.path.join(model_dir, ".fdx_provenance.json")
        meta = {}
        if os.path.exists(prov):
            with open(prov) as f:
                meta = json.load(f)
        meta.update(writer=MARKER, gbdt_model=MODEL_FILE, gbdt_joblib=JOBLIB_FILE)
        meta.setdefault("model", meta.get("model", "logistic_model.joblib"))
        with open(prov, "w") as f:
            json.dump(meta, f)
        return paths

    def log_model(self, mlf, paths: dict) -> str:
        files = {MODEL_FILE: paths["model"], "scaler.joblib": paths["scaler"],
                 "feature_names.json": paths["feature_names"]}
        if paths.get("background"):
            files["shap_background.npy"] = paths["background"]
        return mlf.log_files_model(files, "model", "fdx_gbdt",
                                   {"model_file": MODEL_FILE, "format": "fdx-gbdt/1", "depth": self.ensemble.depth,
                                    "n_trees": self.ensemble.n_trees})


class GBDTPipeline:
    def __init__(self, cfg: TrainConfig | None = None, params: gb.GBDTParams | None = None, comm=None,
                 scale_pos_weight: float | str = "auto", checkpoint_dir: str | None = None,
                 checkpoint_every: int = 10):
        self.cfg = cfg or TrainConfig()
        self.params = params or gb.GBDTParams()
        self.comm = comm
        self.spw = scale_pos_weight
        self.checkpoint_dir, self.checkpoint_every = checkpoint_dir, checkpoint_every

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> GBDTResult:
        cfg = self.cfg
        comm = self.comm if (self.comm is not None and self.comm.world_size > 1) else None
        rank = comm.rank if comm else 0
        t = {}
        t0 = time.perf_counter()
        n, d = X.shape
        stats = scaler_ops.scaler_fit(X, comm=comm)
        idx_min = scaler_ops.compact_indices(y, 1)
        n_min = int(idx_min.shape[0])
        def quota(n_r, nmin_r):
            return max(0, int(round((n_r - nmin_r) * cfg.sampling_ratio)) - nmin_r) if (cfg.smote and nmin_r > 0) else 0

        # SMOTE: single process, or under DP the exact global scheme of models/pipeline.py (every
        # rank a 128-aligned slice of one global draw sequence over all minority rows)
        ranks = comm.all_gather_ints([n_min, n]) if comm else [[n_min, n]]
        if comm:
            per, s_off = global_smote_slices(ranks, quota, rank)
        else:
            per, s_off = [quota(n, n_min)], 0
        n_new = per[rank]
        neg = float(sum(r[1] - r[0] for r in ranks))
        pos = float(sum(r[0] for r in ranks))
        if self.spw == "auto":  # the fitted rows' balance (post-SMOTE)
            spw = neg / (pos + sum(per)) if pos + sum(per) > 0 else 1.0
        elif self.spw == "reference":  # train_model.py:52-54 (pre-SMOTE, App. D #11)
            spw = neg / pos if pos > 0 else 1.0
        else:
            spw = float(self.spw)
        rows = torch.empty((n + n_new, NCOLS), dtype=torch.float32, device=X.device)
        scaler_ops.scale_cast(X, stats, labels=y, out_dtype="f32", out=rows[:n])
        if sum(per) > 0:
            xmin = rows[:n].index_select(0, idx_min).contiguous()
            counts = [r[0] for r in ranks]
            xall = comm.all_gather_rows(xmin, counts=counts)[0] if comm else xmin
            q_off = int(sum(counts[:rank]))
            k = min(cfg.k_neighbors, xall.shape[0] - 1)
            if k < 1:
                raise ValueError("SMOTE needs at least 2 minority samples")
            nbr = knn_ops.knn_topk(xmin, xall, k=k, self_offset=q_off) if n_min > 0 else \
                torch.empty((0, k), dtype=torch.int32, device=X.device)
            if comm:
                nbr = comm.all_gather_rows(nbr, counts=counts)[0]
            if n_new > 0:
                knn_ops.smote_generate(xall, nbr, 0, n_new, rows[n:], seed=cfg.seed, counter_base=0,
                                       sample_offset=s_off)
        labels = torch.empty(n + n_new, dtype=torch.uint8, device=X.device)
        labels[:n] = y
        labels[n:] = 1
        t["prep"] = time.perf_counter() - t0
        params = gb.GBDTParams(**{**self.params.__dict__, "scale_pos_weight": spw})
        ck = None
        if self.checkpoint_dir:
            from ..utils.checkpoint import CheckpointManager

            ck = CheckpointManager(self.checkpoint_dir, prefix="gbdt", keep=2, rank=rank)
        ens = gb.fit(rows[:, :d], labels, params, comm=comm, checkpoint=ck, checkpoint_every=self.checkpoint_every)
        t["boost"] = time.perf_counter() - t0 - t["prep"]
        return GBDTResult(scaler=stats, ensemble=ens, n_rows=n, n_train_rows=n + n_new, n_minority=n_min,
                          n_synthetic=n_new, scale_pos_weight=spw, timings=t)
