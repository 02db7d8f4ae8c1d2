"""Inference engine shared by the API, the XAI worker and the library predictors.

Holds one linear model + StandardScaler with the scaler folded into the weights
(ops/predict.py fold_scaler), so a request's raw features are read exactly once by the fused
predict + LinearSHAP kernel (K5/K6).  Device policy: ``device="auto"`` uses the GPU when one is
present; CPU execution is exact fp64 numpy (what the reference's sklearn path computes).

Background for LinearSHAP: the standardized training mean (0 by construction), i.e. the
``shap.LinearExplainer(model, X_train_scaled)`` semantics of explain_model.py:24, with the
attributions defined on the model's standardized inputs.
"""
from __future__ import annotations

import logging
import os
import threading

import numpy as np
import torch

from ..compat.sklearn_export import LinearArtifacts, load_artifacts
from ..ops import predict as P

logger = logging.getLogger(__name__)


def _pick_device(device: str) -> torch.device:
    if device == "auto":
        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


class InferenceEngine:
    def __init__(self, artifacts: LinearArtifacts, device: str = "auto", bg_std: np.ndarray | None = None,
                 source: str = "local"):
        self.art = artifacts
        self.source = source
        self.d = len(artifacts.mean)
        self.feature_names = list(artifacts.feature_names)
        self.a, self.c, self.bias = P.fold_scaler(artifacts.padded_weights(), artifacts.mean, artifacts.scale, bg_std)
        self.device = _pick_device(device)
        self._lock = threading.Lock()
        if self.device.type == "cuda":
            from ..ops.native import native

            native()  # fail loudly rather than serve through an eager fallback
            self._a = torch.from_numpy(self.a).to(self.device)
            self._c = torch.from_numpy(self.c).to(self.device)
            self._stream = torch.cuda.Stream(self.device)

    @classmethod
    def from_paths(cls, model_path=None, scaler_path=None, features_path=None, device="auto") -> "InferenceEngine":
        model_path = model_path or os.getenv("MODEL_PATH", "./models/logistic_model.joblib")
        scaler_path = scaler_path or os.getenv("SCALER_PATH") or os.path.join(os.path.dirname(model_path),
                                                                               "scaler.joblib")
        features_path = features_path or os.getenv("FEATURE_NAMES_PATH", "./models/feature_names.json")
        return cls(load_artifacts(model_path, scaler_path, features_path), device=device, source="local")

    # ---- core ----------------------------------------------------------------------------
    def predict_explain(self, X: np.ndarray):
        """X raw features [B, d] -> (prob [B], logit [B], phi [B, d]) as numpy."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        if X.ndim != 2 or X.shape[1] != self.d:
            raise ValueError(f"expected [B, {self.d}] features, got {X.shape}")
        if self.device.type != "cuda" or X.shape[0] == 0:
            return self._cpu(X)
        with self._lock, torch.cuda.stream(self._stream):
            xt = torch.from_numpy(X).pin_memory().to(self.device, non_blocking=True)
            prob, phi, logit = P.predict_shap_raw(xt, self._a, self._c, self.bias, want_logit=True)
            out = torch.cat([prob[:, None], logit[:, None], phi], 1).cpu()
        o = out.numpy()
        return o[:, 0].astype(np.float64), o[:, 1].astype(np.float64), o[:, 2:].astype(np.float64)

    def _cpu(self, X: np.ndarray):
        Xd = X.astype(np.float64)
        z = Xd @ self.a[: self.d] + self.bias
        p = 1.0 / (1.0 + np.exp(-z))
        phi = self.a[None, : self.d] * (Xd - self.c[None, : self.d])
        return p, z, phi

    def predict(self, X: np.ndarray):
        p, _, _ = self.predict_explain(X)
        return (p > 0.5).astype(np.int64), p

    def expected_value(self) -> float:
        """Model output (log-odds) at the background point: logit(x = c) = sum a*c + bias."""
        return float(self.a[: self.d] @ self.c[: self.d] + self.bias)

    def health(self) -> bool:
        return np.all(np.isfinite(self.a)) and np.isfinite(self.bias)
