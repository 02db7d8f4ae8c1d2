"""SMOTE estimator with the imblearn API (reference: train_model.py:65-66, preprocess.py:43-44).

``SMOTE(random_state=42, k_neighbors=5, sampling_strategy="auto"|"minority"|float)
.fit_resample(X, y)`` on numpy arrays of already-scaled features (as the reference calls it),
computed with the device k-NN (K8, exact fp32 MFMA) and Philox interpolation (K9).  Output rows
are the originals followed by the synthetic minority rows (imblearn's ordering).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import knn as K
from ..ops.layout import NCOLS


class SMOTE:
    def __init__(self, sampling_strategy="auto", random_state: int = 42, k_neighbors: int = 5, device: str = "auto"):
        self.sampling_strategy = sampling_strategy
        self.random_state = int(random_state or 0)
        self.k_neighbors = k_neighbors
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)

    def _n_new(self, n_min: int, n_maj: int) -> int:
        s = self.sampling_strategy
        if s in ("auto", "minority", "not majority", "all"):
            return max(0, n_maj - n_min)
        if isinstance(s, float):
            return max(0, int(round(s * n_maj)) - n_min)
        raise ValueError(f"unsupported sampling_strategy {s!r}")

    def fit_resample(self, X, y):
        X = np.asarray(X, dtype=np.float32)
        y = np.asarray(y).astype(np.int64)
        n, d = X.shape
        if d > 30:
            raise ValueError("at most 30 features")
        classes, counts = np.unique(y, return_counts=True)
        if len(classes) != 2:
            raise ValueError("binary labels expected")
        minority = classes[np.argmin(counts)]
        mask = y == minority
        n_min, n_maj = int(mask.sum()), int((~mask).sum())
        n_new = self._n_new(n_min, n_maj)
        if n_new == 0:
            return X.copy(), y.copy()
        k = min(self.k_neighbors, n_min - 1)
        if k < 1:
            raise ValueError("SMOTE needs at least 2 minority samples")
        C = np.zeros((n_min, NCOLS), np.float32)
        C[:, :d] = X[mask]
        Ct = torch.from_numpy(C).to(self.device)
        nbr = K.knn_topk(Ct, Ct, k=k, self_offset=0)
        out = torch.empty((n_new, NCOLS), device=self.device, dtype=torch.float32)
        if self.device.type == "cuda":
            # generate in bf16 storage on device, widen: same Philox draws as the CPU path
            outb = torch.empty((n_new, NCOLS), device=self.device, dtype=torch.bfloat16)
            K.smote_generate(Ct, nbr, 0, n_new, outb, seed=self.random_state, counter_base=0)
            out = outb.float()
        else:
            from ..ops import reference as ref

            out = torch.from_numpy(ref.smote_generate(C, nbr.numpy(), 0, n_new, self.random_state, 0))
        Xn = out[:, :d].cpu().numpy()
        X_res = np.concatenate([X, Xn], 0)
        y_res = np.concatenate([y, np.full(n_new, minority, dtype=y.dtype)])
        return X_res, y_res
