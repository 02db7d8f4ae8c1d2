"""K12 device cross-validation of the GBDT family: the reference's actual training job.

Reference (train_model.py:49-110): StandardScaler fitted once on the training split;
StratifiedKFold(5, shuffle, random_state=42); inside every fold SMOTE(random_state=42) on the
fold's training rows, XGBClassifier(n_estimators=100, max_depth=5, learning_rate=0.1) fit,
predict_proba on the fold's validation rows and roc_auc_score; then SMOTE on the whole split, the
final fit and the test AUC -- 6 SMOTE + 6 boosting fits + 6 AUCs.

MI355X layout (no per-fold copy of the training rows):
  * fold codes (ops/split.assign: keyed Feistel, stratified) and ONE fold-sorted permutation;
  * the split's scaler (one statistics pass) and its standardized fp32 rows in fold-sorted order
    (one gathered cast) -> quantile cuts from one strided sample of the whole split -> the binned
    u8 table [n, 32] in fold order; the fp32 copy is dropped once binned;
  * fold k fits the table minus its own block (gbdt.hip row hole, ops/gbdt.fit_binned): level 0
    walks the table around the block and deeper levels follow the partition's row ids;
  * fold k's SMOTE minority = the positive rows of the other folds (standardized fp32, gathered
    once in fold order); exact MFMA k-NN among them and Philox draws; the samples are binned
    straight into the table's tail (labels 1) -- one tail, reused by every fit;
  * every round's margin walk covers the hole too, so after the last round the block's margins ARE
    the fold's validation scores: exact AUC with no separate predict pass;
  * final fit: the whole table + its SMOTE tail; test rows standardized and scored by the GBDT
    predict kernel.
Cuts come from one quantile pass for all six fits (xgboost sketches each fit's own rows); a fold's
fit on an explicit copy of its rows with the same cuts grows bit-identical trees
(tests/test_gbdt_cv_gpu.py).  Folds come from the keyed Feistel assignment unless the caller passes
``fold_codes`` (train.py: sklearn's StratifiedKFold(5, shuffle, 42) membership in split=sklearn
mode, so the folds are the reference's; tests/test_gbdt_cv_gpu.py::test_gbdt_cv_sklearn_folds).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import gbdt as gb
from ..ops import knn as knn_ops
from ..ops import metrics as metric_ops
from ..ops import scaler as scaler_ops
from .cv import resolve_fold_codes
from .gbdt import GBDTResult
from .pipeline import TrainConfig


@dataclass
class GBDTCVResult:
    fold_aucs: list
    final: GBDTResult
    test_auc: float | None
    fold_ms: list = field(default_factory=list)    # device time of each fold (k-NN .. AUC)
    final_ms: float = 0.0
    prep_ms: float = 0.0                           # fold codes, permutation, scaler, cuts, binning
    total_ms: float = 0.0                          # wall clock, whole job incl. the test AUC
    fold_rows: list = field(default_factory=list)  # rows each fold's trees were fit on (real + SMOTE)

    @property
    def cv_auc_mean(self) -> float:
        return float(np.mean(self.fold_aucs))

    @property
    def cv_auc_std(self) -> float:
        return float(np.std(self.fold_aucs))


class DeviceGBDTCV:
    """train_model.py's job (5-fold CV with SMOTE inside each fold, final fit, test AUC) for the
    GBDT family on one GPU, on one binned fold-sorted table."""

    def __init__(self, cfg: TrainConfig | None = None, params: gb.GBDTParams | None = None, n_folds: int = 5,
                 seed: int = 42, scale_pos_weight: float | str = "auto"):
        self.cfg = cfg or TrainConfig()
        self.params = params or gb.GBDTParams()
        self.n_folds = int(n_folds)
        self.seed = int(seed)
        self.spw = scale_pos_weight

    def _spw(self, neg: float, pos: float, pos_fit: float) -> float:
        if self.spw == "auto":  # the fitted rows' balance (post-SMOTE), models/gbdt.GBDTPipeline
            return neg / pos_fit if pos_fit > 0 else 1.0
        if self.spw == "reference":  # train_model.py:52-54 (pre-SMOTE counts, App. D #11)
            return neg / pos if pos > 0 else 1.0
        return float(self.spw)

    def run(self, X: torch.Tensor, y: torch.Tensor, X_test: torch.Tensor | None = None,
            y_test: torch.Tensor | None = None, fold_codes=None) -> GBDTCVResult:
        """``fold_codes``: per-row fold index of the training rows (models/cv.resolve_fold_codes)."""
        cfg, K = self.cfg, self.n_folds
        if not X.is_cuda:
            raise ValueError("DeviceGBDTCV runs on the device (train.py's per-fold path covers host tables)")
        if not cfg.smote:
            raise ValueError("DeviceGBDTCV implements the reference's SMOTE-in-fold semantics (smote=True)")
        dev = X.device
        n, d = X.shape
        t_wall = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 3)]
        ev[0].record()
        # ---- fold codes, fold-sorted permutation, the fold's positives ------------------------
        codes = resolve_fold_codes(y, K, self.seed, fold_codes)
        key = (codes * 2 + y).to(torch.uint8)
        pend_f = [scaler_ops.compact_indices_async(codes, t) for t in range(K)]
        pend_p = [scaler_ops.compact_indices_async(key, 2 * t + 1) for t in range(K)]
        folds = [p.result() for p in pend_f]
        pos_parts = [p.result() for p in pend_p]
        perm = torch.cat(folds)
        pos = [int(p.shape[0]) for p in pos_parts]
        bounds = np.concatenate([[0], np.cumsum([int(f.shape[0]) for f in folds])]).astype(np.int64)
        pbounds = np.concatenate([[0], np.cumsum(pos)]).astype(np.int64)
        # ---- the split's scaler, cuts and the binned fold-sorted table -------------------------
        stats = scaler_ops.scaler_fit(X)
        xs = scaler_ops.scale_cast(X, stats, out_dtype="f32", idx=perm)  # [n, 32] fold-sorted
        p = self.params.validate()
        cuts = gb.quantile_cuts(xs[:, :d], p.max_bin, p.cut_sample_rows)
        n_pos = int(sum(pos))

        def quota(n_tr: int, n_min: int) -> int:
            return max(0, int(round((n_tr - n_min) * cfg.sampling_ratio)) - n_min) if n_min > 0 else 0

        # the SMOTE tail holds the largest quota of the six fits (with sampling_ratio < 1 a fold's
        # quota can exceed the final fit's by rounding near the class balance)
        cap = max([quota(n, n_pos)] + [quota(n - int(bounds[k + 1] - bounds[k]), n_pos - pos[k]) for k in range(K)])
        bins = torch.empty((n + cap, 32), dtype=torch.uint8, device=dev)
        gb.bin_rows(xs[:, :d], cuts[0], cuts[1], out=bins[:n])
        del xs
        lab = torch.empty(n + cap, dtype=torch.uint8, device=dev)
        lab[:n] = y[perm]
        lab[n:] = 1
        xpos = scaler_ops.scale_cast(X, stats, out_dtype="f32", idx=torch.cat(pos_parts))  # fold-sorted positives
        syn = torch.empty((max(cap, 1), 32), dtype=torch.float32, device=dev)  # SMOTE samples before binning
        ev[1].record()
        # diagnostics (tests): the table and each fit's rows
        self.bins, self.labels, self.perm, self.bounds, self.cuts, self.stats = bins, lab, perm, bounds, cuts, stats
        self.fit_rows = []

        def one_fit(k: int | None):
            """Fold k (None: the final fit on the whole split) -> (ensemble, margins of every table row)."""
            if k is None:
                hole, xmin = (0, 0), xpos
            else:
                hole = (int(bounds[k]), int(bounds[k + 1] - bounds[k]))
                xmin = torch.cat([xpos[: pbounds[k]], xpos[pbounds[k + 1]:]])
            n_tr = n - hole[1]
            n_min = int(xmin.shape[0])
            n_new = quota(n_tr, n_min)
            if n_new > 0:
                kk = min(cfg.k_neighbors, n_min - 1)
                if kk < 1:
                    raise ValueError("SMOTE needs at least 2 minority samples")
                nbr = knn_ops.knn_topk(xmin, xmin, k=kk, self_offset=0)
                knn_ops.smote_generate(xmin, nbr, 0, n_new, syn[:n_new], seed=cfg.seed)
                gb.bin_rows(syn[:n_new, :d], cuts[0], cuts[1], out=bins[n:n + n_new])
            spw = self._spw(float(n_tr - n_min), float(n_min), float(n_min + n_new))
            params = gb.GBDTParams(**{**p.__dict__, "scale_pos_weight": spw})
            ens, margin = gb.fit_binned(bins[:n + n_new], lab[:n + n_new], cuts, params, hole=hole,
                                        return_margin=True)
            self.fit_rows.append((hole, n_new))
            return ens, margin, n_tr + n_new, n_min, n_new, spw

        self._one_fit = one_fit  # tests: refit one fold against the same table
        aucs, fold_rows = [], []
        for k in range(K):
            _, margin, n_fit, _, _, _ = one_fit(k)
            b0, b1 = int(bounds[k]), int(bounds[k + 1])
            auc, _ = metric_ops.auc_known_positives(margin[b0:b1].contiguous(), lab[b0:b1], pos[k])
            aucs.append(auc)
            fold_rows.append(n_fit)
            ev[2 + k].record()
        ens, _, n_fit, n_min, n_new, spw = one_fit(None)
        ev[2 + K].record()
        final = GBDTResult(scaler=stats, ensemble=ens, n_rows=n, n_train_rows=n_fit, n_minority=n_min,
                           n_synthetic=n_new, scale_pos_weight=spw)
        test_auc = None
        if X_test is not None and y_test is not None:
            test_auc = float(final.evaluate(X_test, y_test)["auc"])
        torch.cuda.synchronize(dev)
        fold_aucs = [float(a) for a in aucs]
        return GBDTCVResult(fold_aucs=fold_aucs, final=final, test_auc=test_auc,
                            fold_ms=[ev[1 + k].elapsed_time(ev[2 + k]) for k in range(K)],
                            final_ms=ev[1 + K].elapsed_time(ev[2 + K]), prep_ms=ev[0].elapsed_time(ev[1]),
                            total_ms=(time.perf_counter() - t_wall) * 1e3, fold_rows=fold_rows)
