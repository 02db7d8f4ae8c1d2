"""K12 device cross-validation of the LOGISTIC model family on one device-resident table.

The reference runs this job with XGBClassifier (train_model.py:58-106); its GBDT counterpart is
models/gbdt_cv.py.  Folds come from a keyed Feistel stratified assignment (ops/split.assign), not
sklearn's StratifiedKFold(shuffle, 42) permutation: statistically equivalent folds, so fold-level
AUC parity with the reference is unpinned -- unless the caller passes ``fold_codes``: train.py hands
in sklearn's StratifiedKFold(5, shuffle=True, random_state=42) membership in ``split=sklearn`` mode
(and the K3 codes of the device split in ``split=device`` mode), so the job's folds are exactly the
per-fold path's (tests/test_cv_gpu.py::test_device_cv_sklearn_folds).

Reference (train_model.py:36-110): StandardScaler fitted once on the training split; 5-fold
StratifiedKFold(shuffle, random_state=42) over it; inside every fold SMOTE(random_state=42) on the
fold's training rows, a fit, predict_proba on the fold's validation rows and roc_auc_score; then
SMOTE on the whole training split, the final fit and the test AUC -- 6 SMOTE + fit + AUC rounds.

MI355X layout (no per-fold copy of the training rows):
  * fold codes: ops/split.assign (keyed Feistel, stratified, sizes within one row per class);
  * one permutation sorts the training rows by fold (five stable compactions; five more list each
    fold's positives);
  * ONE fused scaler pass in scatter form (ops/scaler.scaler_fit_cast(out_idx=...)) reads the raw
    table once, in order, and writes the fold-sorted training table (pivot-shifted bf16 / fp8 rows)
    plus the statistics of the whole split (the reference's single scaler);
  * fold k trains on the table minus its own block: the logistic passes step over the block
    (ops/logreg ``hole``, logreg.hip RowHole);
  * fold k's SMOTE minority = the positive tails of the other folds' blocks: the standardized fp32
    positives are gathered once, fold-sorted, and each fold concatenates its four runs (~1.4 MB);
    exact k-NN among them, virtual samples (never stored);
  * fold k's validation logits come straight from the raw rows under the fit's device weights
    (predict.hip predict_gather_logit), and its exact AUC from the sorted-positives count (the
    fold's positive count is known on the host: no read-back) -- the host never waits inside the job: Newton fits after the first run with the first fold's iteration
    count and are verified at the end (a short prediction finishes the fit and re-scores its fold).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import knn as knn_ops
from ..ops import logreg as lr_ops
from ..ops import metrics as metric_ops
from ..ops import scaler as scaler_ops
from ..ops import split as split_ops
from ..ops.layout import NCOLS, TORCH_STORAGE
from ..ops.native import native, ptr, stream_of
from .pipeline import PipelineResult, TrainConfig, evaluate


@dataclass
class CVResult:
    fold_aucs: list
    final: PipelineResult
    test_auc: float | None
    fold_ms: list = field(default_factory=list)     # device time of each fold (k-NN .. AUC)
    final_ms: float = 0.0                           # device time of the final fit
    prep_ms: float = 0.0                            # fold codes, permutation, scaler pass, positives
    total_ms: float = 0.0                           # wall clock, whole job incl. the test AUC
    fold_iters: list = field(default_factory=list)
    fold_rows: list = field(default_factory=list)   # post-SMOTE training rows of each fold

    @property
    def cv_auc_mean(self) -> float:
        return float(np.mean(self.fold_aucs))

    @property
    def cv_auc_std(self) -> float:
        return float(np.std(self.fold_aucs))


def fold_codes_from_splits(splits, n: int) -> np.ndarray:
    """[(train_idx, val_idx)] * K (sklearn StratifiedKFold.split over n rows) -> uint8 fold code of
    every row (the fold it validates in).  Every row must validate in exactly one fold."""
    codes = np.full(int(n), 255, np.uint8)
    for k, (_, va) in enumerate(splits):
        va = np.asarray(va, dtype=np.int64)
        if (codes[va] != 255).any():
            raise ValueError("a row validates in more than one fold")
        codes[va] = k
    if (codes == 255).any():
        raise ValueError("the folds do not cover every row")
    return codes


def resolve_fold_codes(y: torch.Tensor, K: int, seed: int, fold_codes=None) -> torch.Tensor:
    """The job's per-row fold codes on y's device: the caller's (checked) or the K3 Feistel ones."""
    if fold_codes is None:
        return split_ops.assign(y, test_frac=0.0, n_folds=K, seed=seed)
    c = torch.as_tensor(np.asarray(fold_codes) if not isinstance(fold_codes, torch.Tensor) else fold_codes)
    if c.dim() != 1 or c.shape[0] != y.shape[0]:
        raise ValueError(f"fold_codes must be 1-D with one code per training row ({y.shape[0]})")
    c = c.to(device=y.device, dtype=torch.uint8).contiguous()
    if int(c.max()) >= K:  # one host read per job (the caller's codes are host data anyway)
        raise ValueError(f"fold codes must lie in 0..{K - 1}")
    return c


class DeviceCV:
    """The train_model.py job shape (CV + final fit + AUCs) for the logistic model family on one GPU
    (the reference's XGB family: models/gbdt_cv.DeviceGBDTCV)."""

    def __init__(self, cfg: TrainConfig | None = None, n_folds: int = 5, seed: int = 42, warm_start: bool = True):
        self.cfg = cfg or TrainConfig()
        self.n_folds = int(n_folds)
        self.seed = int(seed)
        # Newton: every fit after the first starts from the previous fit's weights (the same convex
        # objective up to 20% of the rows, so its optimum is near; the fit still runs to the same
        # tolerance from there, without the progressive warm-up)
        self.warm_start = bool(warm_start)
        self._ws: list = []
        self._bws: list = []  # per-fit SMOTE bucket workspaces (side-stream sorts), kept across runs
        self._side = None
        if self.cfg.solver not in ("newton", "sgd"):
            raise ValueError("DeviceCV fits the logistic solvers (newton | sgd)")

    def run(self, X: torch.Tensor, y: torch.Tensor, X_test: torch.Tensor | None = None,
            y_test: torch.Tensor | None = None, fold_codes=None) -> CVResult:
        """``fold_codes``: per-row fold index (0..K-1) of the training rows, e.g. sklearn's
        StratifiedKFold membership (fold_codes_from_splits); None: the keyed Feistel assignment."""
        cfg, K = self.cfg, self.n_folds
        if not X.is_cuda:
            raise ValueError("DeviceCV runs on the device (train.py's CV path covers host tables)")
        if cfg.smote_scope != "global" or not cfg.smote:
            raise ValueError("DeviceCV implements the reference's SMOTE-in-fold semantics (smote=True)")
        dev = X.device
        n, d = X.shape
        t_wall = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 3)]
        ev[0].record()
        # ---- fold codes and the (fold, label) permutation -----------------------------------
        codes = resolve_fold_codes(y, K, self.seed, fold_codes)
        # the table is sorted by fold only: inside a block the rows keep their order, so the
        # sub-sampled warm-up passes (runs of row tiles) see both classes in proportion.  (Sorted by
        # (fold, label), a fold's positives formed one contiguous run that a 1/16 tile sample took
        # whole or missed: 4 full-data Newton iterations per fold instead of 2.)
        key = (codes * 2 + y).to(torch.uint8)
        pend_f = [scaler_ops.compact_indices_async(codes, t) for t in range(K)]
        pend_p = [scaler_ops.compact_indices_async(key, 2 * t + 1) for t in range(K)]
        folds = [p.result() for p in pend_f]
        pos_parts = [p.result() for p in pend_p]
        perm = torch.cat(folds)
        pos = [int(p.shape[0]) for p in pos_parts]
        bounds = np.concatenate([[0], np.cumsum([int(f.shape[0]) for f in folds])]).astype(np.int64)
        pbounds = np.concatenate([[0], np.cumsum(pos)]).astype(np.int64)

        def draw(k: int | None):
            """(minority rows, k, SMOTE samples) of fold k's fit (None: the final fit)."""
            hl = 0 if k is None else int(bounds[k + 1] - bounds[k])
            nm = int(pbounds[-1]) - (0 if k is None else int(pbounds[k + 1] - pbounds[k]))
            nn = max(0, int(round((n - hl - nm) * cfg.sampling_ratio)) - nm) if nm > 0 else 0
            return nm, min(cfg.k_neighbors, nm - 1), nn

        # Every fit's bucket sort needs only its draw, not its neighbours: all of them run on a side
        # stream from here, beside the scaler pass and the first folds (FDX_SMOTE_OVERLAP=0: each
        # in line before its fit).  The workspaces are sized on this stream first, then the side
        # stream starts from its present position (a fresh buffer may reuse a block a queued
        # kernel of this stream still reads).
        pre = {}
        if os.environ.get("FDX_SMOTE_OVERLAP", "scaler") != "0":
            specs = {}
            for k in list(range(K)) + [None]:
                nm, kk, nn = draw(k)
                slot = K if k is None else k
                if nn > 0 and kk >= 1 and nm * kk <= lr_ops.virtual_max_picks() and nn <= lr_ops.virtual_max_samples():
                    while len(self._bws) <= slot:
                        self._bws.append(lr_ops.BucketWorkspace())
                    self._bws[slot].reserve(dev, nm, kk, nn)
                    specs[k] = (slot, nm, kk, nn)
            if specs:
                if self._side is None or self._side.device != dev:
                    self._side = torch.cuda.Stream(dev)
                start = torch.cuda.Event()
                start.record()
                self._side.wait_event(start)
                for k, (slot, nm, kk, nn) in specs.items():
                    w = lr_ops.bucket_lambdas(nm, kk, nn, 0, cfg.seed, 0, dev, self._bws[slot], self._side.cuda_stream)
                    done = torch.cuda.Event()
                    done.record(self._side)
                    pre[k] = (w, done)
        # ---- ONE fused scaler pass: fold-sorted training table + the split's statistics -------
        rows = torch.empty((n, NCOLS), device=dev, dtype=TORCH_STORAGE[cfg.storage])
        dest = torch.empty(n, device=dev, dtype=torch.int64)  # row i of X -> table row dest[i]
        dest[perm] = torch.arange(n, device=dev, dtype=torch.int64)
        stats = scaler_ops.scaler_fit_cast(X, y, rows, fp8_scale=cfg.fp8_scale, out_idx=dest)
        y_perm = y[perm]
        pos_idx = torch.cat(pos_parts)
        xpos = scaler_ops.scale_cast(X, stats, labels=y, out_dtype="f32", idx=pos_idx)  # fold-sorted
        ev[1].record()
        m = native()
        s = stream_of(rows)
        w0 = np.zeros(NCOLS)
        if cfg.init_std > 0:
            w0[:d] = np.random.default_rng(cfg.seed).normal(0.0, cfg.init_std, d)
        fits, logits, aucs, virt_keep = [], [], [], []
        pred = {}          # full-data iterations predicted per kind of fit ("cold" | "warm")
        used_pred = []     # the prediction each fold's fit was enqueued with
        prev_ws = [None]
        # diagnostics (tests): the fold-sorted table and what each fit ran on
        self.rows, self.perm, self.bounds, self.stats, self.virtuals = rows, perm, bounds, stats, []

        def one_fit(k: int | None):
            """Fold k (None: the final fit on the whole split)."""
            if k is None:
                hole, xmin = (0, 0), xpos
            else:
                hole = (int(bounds[k]), int(bounds[k + 1] - bounds[k]))
                xmin = torch.cat([xpos[: pbounds[k]], xpos[pbounds[k + 1]:]])
            n_tr = n - hole[1]
            n_min = int(xmin.shape[0])
            n_new = max(0, int(round((n_tr - n_min) * cfg.sampling_ratio)) - n_min) if n_min > 0 else 0
            cw = (1.0, 1.0)
            if cfg.class_weight == "balanced":
                tot, pw = float(n_tr + n_new), float(n_min + n_new)
                cw = (tot / (2.0 * max(tot - pw, 1.0)), tot / (2.0 * max(pw, 1.0)))
            kk = min(cfg.k_neighbors, n_min - 1)
            parents = torch.empty((n_min, NCOLS), dtype=torch.bfloat16, device=dev)
            nbr = knn_ops.knn_topk(xmin, xmin, k=kk, self_offset=0, parents=parents, parents_affine=stats.aff)
            v = lr_ops.VirtualSmote(parents, nbr.contiguous(), n_new, seed=cfg.seed)
            if k in pre:  # sorted on the side stream: this fit's passes wait for it
                torch.cuda.current_stream(dev).wait_event(pre[k][1])
                v.adopt(pre[k][0])
            else:
                v.prepare()
            # one workspace per fit, kept across runs (every fit of a run is verified before it
            # returns; the pinned flag words are costly to allocate)
            slot = K if k is None else k
            if len(self._ws) <= slot or self._ws[slot].state.device != dev:
                while len(self._ws) <= slot:
                    self._ws.append(None)
                self._ws[slot] = lr_ops.LRWorkspace(dev)
                self._ws[slot].prepare_flags()
            ws = self._ws[slot]
            if cfg.solver == "newton":
                warm = self.warm_start and prev_ws[0] is not None
                kind = "warm" if warm else "cold"
                p = pred.get(kind)
                f = lr_ops.newton_fit(rows, C=cfg.C, tol=cfg.tol, max_iter=cfg.max_iter, d=d, w0=w0, class_w=cw,
                                      fit_intercept=cfg.fit_intercept, fp8_scale=cfg.fp8_scale,
                                      check_every=cfg.check_every, workspace=ws, hess_stride=cfg.hess_stride,
                                      affine=stats.aff, full_iters=p, virtual=v, hole=hole,
                                      progressive=[] if warm else "auto",
                                      w0_from=prev_ws[0].state if warm else None)
                if p is None:  # the first fit of each kind ran host-checked: its count predicts the rest
                    pred[kind] = p = f.full_phase_iters
                used_pred.append(p)
                prev_ws[0] = ws
            else:
                f = lr_ops.sgd_fit(rows, C=cfg.C, lr=cfg.sgd_lr, momentum=cfg.sgd_momentum, epochs=cfg.sgd_epochs,
                                   batches=cfg.sgd_batches, average=cfg.sgd_average, tol=cfg.sgd_tol,
                                   subsample=cfg.sgd_subsample, extra_epochs=cfg.sgd_extra_epochs,
                                   avg_from=cfg.sgd_avg_from, epoch_batches=cfg.sgd_epoch_batches, d=d, w0=w0,
                                   class_w=cw,
                                   fit_intercept=cfg.fit_intercept, fp8_scale=cfg.fp8_scale, workspace=ws,
                                   affine=stats.aff, virtual=v, hole=hole)
            virt_keep.append(v)
            self.virtuals.append(v)
            return f, ws, n_tr + n_new, n_min

        def score(k: int, ws) -> tuple:
            b0, b1 = int(bounds[k]), int(bounds[k + 1])
            z = torch.empty(b1 - b0, device=dev, dtype=torch.float32)
            m.predict_gather_logit(ptr(X), ptr(perm[b0:b1]), b1 - b0, d, ptr(ws.state), ptr(stats.mean64),
                                   ptr(stats.scale64), ptr(z), s)
            # the fold's positive count is known here: the sync-free sorted-positives count (~40 us)
            # instead of the 5-pass radix sort (~240 us at 2M validation rows)
            auc, _ = metric_ops.auc_known_positives(z, y_perm[b0:b1], pos[k])
            return z, auc

        fold_rows = []
        for k in range(K):
            f, ws, n_post, n_min = one_fit(k)
            z, auc = score(k, ws)
            fits.append((f, ws))
            aucs.append(auc)
            fold_rows.append(n_post)
            ev[2 + k].record()
        f_fin, ws_fin, n_post, n_min = one_fit(None)
        ev[2 + K].record()
        # ---- settle: every deferred fit verified; a fit that had to continue is re-scored -----
        for k, (f, ws) in enumerate(fits):
            if isinstance(f, lr_ops.PendingFit) and f.deferred:
                f.verify()
                if f.full_phase_iters > used_pred[k]:
                    aucs[k] = score(k, ws)[1]
        if isinstance(f_fin, lr_ops.PendingFit):
            f_fin.verify()
        torch.cuda.synchronize(dev)
        fold_aucs = [float(a) for a in aucs]
        self.fits = [f for f, _ in fits]
        final = PipelineResult(scaler=stats, fit=f_fin, n_rows=n, n_train_rows=n_post, n_minority=n_min,
                               n_synthetic=n_post - n)
        test_auc = float(evaluate(final, X_test, y_test)["auc"]) if X_test is not None else None
        total = (time.perf_counter() - t_wall) * 1e3
        fold_ms = [ev[1 + k].elapsed_time(ev[2 + k]) for k in range(K)]
        return CVResult(fold_aucs=fold_aucs, final=final, test_auc=test_auc, fold_ms=fold_ms,
                        final_ms=ev[1 + K].elapsed_time(ev[2 + K]), prep_ms=ev[0].elapsed_time(ev[1]),
                        total_ms=total, fold_iters=[int(f.n_iter) for f, _ in fits], fold_rows=fold_rows)
