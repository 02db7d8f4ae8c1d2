"""End-to-end device training pipeline: the MI355X replacement for train_model.py's hot path.

Reference call stack (train_model.py:20-114):
    split -> StandardScaler.fit(train) -> SMOTE(k=5).fit_resample -> classifier.fit -> AUC
Here every numeric step is a HIP kernel on the rank's row shard:
    K1 scaler stats (+ all-reduce C1) -> K2 standardize/pad/cast into the training buffer
    -> stable minority compaction -> K2 gather (fp32 minority rows) -> all-gather C3
    -> K8 MFMA k-NN (local queries vs global minority) -> K9 Philox SMOTE rows written in place
       from bf16 parents in the training rows' space -- or, for the Newton fit, regenerated
       inside every K4 pass (TrainConfig.virtual_smote)
    -> K4 Newton (all-reduce C5 per iteration) or minibatch SGD (all-reduce C4 per minibatch), both
       folding the virtual SMOTE samples into their passes
Evaluation: folded-scaler predict on raw fp32 test rows (K5) -> exact AUC (K10) + confusion.
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
from ..ops import predict as pred_ops
from ..ops import scaler as scaler_ops
from ..obs import tracing
from ..ops.layout import BIAS_COL, DEFAULT_FP8_SCALE, NCOLS, TORCH_STORAGE


@dataclass
class TrainConfig:
    solver: str = "newton"          # newton | sgd
    C: float = 1.0
    tol: float = 1e-4               # max |grad| of the mean objective: the reference model's
                                    # LogisticRegression(tol=1e-4) lbfgs stopping rule (App. C)
    max_iter: int = 25
    fit_intercept: bool = True
    class_weight: str | None = None  # None | "balanced"
    smote: bool = True
    k_neighbors: int = 5
    sampling_ratio: float = 1.0     # minority : majority after SMOTE (1.0 = imblearn 'auto')
    seed: int = 42
    storage: str = "bf16"           # bf16 | fp8
    # Newton on GPU (bf16 or fp8 rows): scaler statistics and the row cast share one read of X
    # (rows stay shifted / prescaled; the solver applies the standardization as an exact affine
    # map of its sums)
    fold_scaler: bool = True
    fp8_scale: float = DEFAULT_FP8_SCALE
    # minibatch SGD (config 3, ops/logreg.sgd_fit): `sgd_batches` disjoint strided minibatches per
    # epoch, curvature-normalised momentum steps (per-epoch step scalars), Polyak averaging over the
    # last epoch, convergence state on the epoch gradient
    sgd_lr: tuple = lr_ops.SGD_LR
    sgd_momentum: float = lr_ops.SGD_MOMENTUM
    sgd_epochs: int = lr_ops.SGD_EPOCHS
    sgd_batches: int = lr_ops.SGD_BATCHES
    sgd_subsample: tuple = lr_ops.SGD_SUB  # per-epoch row sub-sample (growing-batch schedule)
    sgd_extra_epochs: int = lr_ops.SGD_EXTRA_EPOCHS  # run only while not converged
    sgd_avg_from: int = lr_ops.SGD_AVG_FROM  # first Polyak-averaged epoch
    sgd_epoch_batches: tuple = lr_ops.SGD_EPOCH_BATCHES  # per-epoch minibatch counts
    sgd_average: bool = True
    sgd_tol: float = lr_ops.SGD_TOL
    check_every: int = 1            # Newton: iterations per convergence-flag read (host reads one chunk behind)
    # Newton, one process, resident rows: enqueue the full-data iteration count the previous fit
    # of this shape needed and verify convergence when the training buffer is next reused (two
    # buffers alternate) -- no host wait and no trailing no-op iterations inside the fit
    deferred_check: bool = True
    init_std: float = 0.01          # random-init weights ~ N(0, init_std^2) (seeded by `seed`)
    hess_stride: int | str = "auto"  # Newton: Hessian from every k-th row tile (gradient always exact)
    # SMOTE under data parallelism: "global" = the single-process result exactly -- every rank
    # draws a 128-aligned slice of ONE global sample sequence over ALL minority rows and their
    # global neighbours (all-gather of minority rows C3 and of the k-NN index rows), so the union
    # of the ranks' synthetic rows equals the one-process SMOTE output bit for bit; "shard" = each
    # rank oversamples its own minority rows (per-partition SMOTE: constant work per rank)
    smote_scope: str = "global"
    # Both solvers, bf16 or fp8 device rows: the SMOTE rows are never stored.  Each sample's lambda
    # is bucketed by pick once per fit; every logistic pass folds a pick's samples in through
    # fixed-point sums over its lambdas against the two L2-resident parent rows
    # (ops/logreg.VirtualSmote, logreg.hip pick_terms).  The interpolants enter at fp32 (the stored
    # path rounds each to bf16 / e4m3).  At the bench shape half the training rows are synthetic:
    # no 512 MB SMOTE write and half the bytes per pass.
    virtual_smote: bool = True


@dataclass
class PipelineResult:
    scaler: scaler_ops.ScalerStats
    fit: lr_ops.FitInfo            # or lr_ops.PendingFit (device fits: read lazily)
    n_rows: int                    # local raw training rows
    n_train_rows: int              # local post-SMOTE rows
    n_minority: int
    n_synthetic: int
    timings: dict = field(default_factory=dict)

    @property
    def w(self) -> np.ndarray:
        """[32] float64 standardized-space weights, w[30] = intercept."""
        return self.fit.w

    @property
    def coef(self) -> np.ndarray:
        return self.w[: self.scaler.d].copy()

    @property
    def intercept(self) -> float:
        return float(self.w[BIAS_COL])

    def folded(self, bg_std=None):
        mean, _, scale = self.scaler.numpy()
        return pred_ops.fold_scaler(self.w, mean, scale, bg_std)


class _Timer:
    """Phase timer (profile=True: device-synchronised wall time per phase) and, with
    FDX_ROCTX_PHASES=1, a roctx marker at every phase end so ``rocprofv3 --marker-trace`` lines the
    kernels up with the pipeline phases (the fit itself is one roctx range, see DevicePipeline)."""

    def __init__(self, device, enabled: bool):
        self.enabled = enabled and device.type == "cuda"
        self.device = device
        self.t = {}
        self._last = time.perf_counter()
        self.rx = tracing.roctx_phases() if device.type == "cuda" else None
        if self.rx is not None:
            self.rx.roctxRangePushA(b"fdx.pipeline.fit")

    def mark(self, name: str):
        if self.rx is not None:
            tracing.roctx_mark(self.rx, "fdx.phase_end:" + name)
            if name == "fit":  # the solver is the last phase of every fit path
                self.rx.roctxRangePop()
        if not self.enabled:
            return
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        self.t[name] = self.t.get(name, 0.0) + (now - self._last)
        self._last = now


class DevicePipeline:
    def __init__(self, cfg: TrainConfig | None = None, comm=None):
        self.cfg = cfg or TrainConfig()
        self.comm = comm
        self._ws = None
        self._buf = None   # the training buffer of the latest fit
        # deferred convergence checks: two training buffers / solver workspaces alternate; the fit
        # whose rows live in buffer b is verified before b is written again
        self._bufs, self._wss, self._pending = [None, None], [None, None], [None, None]
        self._bi = self._cur = 0
        self._full_pred = None  # (signature, full-data iterations of the last settled fit)
        self._virtual = None    # VirtualSmote of the latest fit (None: its SMOTE rows are stored)
        # its bucket buffers, one set per training buffer (a fit's set is reused once it is settled)
        self._bws = [lr_ops.BucketWorkspace(), lr_ops.BucketWorkspace()]
        self._side = None  # side stream of the SMOTE bucket sort (overlaps the k-NN)
        self._defer_now = False

    def _side_stream(self, dev) -> torch.cuda.Stream:
        if self._side is None or self._side.device != dev:
            # FDX_SMOTE_SIDE_PRIO=-1: a high-priority side stream (lab knob; torch's range is [-1, 0])
            self._side = torch.cuda.Stream(dev, priority=int(os.environ.get("FDX_SMOTE_SIDE_PRIO", "0")))
        return self._side

    def _world(self):
        c = self.comm
        return (c.rank, c.world_size) if c is not None else (0, 1)

    def _settle(self, b: int):
        """Verify the fit whose rows live in buffer b (finishing it if its predicted iteration
        count was short) and learn its full-data iteration count for the next prediction."""
        f, self._pending[b] = self._pending[b], None
        if f is not None:
            sig = f._fdx_sig
            f.verify()
            self._full_pred = (sig, f.full_phase_iters)

    def settle(self) -> "DevicePipeline":
        """Verify every fit still waiting for its deferred convergence check.  Under data
        parallelism this is a collective point: every rank calls it at the same place (its
        continuation may run gradient all-reduces); a DP fit's fields can only be read after it."""
        for b in range(2):
            self._settle(b)
        return self

    def _train_buffer(self, n_rows: int, device, allow_double: bool = False) -> torch.Tensor:
        cfg = self.cfg
        dt = TORCH_STORAGE[cfg.storage]
        world = self._world()[1]
        double = allow_double and cfg.deferred_check and cfg.solver == "newton" and device.type == "cuda"
        b = self._bi if double else 0
        for i in range(2):  # a buffer about to be written must not hold an unverified fit
            if i == b or not double:
                self._settle(i)
        buf = self._bufs[b]
        if buf is None or buf.shape[0] < n_rows or buf.device != device or buf.dtype != dt:
            self._bufs[b] = None
            need = n_rows * NCOLS * torch.empty((), dtype=dt).element_size()
            # under DP every rank must take the same branch (the deferred fit's collectives run at
            # different points than a checked fit's): decide from the device's total memory, which
            # is the same on every rank, not from its free memory
            def room():
                return (torch.cuda.get_device_properties(device).total_memory // 2 if world > 1
                        else torch.cuda.mem_get_info(device)[0])
            if double and b == 1 and room() < 2 * need:
                double, b = False, 0  # no room for a second buffer: checked fits, one buffer
                self._settle(0)
                buf = self._bufs[0]
            if buf is None or buf.shape[0] < n_rows or buf.device != device or buf.dtype != dt:
                buf = self._bufs[b] = torch.empty((n_rows, NCOLS), device=device, dtype=dt)
        if double:
            # allocate the other buffer NOW too: its first allocation (a large hipMalloc, ~0.1 s)
            # must land in the first fit, not in whichever later fit first alternates to it
            o = self._bufs[b ^ 1]
            if o is None or o.shape[0] < n_rows or o.device != device or o.dtype != dt:
                self._bufs[b ^ 1] = torch.empty((n_rows, NCOLS), device=device, dtype=dt)
        self._buf, self._cur, self._defer_now = buf, b, double
        return buf[:n_rows]

    def training_rows(self, res: "PipelineResult") -> torch.Tensor:
        """The latest fit's post-SMOTE training rows as one stored tensor (diagnostic tools): a
        fit over virtual SMOTE rows has them materialised into the buffer's tail first."""
        rows = self._buf[: res.n_train_rows]
        if self._virtual is not None:
            self._virtual.materialize(rows[res.n_rows:], self.cfg.fp8_scale)
        return rows

    def training_objective(self, res: "PipelineResult", w: np.ndarray | None = None) -> dict:
        """The exact objective (sklearn's: mean weighted log-loss + ||w||^2 / (2 C S)) and gradient
        max-norm of standardized-space weights ``w`` (default: the latest fit's) over the latest
        fit's training set -- stored rows plus its SMOTE samples, virtual or stored -- from one
        device pass (the solvers' own sums, not an estimate).  Diagnostic: compares solvers on
        the same training set; call it before the next fit reuses the buffers."""
        cfg = self.cfg
        w = np.asarray(res.w if w is None else w, dtype=np.float64).copy()
        rows = self._buf[: res.n_rows] if self._virtual is not None else self._buf[: res.n_train_rows]
        d = res.scaler.d
        aff = getattr(res.scaler, "aff", None)
        wf = w.copy()
        if aff is not None:  # pivot-shifted rows: fold the standardization into the weights
            a = aff.double().cpu().numpy()
            c, inv = a[:32], a[32:]
            wf[:d] = w[:d] * inv[:d]
            wf[BIAS_COL] = w[BIAS_COL] - float(np.sum(w[:d] * inv[:d] * c[:d]))
        wf[31] = 0.0
        cw = (1.0, 1.0)
        if cfg.class_weight == "balanced":
            tot, pos = float(res.n_train_rows), float(res.n_minority + res.n_synthetic)
            cw = (tot / (2.0 * max(tot - pos, 1.0)), tot / (2.0 * max(pos, 1.0)))
        g, loss, wsum, _ = lr_ops.logreg_pass(rows, torch.from_numpy(wf).float(), class_w=cw, hessian=False,
                                              fp8_scale=cfg.fp8_scale, virtual=self._virtual)
        if aff is not None:
            g = g.copy()
            g[:d] = inv[:d] * (g[:d] - c[:d] * g[BIAS_COL])
        S = wsum if wsum > 0 else 1.0
        grad = np.zeros(32)
        grad[:d] = g[:d] / S + w[:d] / (cfg.C * S)
        if cfg.fit_intercept:
            grad[BIAS_COL] = g[BIAS_COL] / S
        return {"objective": loss / S + 0.5 * float(w[:d] @ w[:d]) / (cfg.C * S),
                "grad_max": float(np.abs(grad).max()), "weight": wsum}

    def fit_host(self, X: torch.Tensor, y: torch.Tensor, device=None, budget: int | None = None,
                 profile: bool = False) -> PipelineResult:
        """Fit from host-resident raw rows (the parsed table), planned against free HBM
        (runtime/hbm.py): ``resident`` uploads once and runs the fused fast path; ``stream_raw``
        keeps the raw shard on the host and streams it twice (exact statistics, then
        standardize+cast into the device-resident training rows) -- a shard larger than HBM
        trains as long as its training rows fit."""
        from ..runtime import hbm

        cfg = self.cfg
        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        n, d = X.shape
        frac = float(y[: 1 << 20].float().mean()) if n else 0.0
        plan = hbm.plan_fit(n, d, cfg.storage, cfg.smote, cfg.sampling_ratio, minority_frac=max(frac, 1e-3),
                            dev=dev, budget=budget)
        self.last_plan = plan
        if plan.mode == "resident":
            res = self.fit(X.to(dev, non_blocking=True), y.to(dev, non_blocking=True), profile)
        else:
            res = self._fit_streaming(X, y, dev, plan, profile)
        res.timings["hbm_plan"] = plan.as_dict()
        hbm.observe_hbm(dev)
        return res

    def _fit_streaming(self, X, y, dev, plan, profile) -> PipelineResult:
        cfg = self.cfg
        rank, world = self._world()
        comm = self.comm if world > 1 else None
        tm = _Timer(dev, profile)
        n, d = X.shape
        cap = n + (int(np.ceil(n * max(cfg.sampling_ratio, 1.0))) + 128 if cfg.smote else 0)
        rows_cap = self._train_buffer(cap, dev)
        chunks = _HostChunks(X, y, dev, plan.chunk_rows)
        pivot = X[0].to(dev, torch.float32) if n else torch.zeros(d, device=dev)
        if comm is not None:
            pivot = comm.broadcast(pivot.contiguous(), src=0)
        # pass 1: exact shifted fp64 sums over the streamed chunks (C1 all-reduce after)
        sums = torch.zeros(64, dtype=torch.float64, device=dev)
        for _, xd, _ in chunks:
            sums += scaler_ops.scaler_partial_sums(xd, pivot)
        if comm is not None:
            sums[31:32].fill_(float(n))
            sums = comm.all_reduce(sums)
            stats = scaler_ops.scaler_finalize(sums, None, pivot, d)
        else:
            stats = scaler_ops.scaler_finalize(sums, float(n), pivot, d)
        tm.mark("scaler_fit")
        # pass 2: standardize + cast into the resident training rows; minority rows in fp32
        xmins = []
        for c0, xd, yd in chunks:
            m = xd.shape[0]
            scaler_ops.scale_cast(xd, stats, labels=yd, out_dtype=cfg.storage, out=rows_cap[c0:c0 + m],
                                  fp8_scale=cfg.fp8_scale)
            idx = scaler_ops.compact_indices(yd, 1)
            if idx.numel():
                xmins.append(scaler_ops.scale_cast(xd, stats, labels=yd, out_dtype="f32", idx=idx))
        xmin = torch.cat(xmins) if xmins else torch.empty((0, NCOLS), dtype=torch.float32, device=dev)
        _maybe_fault(rank)
        # host_ordered: the last chunk's compact_indices waited for its count, behind every earlier kernel
        return self._finish(stats, rows_cap, n, d, int(xmin.shape[0]), False, tm, comm, rank, dev, lambda: xmin,
                            host_ordered=n > 0)

    def fit(self, X: torch.Tensor, y: torch.Tensor, profile: bool = False) -> PipelineResult:
        cfg = self.cfg
        if cfg.smote_scope not in ("global", "shard"):
            raise ValueError("smote_scope must be 'global' or 'shard'")
        dev = X.device
        rank, world = self._world()
        comm = self.comm if world > 1 else None
        tm = _Timer(dev, profile)
        n, d = X.shape
        fused = (cfg.fold_scaler and cfg.storage in ("bf16", "fp8") and cfg.solver in ("newton", "sgd")
                 and dev.type == "cuda" and scaler_ops.fused_cast_ok(X))
        # training buffer sized for the largest possible SMOTE output, so the cast does not wait
        # for the minority count (+128: a global-scope slice boundary moves by < 128 rows)
        cap = n + (int(np.ceil(n * max(cfg.sampling_ratio, 1.0))) + 128 if cfg.smote else 0)
        rows_cap = self._train_buffer(cap, dev, allow_double=True)
        self._fit_start = None  # set below on the fused path only (never an earlier fit's event)
        if fused:
            # ---- K1+K2 fused: statistics (C1 all-reduce inside) + shifted bf16 / fp8 rows ----
            # ---- class counts (C2) IN FRONT of the pass on the compute stream: the count/scan read
            # only the labels (~10 us), their total lands in a mapped pinned word, and the host
            # enqueues the whole minority -> k-NN -> SMOTE chain while the 265 us pass runs, so the
            # chain starts with no host gap.  With the Newton fit's deferred convergence check the
            # host is a fit ahead, so the count no longer sits behind a host wait at the fit
            # boundary (profiles/r3_q/count_front_ab.txt: 1.273 vs 1.309 ms per step with the
            # count on a side stream beside the pass, the round-2 winner).
            # the compute stream's position before this fit: under FDX_SMOTE_OVERLAP=scaler the SMOTE
            # bucket sort's side stream starts from here, beside the scaler pass (_finish).  Only
            # then: the marker costs the command processor ~7 us at the fit boundary (r6_marker)
            if os.environ.get("FDX_SMOTE_OVERLAP", "knn") == "scaler":
                self._fit_start = torch.cuda.Event()
                self._fit_start.record()
            pending = scaler_ops.compact_indices_async(y, 1)
            stats = scaler_ops.scaler_fit_cast(X, y, rows_cap[:n], comm=comm, fp8_scale=cfg.fp8_scale)
            tm.mark("scaler_fit")
        else:
            # ---- K1: scaler statistics (C1 all-reduce inside) ----------------------------
            stats = scaler_ops.scaler_fit(X, comm=comm)
            tm.mark("scaler_fit")
            pending = scaler_ops.compact_indices_async(y, 1)
            # ---- K2: standardize + pad + cast the real rows (label in col 31) --------------
            scaler_ops.scale_cast(X, stats, labels=y, out_dtype=cfg.storage, out=rows_cap[:n],
                                  fp8_scale=cfg.fp8_scale)
        idx_min = pending.result()
        n_min = int(idx_min.shape[0])
        _maybe_fault(rank)
        return self._finish(stats, rows_cap, n, d, n_min, fused, tm, comm, rank, dev,
                            lambda: scaler_ops.scale_cast(X, stats, labels=y, out_dtype="f32", idx=idx_min),
                            host_ordered=True)

    def _finish(self, stats, rows_cap, n, d, n_min, fused, tm, comm, rank, dev, get_xmin,
                host_ordered: bool = False) -> PipelineResult:
        """SMOTE (+ DP exchange) and the solver on the device-resident training rows
        rows_cap[:n] (shared by the resident and the host-streaming preparation).  host_ordered:
        the host has waited for a compute-stream result enqueued behind every earlier kernel (the
        minority count), so everything enqueued before this fit has finished."""
        cfg = self.cfg

        def quota(n_r, nmin_r):
            return max(0, int(round((n_r - nmin_r) * cfg.sampling_ratio)) - nmin_r) if (cfg.smote and nmin_r > 0) else 0

        # DP: one small all-gather of (minority, rows) per rank gives every rank the minority
        # counts (for the row all-gather) and every rank's post-SMOTE size (for the identical
        # Newton schedule) -- no further host-synchronising collectives in the fit.
        ranks = comm.all_gather_ints([n_min, n]) if comm is not None else [[n_min, n]]
        glob = comm is not None and cfg.smote_scope == "global"
        if glob:
            new_per_rank, s_off = global_smote_slices(ranks, quota, rank)
        else:
            new_per_rank, s_off = [quota(r[1], r[0]) for r in ranks], 0
        n_new = new_per_rank[rank]
        n_sched = min(r[1] + q for r, q in zip(ranks, new_per_rank))
        if n + n_new > rows_cap.shape[0]:  # global_smote_slices guarantees this never fires
            raise RuntimeError(f"SMOTE slice of {n_new} rows exceeds the training buffer ({rows_cap.shape[0]} rows)")
        rows = rows_cap[: n + n_new]
        # ---- class weights ---------------------------------------------------------------
        class_w = (1.0, 1.0)
        if cfg.class_weight == "balanced":  # global counts from the exchanged (minority, rows) pairs
            tot = float(sum(r[1] + q for r, q in zip(ranks, new_per_rank)))
            pos = float(sum(r[0] + q for r, q in zip(ranks, new_per_rank)))
            class_w = (tot / (2.0 * max(tot - pos, 1.0)), tot / (2.0 * max(pos, 1.0)))
        virt = None
        # Both row formats, both solvers: the SMOTE samples are generated inside every pass instead of
        # being written once and streamed by every pass.  (fp8 Newton took stored rows until its pass
        # could run pick tiles mid-loop without spilling -- logreg.hip logreg_pass_fp8w_kernel.)
        virt_ok = (cfg.virtual_smote and dev.type == "cuda" and class_w[1] <= lr_ops.VIRTUAL_MAX_WEIGHT
                   and cfg.solver in ("newton", "sgd"))
        tm.mark("scale_cast")
        # global scope: every rank joins the row and neighbour all-gathers whenever ANY rank has a
        # quota; shard scope has no collective in this block, so only a rank with its own quota enters
        if (sum(new_per_rank) > 0) if glob else (n_new > 0):
            # ---- minority rows in fp32, gathered across ranks (C3) -----------------------
            xmin = get_xmin()
            if glob:
                xall, counts = comm.all_gather_rows(xmin, counts=[r[0] for r in ranks])
                q_off = int(sum(counts[:rank]))
            else:
                xall, q_off = xmin, 0
            tm.mark("minority_gather")
            k = min(cfg.k_neighbors, xall.shape[0] - 1)
            if k < 1:
                raise ValueError("SMOTE needs at least 2 minority samples")
            # Virtual SMOTE's bucket sort needs only the draw (picks = minority rows x k, samples,
            # seed), not the neighbour table: it can run on a side stream.  FDX_SMOTE_OVERLAP: "knn"
            # (default) the whole sort from here on, with no event in front of it unless its buffers
            # grew -- it runs beside the scaler pass that is still going; "scaler" counts + records
            # from the fit's start and the lambda assembly beside the k-NN; "0" in line (quick
            # benches, profiles/r6_marker: 0.983 / 0.980 / 1.018 ms means, 0.978 / 0.971 / 1.010
            # medians; before the events came off the fit boundary, r6_smote_overlap: 0.990 /
            # 0.995-1.003 / 1.029 medians).
            mq_all = int(xall.shape[0])  # the neighbour table's rows (all ranks' under global scope)
            use_virt = (n_new > 0 and virt_ok and mq_all * k <= lr_ops.virtual_max_picks()
                        and n_new <= lr_ops.virtual_max_samples())
            pre_w = None
            mode = os.environ.get("FDX_SMOTE_OVERLAP", "knn")
            if use_virt and mode != "0":
                main = torch.cuda.current_stream(dev)
                side = self._side_stream(dev)
                # buffers (re)allocated now come from the compute stream's pool, possibly from
                # blocks its queued kernels still use: then the sort waits for the present position
                grew = self._bws[self._cur].reserve(dev, mq_all, k, n_new)
                # Otherwise every earlier use of the buffers (an earlier fit's passes) is already
                # done: the host has seen this fit's minority count (idx_min above), written by a
                # kernel behind all of them on the compute stream -- no event needed, and the sort
                # starts at once, beside the scaler pass.  An event recorded behind the scaler pass
                # costs a marker there and holds the sort back into the k-NN's critical path
                # (profiles/r6_marker).
                ev = getattr(self, "_fit_start", None) if (mode == "scaler" and not grew) else None
                if ev is None and (grew or not host_ordered):
                    ev = torch.cuda.Event()
                    ev.record(main)
                self._fit_start = None
                if ev is not None:
                    side.wait_event(ev)
                bargs = (mq_all, k, n_new, s_off, cfg.seed, 0 if glob else rank, dev, self._bws[self._cur],
                         side.cuda_stream)
                if mode == "scaler":
                    # counts + records beside the scaler pass; the lambda assembly (stage 2) waits for
                    # the k-NN, whose latency-bound collect leaves CUs idle -- beside the small
                    # memory-bound kernels in between it slowed each of them ~3x (profiles/r6_p5)
                    lr_ops.bucket_lambdas(*bargs, stages=(0, 1))
                    at_knn = torch.cuda.Event()
                    at_knn.record(main)
                    side.wait_event(at_knn)
                    pre_w = lr_ops.bucket_lambdas(*bargs, stages=(2,))
                else:
                    pre_w = lr_ops.bucket_lambdas(*bargs)
                bucket_done = torch.cuda.Event()
                bucket_done.record(side)
            # SMOTE interpolation is affine-equivariant: with pivot-shifted training rows the
            # neighbours found in standardized space are interpolated in shifted coordinates.
            # Parents live in the training rows' space (bf16, pivot-shifted when the scaler is
            # folded): half the gather bytes of fp32 parents and no per-sample affine map.  The
            # k-NN operand prep writes them from the same read of the minority rows.
            parents = None
            if n_new > 0 and n_min > 0:
                parents = torch.empty((xall.shape[0], NCOLS), dtype=torch.bfloat16, device=dev)
            nbr = knn_ops.knn_topk(xmin, xall, k=k, self_offset=q_off, parents=parents,
                                   parents_affine=stats.aff if (fused and parents is not None) else None) \
                if n_min > 0 else torch.empty((0, k), dtype=torch.int32, device=dev)
            if glob:  # every rank needs every minority row's neighbour list (int32, k per row)
                nbr, _ = comm.all_gather_rows(nbr, counts=[r[0] for r in ranks])
                q_off = 0
            tm.mark("knn")
            if n_new > 0:
                if parents is None:
                    parents = knn_ops.smote_parents(xall, stats.aff if fused else None)
                if use_virt:  # folded into every logistic pass
                    virt = lr_ops.VirtualSmote(parents, nbr.contiguous(), n_new, q_offset=q_off, sample_offset=s_off,
                                               seed=cfg.seed, counter_base=0 if glob else rank)
                    if pre_w is not None:  # the side stream's buckets: the fit's passes wait for them
                        main = torch.cuda.current_stream(dev)
                        if not _settled_on_host(bucket_done, main):
                            main.wait_event(bucket_done)
                        virt.adopt(pre_w)
                    else:  # the once-per-fit bucket sort of the samples' lambdas, timed as the SMOTE phase
                        virt.prepare(self._bws[self._cur])
                else:
                    knn_ops.smote_generate(parents, nbr, q_off, n_new, rows[n:], seed=cfg.seed,
                                           counter_base=0 if glob else rank, fp8_scale=cfg.fp8_scale,
                                           sample_offset=s_off)
            tm.mark("smote_generate")
        # ---- K4: fit ---------------------------------------------------------------------
        b = self._cur
        if dev.type == "cuda":
            for i in ((0, 1) if self._defer_now else (b,)):  # both at once (see _train_buffer)
                if self._wss[i] is None or self._wss[i].device != dev:
                    self._wss[i] = lr_ops.LRWorkspace(dev)
                    self._wss[i].prepare_flags()
        self._ws = self._wss[b]
        w0 = np.zeros(NCOLS)
        if cfg.init_std > 0:
            w0[:d] = np.random.default_rng(cfg.seed).normal(0.0, cfg.init_std, d)
        if cfg.solver == "newton":
            defer = self._defer_now and dev.type == "cuda"
            # global quantities only: under DP every rank must make the same prediction (the
            # predicted iterations carry the same all-reduces on every rank)
            n_global = int(sum(r[1] + q for r, q in zip(ranks, new_per_rank)))
            sig = (n_global, n_sched, len(ranks), cfg.C, cfg.tol, cfg.max_iter, tuple(class_w),
                   str(cfg.hess_stride), fused, cfg.storage)
            pred = self._full_pred[1] if (defer and self._full_pred and self._full_pred[0] == sig) else None
            fit = lr_ops.newton_fit(rows_cap[:n] if virt is not None else rows, C=cfg.C, tol=cfg.tol, max_iter=cfg.max_iter, class_w=class_w, d=d, w0=w0,
                                    fit_intercept=cfg.fit_intercept, comm=comm, fp8_scale=cfg.fp8_scale,
                                    check_every=cfg.check_every, workspace=self._ws, hess_stride=cfg.hess_stride,
                                    n_sched=n_sched, affine=stats.aff if fused else None, full_iters=pred,
                                    virtual=virt)
            if defer and isinstance(fit, lr_ops.PendingFit):
                fit._fdx_sig = sig
                self._pending[b] = fit
                self._bi = b ^ 1
        elif cfg.solver == "sgd":
            fit = lr_ops.sgd_fit(rows_cap[:n] if virt is not None else rows, C=cfg.C, lr=cfg.sgd_lr,
                                 momentum=cfg.sgd_momentum, epochs=cfg.sgd_epochs, batches=cfg.sgd_batches,
                                 average=cfg.sgd_average, tol=cfg.sgd_tol, subsample=cfg.sgd_subsample,
                                 extra_epochs=cfg.sgd_extra_epochs, avg_from=cfg.sgd_avg_from,
                                 epoch_batches=cfg.sgd_epoch_batches,
                                 class_w=class_w, d=d, w0=w0,
                                 fit_intercept=cfg.fit_intercept, comm=comm, fp8_scale=cfg.fp8_scale,
                                 workspace=self._ws, affine=stats.aff if fused else None, virtual=virt)
        else:
            raise ValueError(f"unknown solver {cfg.solver!r}")
        tm.mark("fit")
        self._virtual = virt
        return PipelineResult(scaler=stats, fit=fit, n_rows=n, n_train_rows=n + n_new, n_minority=n_min,
                              n_synthetic=n_new, timings=dict(tm.t))


def _settled_on_host(ev, main, budget_s: float = None) -> bool:
    """Poll a side-stream event from the host while the compute stream still has queued work:
    True once it has completed -- then the compute stream needs no wait on it (the kernels enqueued
    from here on start after it, and each dispatch acquires their inputs), which saves the ~6 us
    the command processor spends on a cross-stream barrier packet (profiles/r6_marker).  False when
    the compute stream ran dry or the budget (FDX_SORT_POLL_US, default 400) ran out: wait on it."""
    if budget_s is None:
        budget_s = float(os.environ.get("FDX_SORT_POLL_US", "400")) * 1e-6
    t0 = time.perf_counter()
    while True:
        if ev.query():
            return True
        if main.query() or time.perf_counter() - t0 > budget_s:
            return False


class _HostChunks:
    """Double-buffered host -> device streaming of raw row chunks: the H2D copy of chunk i+1 runs
    on a side stream while the compute stream works on chunk i (events order the buffer reuse)."""

    def __init__(self, X: torch.Tensor, y: torch.Tensor, dev: torch.device, chunk: int):
        self.X, self.y, self.dev, self.chunk = X, y, dev, int(chunk)
        self.n, self.d = X.shape
        self.cuda = dev.type == "cuda"
        if self.cuda:
            self.pinned = X.is_pinned() and y.is_pinned()
            if not self.pinned:
                self.px = [torch.empty((self.chunk, self.d), dtype=torch.float32, pin_memory=True) for _ in range(2)]
                self.py = [torch.empty(self.chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self.dx = [torch.empty((self.chunk, self.d), dtype=torch.float32, device=dev) for _ in range(2)]
            self.dy = [torch.empty(self.chunk, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.copy_stream = torch.cuda.Stream(dev)
            self.copied = [torch.cuda.Event() for _ in range(2)]
            self.consumed = [torch.cuda.Event() for _ in range(2)]
            self.staged = [torch.cuda.Event() for _ in range(2)]

    def _issue(self, c0: int, slot: int):
        c1 = min(self.n, c0 + self.chunk)
        m = c1 - c0
        if self.pinned:
            sx, sy = self.X[c0:c1], self.y[c0:c1]
        else:
            self.staged[slot].synchronize()  # the previous H2D out of this pinned slot is done
            self.px[slot][:m].copy_(self.X[c0:c1])
            self.py[slot][:m].copy_(self.y[c0:c1])
            sx, sy = self.px[slot][:m], self.py[slot][:m]
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(self.consumed[slot])  # compute is done with this device slot
            self.dx[slot][:m].copy_(sx, non_blocking=True)
            self.dy[slot][:m].copy_(sy, non_blocking=True)
            self.staged[slot].record(self.copy_stream)
            self.copied[slot].record(self.copy_stream)

    def __iter__(self):
        starts = list(range(0, self.n, self.chunk))
        if not self.cuda:
            for c0 in starts:
                c1 = min(self.n, c0 + self.chunk)
                yield c0, self.X[c0:c1].to(self.dev), self.y[c0:c1].to(self.dev)
            return
        cur = torch.cuda.current_stream(self.dev)
        if starts:
            self._issue(starts[0], 0)
        for i, c0 in enumerate(starts):
            slot = i & 1
            if i + 1 < len(starts):
                self._issue(starts[i + 1], slot ^ 1)
            m = min(self.n, c0 + self.chunk) - c0
            cur.wait_event(self.copied[slot])
            yield c0, self.dx[slot][:m], self.dy[slot][:m]
            self.consumed[slot].record(cur)


def _maybe_fault(rank: int):
    """FDX_FAULT=dp_rank_crash:<r> makes rank r raise mid-fit (between two collectives) -- the
    lost-rank drill of tests/test_distributed.py: every rank must exit non-zero, none may hang."""
    import os

    f = os.environ.get("FDX_FAULT", "")
    if f.startswith("dp_rank_crash:") and int(f.split(":", 1)[1]) == rank:
        raise RuntimeError(f"FDX_FAULT: simulated crash of rank {rank} mid-fit")


def global_smote_slices(ranks, quota, rank: int):
    """(rows per rank, this rank's 128-aligned sample offset) for global-scope DP SMOTE: the
    global quota (one-process formula on the summed counts) is cut at 128-aligned boundaries
    near each rank's share IN PROPORTION TO ITS RAW ROWS, so every rank's slice starts on a Philox
    pair block and fits the training buffer the rank sized before the exchange
    (n_r + ceil(n_r * ratio) + 128: the share is <= n_r * ratio and rounding moves a slice by < 128
    rows) -- also on a rank that holds no minority rows -- and post-SMOTE rows stay balanced."""
    n_g = sum(r[1] for r in ranks)
    nmin_g = sum(r[0] for r in ranks)
    total = quota(n_g, nmin_g)
    bounds = [0]
    acc = 0
    for r in ranks[:-1]:
        acc += r[1]
        cum = total * acc // max(n_g, 1)
        bounds.append(min(total, max(bounds[-1], 128 * ((cum + 64) // 128))))
    bounds.append(total)
    per = [bounds[i + 1] - bounds[i] for i in range(len(ranks))]
    return per, bounds[rank]


def evaluate(result: PipelineResult, X_test: torch.Tensor, y_test: torch.Tensor, comm=None) -> dict:
    """Exact test ROC-AUC + confusion matrix at p > 0.5 (evaluate_model.py:26-53).  A collective
    point under data parallelism: a fit still waiting for its deferred check is settled here, on
    every rank."""
    if isinstance(result.fit, lr_ops.PendingFit):
        result.fit.verify()
    a, c, bias = result.folded()
    dev = X_test.device
    at = torch.from_numpy(a).to(dev)
    ct = torch.from_numpy(c).to(dev)
    _, _, logit = pred_ops.predict_shap_raw(X_test, at, ct, bias, dphi=0, want_logit=True)
    if comm is not None and comm.world_size > 1:
        logit_all, _ = comm.all_gather_rows(logit.reshape(-1, 1))
        y_all, _ = comm.all_gather_rows(y_test.reshape(-1, 1))
        logit, y_test = logit_all.reshape(-1).contiguous(), y_all.reshape(-1).contiguous()
    auc = metric_ops.roc_auc(logit, y_test)
    cm = metric_ops.confusion_counts(logit, y_test, 0.0)
    tn, fp, fn, tp = (int(v) for v in cm)
    return {"auc": auc, "tn": tn, "fp": fp, "fn": fn, "tp": tp,
            "recall": tp / max(tp + fn, 1), "precision": tp / max(tp + fp, 1),
            "accuracy": (tp + tn) / max(tn + fp + fn + tp, 1)}


def result_summary(r: PipelineResult) -> dict:
    d = {k: v for k, v in lr_ops.fit_asdict(r.fit).items() if k != "w" and k != "history"}
    d.update(n_rows=r.n_rows, n_train_rows=r.n_train_rows, n_minority=r.n_minority, n_synthetic=r.n_synthetic)
    return d
