"""K4 logistic-regression solvers over the padded device rows.

Solvers (all minimise sklearn's objective, ops/reference.py NewtonStateRef docstring):
  * ``newton``  full-batch (HBM-sized minibatch) Newton / IRLS: one fused pass per iteration
                (gradient + loss on VALU, Hessian on MFMA), deterministic reduce, on-device
                fp64 Cholesky step with backtracking.  Converges to sklearn-lbfgs parity in
                ~6-10 passes.  Data parallel: ONE all-reduce of 1088 doubles per iteration.
  * ``sgd``     momentum minibatch SGD over contiguous row windows (gradient-only passes).

The device loop never synchronises with the host inside a chunk of iterations: a device-side
``done`` flag turns converged iterations into no-op launches.
"""
from __future__ import annotations

import time

from dataclasses import dataclass, field

import numpy as np
import torch

from . import reference as ref
from .layout import DEFAULT_FP8_SCALE, LABEL_COL, NCOLS, check_rows, storage_kind
from .native import native, ptr, stream_of

PART_STRIDE = 1088
STATE_SIZE = 256
# state offsets (logreg.hip)
S_W, S_WPREV, S_STEP, S_VEL = 0, 32, 64, 96
S_OBJPREV, S_ITER, S_BACKTRACKS, S_GMAX, S_OBJ, S_NACC, S_CONV = 128, 129, 130, 131, 132, 133, 134


@dataclass
class FitInfo:
    w: np.ndarray                 # [32] float64, padded layout (w[30] = intercept)
    n_iter: int
    n_newton_steps: int
    converged: bool
    objective: float
    grad_max: float
    history: list = field(default_factory=list)


@dataclass
class VirtualSmote:
    """SMOTE samples a Newton fit reads without their ever being stored (launchers.h SmoteView).

    The fit's rows are ``rows`` (the stored real rows) followed by ``n_new`` samples
    x = a + lam (b - a) drawn exactly as ``knn.smote_generate`` draws them (same Philox stream,
    parents, neighbour lists): a = parents[q_offset + pick // k], b = parents[nbr[pick]].  Every
    logistic pass folds them in through per-pick sums over the pick's lambdas (logreg.hip
    pick_terms), so a pass streams 2 bytes per sample instead of a 64 B stored row.  The
    interpolants enter at fp32 precision (the stored path rounds each to bf16 / e4m3): the fit is
    the stored-row fit up to that rounding, and bitwise reproducible run to run.
    ``prepare()`` buckets the lambdas by pick on the device (once per fit, smote.hip)."""
    parents: torch.Tensor     # bf16 [m, 32] (knn.smote_parents / knn_topk(parents=...))
    nbr: torch.Tensor         # int32 [mq, k] neighbour rows (indices into parents)
    n_new: int
    q_offset: int = 0
    sample_offset: int = 0    # multiple of 128 (DP ranks: one global draw sequence)
    seed: int = 42
    counter_base: int = 0
    label: float = 1.0
    lam: torch.Tensor | None = None   # int16 [n_new] lambda * 2^16 grouped by pick
    off: torch.Tensor | None = None   # int32 [mq * k] start of each pick's run in lam
    cnt: torch.Tensor | None = None   # int32 [mq * k] its length

    def check(self, rows: torch.Tensor):
        if storage_kind(rows) not in ("bf16", "fp8") or not rows.is_cuda:
            raise ValueError("virtual SMOTE rows need bf16 or fp8 device rows")
        p, nb = self.parents, self.nbr
        if p.dtype != torch.bfloat16 or p.dim() != 2 or p.shape[1] != NCOLS or p.device != rows.device:
            raise ValueError("parents must be bf16 [m, 32] on the rows' device")
        if nb.dtype != torch.int32 or nb.dim() != 2 or nb.device != rows.device or not nb.is_contiguous():
            raise ValueError("nbr must be a contiguous int32 [mq, k] tensor on the rows' device")
        mq, k = nb.shape
        if self.n_new < 0 or self.sample_offset < 0 or self.sample_offset % 128:
            raise ValueError("n_new >= 0 and sample_offset a non-negative multiple of 128")
        if self.n_new and (mq < 1 or k < 1 or self.q_offset < 0 or self.q_offset + mq > p.shape[0]):
            raise ValueError("query rows out of range of the parents")
        if mq * k > virtual_max_picks() or self.n_new > virtual_max_samples():
            raise ValueError("virtual SMOTE: picks or samples exceed the bucket sort's range")
        ref.smote_check_ranges(p.shape[0], mq, k)

    def prepare(self, ws: "BucketWorkspace | None" = None) -> "VirtualSmote":
        """Bucket the samples' lambdas by pick on the parents' device: count, scan, fill.
        ``ws``: reusable buffers (a training loop passes one per in-flight fit), so a fit
        allocates nothing here."""
        if self.off is not None or self.n_new == 0:
            return self
        m = native()
        mq, k = self.nbr.shape
        R = mq * k
        s = stream_of(self.parents)
        n = int(self.n_new)
        nt = m.smote_bucket_bins(R, n) * m.smote_bucket_blocks(n)
        w = (ws or BucketWorkspace()).get(self.parents.device, nt, n, R)
        args = (mq, k, n, int(self.sample_offset), int(self.seed) & (2**64 - 1),
                int(self.counter_base) & (2**64 - 1))
        # stage 0 writes every table entry (no fill) and zeroes the bump allocator
        m.smote_bucket(0, *args, ptr(w.table), 0, 0, 0, 0, 0, ptr(w.bump), s)        # counts [block][bin]
        torch.cumsum(w.table[:nt], 0, dtype=torch.int32, out=w.scan[:nt])          # inclusive scan
        m.smote_bucket(1, *args, ptr(w.scan), ptr(w.rec), 0, 0, 0, 0, ptr(w.bump), s)  # coarse records
        m.smote_bucket(2, *args, ptr(w.scan), ptr(w.rec), ptr(w.tmp), ptr(w.off), ptr(w.cnt), ptr(w.lam),
                       ptr(w.bump), s)
        self.lam, self.off, self.cnt, self._ws = w.lam, w.off, w.cnt, w
        return self

    def rows_f32(self) -> torch.Tensor:
        """The samples as fp32 rows (host): the interpolants the virtual passes fold in."""
        P = self.parents.cpu().float().numpy()
        out = ref.smote_generate(P, self.nbr.cpu().numpy(), self.q_offset, self.n_new, self.seed,
                                 self.counter_base, self.label, sample_offset=self.sample_offset)
        return torch.from_numpy(out)

    def materialize(self, out: torch.Tensor, fp8_scale: float = DEFAULT_FP8_SCALE) -> torch.Tensor:
        """The stored-path rows (smote_generate: the same samples rounded to ``out``'s format)."""
        from . import knn as knn_ops
        return knn_ops.smote_generate(self.parents, self.nbr, self.q_offset, self.n_new, out, seed=self.seed,
                                      counter_base=self.counter_base, label=self.label, fp8_scale=fp8_scale,
                                      sample_offset=self.sample_offset)


class BucketWorkspace:
    """Device buffers of VirtualSmote.prepare, grown on demand and reused fit to fit."""

    def __init__(self):
        self.cap, self.dev = None, None

    def get(self, dev, nt: int, n: int, R: int) -> "BucketWorkspace":
        if self.cap is None or self.dev != dev or nt > self.cap[0] or n > self.cap[1] or R > self.cap[2]:
            i32 = torch.int32
            self.table = torch.empty(nt, dtype=i32, device=dev)
            self.scan = torch.empty(nt, dtype=i32, device=dev)
            self.bump = torch.empty(1, dtype=torch.int64, device=dev)
            self.rec = torch.empty(n, dtype=i32, device=dev)
            self.tmp = torch.empty(n, dtype=i32, device=dev)
            self.lam = torch.empty(n, dtype=torch.int16, device=dev)
            self.off = torch.empty(R, dtype=i32, device=dev)
            self.cnt = torch.empty(R, dtype=i32, device=dev)
            self.cap, self.dev = (nt, n, R), dev
        return self


# the per-sample fixed-point terms of the virtual passes hold a positive-class weight <= 32
VIRTUAL_MAX_WEIGHT = 32.0


def virtual_max_picks() -> int:
    """Largest minority-rows x k that VirtualSmote's bucket sort handles (else SMOTE is stored)."""
    return int(native().smote_bucket_max_picks())


def virtual_max_samples() -> int:
    """Largest per-rank SMOTE sample count VirtualSmote's bucket sort handles."""
    return int(native().smote_bucket_max_samples())


_FIT_FIELDS = ("w", "n_iter", "n_newton_steps", "converged", "objective", "grad_max", "history")


class PendingFit:
    """A device fit whose solver state is on its way to pinned host memory.  Reading any FitInfo
    field waits for that copy only, so a caller that does not look at the result right away (a
    training loop, the benchmark) queues the next fit behind this one with no host round trip at
    the fit boundary.  Pinned slots rotate through a small pool; a slot's previous owner is
    materialised before the slot is reused.

    ``verify`` (newton_fit(full_iters=...)): a deferred convergence check.  The fit was enqueued
    with a predicted number of full-data iterations and no host wait; ``verify()`` (implicit in
    any field read) waits for the last one's flag and, if the fit had not converged, runs the
    remaining iterations then -- so the caller must keep the rows and the workspace untouched
    until the fit is verified (models/pipeline.py double-buffers both)."""

    _pool: list = []
    _pool_dev: list = []
    _owners: list = []
    _next = 0
    _POOL = 8

    def __init__(self, state_dev: torch.Tensor, sgd: bool = False, verify=None, warm_iters: int = 0):
        cls = PendingFit
        if not cls._pool:
            cls._pool = [torch.empty(state_dev.numel(), dtype=torch.float64, pin_memory=True)
                         for _ in range(cls._POOL)]
            cls._owners = [None] * cls._POOL
            # device addresses of the mapped pinned slots: the export kernel stores into them
            cls._pool_dev = [int(native().host_device_pointer(t.data_ptr())) for t in cls._pool]
        slot = cls._next % cls._POOL
        cls._next += 1
        prev = cls._owners[slot]
        if prev is not None:
            prev._materialize()
        cls._owners[slot] = self
        self._slot, self._sgd, self._info = slot, sgd, None
        self._verify, self._state_dev, self.warm_iters = verify, state_dev, int(warm_iters)
        self._export()

    def _export(self):
        cls, slot, st = PendingFit, self._slot, self._state_dev
        if cls._pool_dev[slot] and st.numel() == STATE_SIZE:
            native().logreg_export(ptr(st), cls._pool_dev[slot], stream_of(st))
        else:
            cls._pool[slot].copy_(st, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()

    def verify(self) -> "PendingFit":
        """Resolve a deferred convergence check (no-op for an already checked fit)."""
        v, self._verify = self._verify, None
        if v is not None and v():
            self._export()  # the fit continued: export its final state again
        return self

    @property
    def deferred(self) -> bool:
        return self._verify is not None

    def _materialize(self) -> FitInfo:
        if self._info is None:
            self.verify()
            self._event.synchronize()
            self._info = _info_from_state(PendingFit._pool[self._slot].numpy().copy(), self._sgd)
            if PendingFit._owners[self._slot] is self:
                PendingFit._owners[self._slot] = None
        return self._info

    def __getattr__(self, name):
        if name in _FIT_FIELDS:
            return getattr(self._materialize(), name)
        raise AttributeError(name)

    def as_fit_info(self) -> FitInfo:
        return self._materialize()

    @property
    def full_phase_iters(self) -> int:
        """Full-data iterations the fit ran (after the progressive warm-up)."""
        return int(self._materialize().n_iter) - self.warm_iters


def fit_asdict(fit) -> dict:
    """dataclasses.asdict for FitInfo or PendingFit."""
    f = fit.as_fit_info() if isinstance(fit, PendingFit) else fit
    return {k: getattr(f, k) for k in _FIT_FIELDS}


class LRWorkspace:
    """Device buffers reused across iterations / fits (no allocation inside the loop)."""

    def __init__(self, device, nblocks: int | None = None):
        m = native()
        self.device = device
        # resident grid of each row format's Hessian pass (fp8 kernels hold more blocks per CU)
        self.nblocks = nblocks or m.logreg_pass_blocks(0)
        self.nblocks_fp8 = nblocks or m.logreg_pass_blocks(1)
        self.partial = torch.empty(max(self.nblocks, self.nblocks_fp8) * PART_STRIDE, device=device,
                                   dtype=torch.float32)
        self.red = torch.zeros(PART_STRIDE, device=device, dtype=torch.float64)
        # state (f64[256]) | w32 (f32[32]) | class_w (f32[2]) | done (i32): one device blob, so a
        # reset is ONE async copy from a pinned mirror of the same layout
        self._blob = torch.zeros(_BLOB_BYTES, device=device, dtype=torch.uint8)
        self.state, self.w32, self.class_w, self.done = _blob_views(self._blob)

    def prepare_flags(self, depth: int = 2):
        """The mapped pinned convergence-flag words newton_fit polls (pinned allocations cost tens
        of microseconds to milliseconds: made once per workspace, here or on first use)."""
        if getattr(self, "_flags", None) is None or len(self._flags) < depth + 1:
            m = native()
            self._flags = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(depth + 1)]
            self._flag_dev = [int(m.host_device_pointer(f.data_ptr())) for f in self._flags]
            self._events = [torch.cuda.Event() for _ in range(depth + 1)]
            self._seq = getattr(self, "_seq", 0)

    def reset(self, w0: np.ndarray, class_w=(1.0, 1.0), aff: int = 0):
        """Initial state (w0 in the padded layout, class weights, done = 0) written by ONE kernel
        whose arguments carry the values -- no pinned staging and no H2D blit.  ``aff``: device
        address of the [64] affine map of pivot-shifted rows (w32 gets the folded weights)."""
        w = np.asarray(w0, dtype=np.float64).reshape(-1)
        native().logreg_init(ptr(self.state), ptr(self.w32), ptr(self.class_w), ptr(self.done), w.tolist(),
                             float(class_w[0]), float(class_w[1]), int(aff), stream_of(self.state))


_BLOB_BYTES = 2304


def _blob_views(blob: torch.Tensor):
    return (blob[0:2048].view(torch.float64), blob[2048:2176].view(torch.float32),
            blob[2176:2184].view(torch.float32), blob[2184:2188].view(torch.int32))


# auto Hessian sub-sampling keeps >= ~2M rows in the H estimate: at 16M rows stride 8 converges in
# the same 2 full passes as stride 3 and saves ~19 us of MFMA staging (profiles/r1_s26 trace)
HESS_SAMPLE_ROWS = 1 << 21


GRAD_SLOTS = 34  # red[0:32] gradient, red[32] loss, red[33] weight; red[34] = Hessian-sample weight


def auto_hess_stride(n_rows: int) -> int:
    return int(max(1, min(8, n_rows // HESS_SAMPLE_ROWS)))


# Warm-up phases only need a rough curvature model (they never decide convergence): their Hessian
# from >= 64k rows.  At 16M rows this is stride 16 in both warm-up phases instead of 1 and 2: the
# same 7 iterations (2 full-data), AUC within 1e-6, fit -45 us (profiles/r3_n/newton_lab.json:
# a 1/16-sample pass is 22.8 us with every tile's Hessian, 17.6 with every 8th; a 1/4 pass 56 vs 47).
WARM_HESS_SAMPLE_ROWS = 1 << 16
WARM_HESS_MAX_STRIDE = 16


def auto_warm_hess_stride(n_rows: int) -> int:
    return int(max(1, min(WARM_HESS_MAX_STRIDE, n_rows // WARM_HESS_SAMPLE_ROWS)))


def auto_hess_refresh(n_rows: int) -> int:
    """Full-data Newton iterations per fresh Hessian (lazy Hessian).  Only after a progressive
    warm-up: started near the optimum, a stale Hessian costs no iterations (profiles/r1_s12:
    2 full passes either way) but saves the MFMA work; started cold it slows convergence."""
    return 4 if progressive_schedule(n_rows) else 0


def progressive_schedule(n_rows: int) -> list:
    """Warm-up phases [(tile_subsample, newton_iters), ...] before the full-data phase.  Each
    phase keeps >= ~1M rows, so its optimum is within sampling noise of the full one and the
    full-data phase then needs ~2-3 quadratic-convergence steps."""
    if n_rows >= (8 << 20):
        return [(16, 3), (4, 2)]
    if n_rows >= (2 << 20):
        return [(4, 3)]
    return []


def _pass(m, rows, ws: LRWorkspace, hessian: int, begin: int, end: int, fp8_scale: float, s: int, done=True,
          sub: int = 1, virtual: VirtualSmote | None = None):
    """hessian: 0 = gradient/loss only; h >= 1 = Hessian from every h-th row tile (h = 1 exact).
    sub: visit a uniform 1/sub of the row tiles (progressive Newton warm-up).
    virtual: rows >= rows.shape[0] are virtual SMOTE rows (end may reach n_real + n_new)."""
    dptr = ptr(ws.done) if done else 0
    h = int(hessian)
    if virtual is not None and virtual.n_new > 0:
        v = virtual
        mq, k = v.nbr.shape
        fp8 = storage_kind(rows) != "bf16"
        nb = ws.nblocks_fp8 if fp8 else ws.nblocks
        m.logreg_pass_virtual(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub),
                              ptr(ws.partial), nb, s, ptr(v.parents), ptr(v.nbr), ptr(v.lam), ptr(v.off),
                              ptr(v.cnt), int(rows.shape[0]), int(v.q_offset), int(mq), int(k),
                              float(fp8_scale) if fp8 else 0.0)
    elif storage_kind(rows) == "bf16":
        nb = ws.nblocks
        m.logreg_pass(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub), ptr(ws.partial),
                      nb, s)
    else:
        nb = ws.nblocks_fp8
        m.logreg_pass_fp8(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub), float(fp8_scale),
                          ptr(ws.partial), nb, s)
    # gradient-only: reduce slots 0..33 and keep red[34] (weight of the rows behind the held H)
    m.logreg_reduce(ptr(ws.partial), nb, PART_STRIDE if h else GRAD_SLOTS, ptr(ws.red), dptr, s)


def logreg_pass(rows: torch.Tensor, w: torch.Tensor, class_w=(1.0, 1.0), hessian: bool = True,
                fp8_scale: float = DEFAULT_FP8_SCALE, virtual: VirtualSmote | None = None):
    """One reduced pass: (grad[32], loss, wsum, H[32,32]) as float64 numpy (test/diagnostic API).
    ``virtual``: the pass also covers virtual.n_new SMOTE rows after ``rows``."""
    check_rows(rows)
    if not rows.is_cuda:
        R = ref.rows_to_f32(rows, fp8_scale).numpy()
        return ref.logreg_pass(R, w.cpu().double().numpy(), class_w, hessian)
    m = native()
    ws = LRWorkspace(rows.device)
    ws.reset(w.cpu().double().numpy(), class_w)
    n = rows.shape[0]
    if virtual is not None:
        virtual.check(rows)
        virtual.prepare()
        n += virtual.n_new
    _pass(m, rows, ws, hessian, 0, n, fp8_scale, stream_of(rows), done=False, virtual=virtual)
    red = ws.red.cpu().numpy()
    H = red[64:].reshape(32, 32) if hessian else None
    return red[:32].copy(), float(red[32]), float(red[33]), H


def _default_w0(w0):
    if w0 is None:
        return np.zeros(NCOLS)
    w = np.asarray(w0, dtype=np.float64).copy()
    if w.shape != (NCOLS,):
        raise ValueError("w0 must be [32]")
    w[LABEL_COL] = 0.0
    return w


def _await_flag(flag: torch.Tensor, seq: int, stream: int, spin_s: float = 0.05):
    """Poll a mapped pinned flag word until the Newton update tagged ``seq`` has written it.
    After ``spin_s`` the host stops spinning and synchronises the stream instead (a stalled or
    faulted device then surfaces as the stream's error rather than a hang)."""
    t0 = time.perf_counter()
    while (int(flag[0]) >> 1) != seq:
        if time.perf_counter() - t0 > spin_s:
            native().stream_sync(stream)
            if (int(flag[0]) >> 1) != seq:
                raise RuntimeError("newton_fit: convergence flag not written after the stream drained")
            return


def newton_fit(rows: torch.Tensor, C: float = 1.0, tol: float = 1e-8, max_iter: int = 25,
               class_w=(1.0, 1.0), w0=None, d: int = 30, fit_intercept: bool = True, comm=None,
               fp8_scale: float = DEFAULT_FP8_SCALE, check_every: int = 4, workspace: LRWorkspace | None = None,
               sync: bool = True, hess_stride: int | str = "auto", progressive="auto",
               hess_refresh: int | str = "auto", n_sched: int | None = None,
               local_warmup: bool = True, affine: torch.Tensor | None = None,
               lookahead: int | None = None, full_iters: int | None = None,
               virtual: VirtualSmote | None = None) -> FitInfo:
    """Full-batch Newton on device rows.  ``comm``: parallel.comm.Communicator for DP (rows are
    this rank's shard; the reduced gradient/Hessian vector is all-reduced each iteration).
    ``hess_stride``: Hessian from every k-th row tile ("auto": keep >= ~2M rows per rank);
    gradient and objective always use all rows, so the converged solution is unchanged.
    ``hess_refresh``: in the full-data phase a fresh Hessian only every k-th iteration; the
    iterations in between stream the gradient alone (-36% bytes of MFMA-free work per pass) and
    reuse the last reduced Hessian still held in the workspace (lazy-Hessian Newton).  0 = every
    iteration.  The fixed point is unchanged: only the step's curvature model is older.
    ``affine``: [64] float64 (c | 1/sigma) when the rows are pivot-shifted instead of standardized
    (ops/scaler.scaler_fit_cast): the fit still runs in standardized space (same w, same C).
    ``full_iters``: enqueue exactly that many full-data iterations -- the count
    the previous fit of this shape needed -- with no host wait, and return a PendingFit whose
    ``verify()`` checks convergence later and finishes the fit if the prediction was short.  The
    same iterations run either way; the host-checked loop's trailing no-op iterations and its
    wait at the end of the fit disappear.  Rows and workspace must stay untouched until then.
    Under DP every rank must pass the same ``full_iters`` and verify at the same point of its
    program (the iterations, and a continuation, carry the gradient all-reduces).
    ``virtual``: the fit's rows are ``rows`` followed by virtual.n_new SMOTE rows that are
    regenerated in every pass instead of stored (VirtualSmote; bf16 device rows).  Its tensors,
    like the rows, must stay alive until a deferred fit is verified."""
    check_rows(rows)
    w0 = _default_w0(w0)
    if virtual is not None and virtual.n_new == 0:
        virtual = None
    if virtual is not None and not rows.is_cuda:  # host path: the fp32 interpolants after the rows
        rows = torch.cat([ref.rows_to_f32(rows, fp8_scale, d), virtual.rows_f32()])
        virtual = None
    if virtual is not None:
        virtual.check(rows)
        if class_w[1] > VIRTUAL_MAX_WEIGHT:
            raise ValueError(f"virtual SMOTE: positive class weight {class_w[1]} > {VIRTUAL_MAX_WEIGHT}")
        virtual.prepare()
    if not rows.is_cuda:
        if affine is not None:
            a = affine.cpu().double()
            rows = ((ref.rows_to_f32(rows, fp8_scale, d).double() - a[:32]) * a[32:]).float()
        return _newton_fit_cpu(rows, C, tol, max_iter, class_w, w0, d, fit_intercept, comm, fp8_scale)
    m = native()
    ws = workspace or LRWorkspace(rows.device)
    s = stream_of(rows)
    aff = 0
    if affine is not None:
        if affine.dtype != torch.float64 or affine.numel() != 64 or affine.device != rows.device:
            raise ValueError("affine must be a [64] float64 tensor on the rows' device")
        aff = ptr(affine)
    ws.reset(w0, class_w, aff)  # w0 is standardized-space; w32 gets it folded for shifted rows
    n = rows.shape[0] + (virtual.n_new if virtual is not None else 0)
    hs = auto_hess_stride(n) if hess_stride == "auto" else max(1, int(hess_stride))
    # The warm-up schedule sets the number of collectives, so every rank must derive the same one:
    # from ``n_sched`` (the smallest rank's row count, known to all ranks without a collective when
    # the caller exchanged sizes already) or else from one min-all-reduce.  The Hessian stride is a
    # rank-local choice (each rank rescales its own sub-sampled Hessian).
    if comm is not None and comm.world_size > 1:
        if n_sched is None:
            n_sched = int(comm.all_reduce_scalar(n, op="min"))
    else:
        n_sched = n
    sched = progressive_schedule(n_sched) if progressive == "auto" else list(progressive or [])

    # Progressive warm-up: Newton steps on uniform 1/sub tile subsets (never "converge": tol=0),
    # then full-data Newton until the exact gradient meets `tol`.  Between phases the objective
    # history is reset so backtracking only compares objectives of the same sample.
    # phase_start=1 on a phase's first iteration: the kernel forgets the previous phase's objective
    # and backtrack count (no extra fill kernels between phases).
    # Data parallel: with ``local_warmup`` every rank runs the warm-up on its own shard (no
    # collective per iteration) and the ranks then average their weights with ONE all-reduce --
    # a warm start for the global full-data phase, whose fixed point does not depend on it.
    dp = comm is not None and comm.world_size > 1
    sync_warm = dp and not local_warmup
    first = [0]
    for sub, iters in sched:
        hs_w = auto_warm_hess_stride(n_sched // sub) if hess_stride == "auto" else hs
        for j in range(iters):
            _pass(m, rows, ws, hs_w, 0, n, fp8_scale, s, sub=sub, virtual=virtual)
            if sync_warm:
                comm.all_reduce_(ws.red)
            m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), d, float(C), 0.0, 1 << 30,
                            int(fit_intercept), int(j == 0), aff, s)
        first[0] = 1
    if dp and local_warmup and sched:
        wv = ws.state[S_W:S_W + 32]
        comm.all_reduce_(wv)
        wv.div_(comm.world_size)
        ws.state[S_WPREV:S_WPREV + 32].copy_(wv)
        if aff:
            m.logreg_fold(ptr(ws.state), aff, ptr(ws.w32), s)
        else:
            ws.w32.copy_(wv)
            ws.w32[LABEL_COL] = 0.0
    warm = sum(it for _, it in sched)

    refresh = auto_hess_refresh(n_sched) if hess_refresh == "auto" else int(hess_refresh)
    full_it = [0]

    def enqueue_chunk(k: int, done_host: int = 0, seq: int = 0) -> int:
        for i in range(k):
            # a fresh Hessian on the first full-data iteration, then every refresh-th (starting
            # the full phase from the warm-up's 4M-row Hessian instead cost one more full pass:
            # 8 vs 7 iterations, profiles/r1_s25)
            fresh = refresh <= 0 or full_it[0] % refresh == 0
            full_it[0] += 1
            _pass(m, rows, ws, hs if fresh else 0, 0, n, fp8_scale, s, virtual=virtual)
            if comm is not None and comm.world_size > 1:
                # a gradient-only pass leaves the (already all-reduced) Hessian and its weight
                comm.all_reduce_(ws.red if fresh else ws.red[:GRAD_SLOTS])
            m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), d, float(C), float(tol),
                            int(max_iter + warm), int(fit_intercept), first[0], aff, s,
                            done_host if i == k - 1 else 0, seq)
            first[0] = 0
        return k

    # Convergence is checked ``lookahead`` chunks behind: chunks i+1..i+lookahead are already
    # queued when the host reads chunk i's `done` flag (async copy into pinned memory), so the GPU
    # keeps ``lookahead`` iterations of work while the host wakes up and enqueues the next one
    # (a fp8 full-data pass is ~50 us: one chunk of slack left the GPU waiting on the host).
    # Iterations after convergence are device-side no-ops (uniform early exit on `done`, a few us
    # each).  Every rank reads identical flags.
    # Under DP every queued iteration also queues its gradient all-reduce, which runs in full even
    # when the iteration is a no-op (~15 us per collective at 8 ranks, profiles/r2_s3l): one chunk
    # of slack there (a full-data pass is >= ~60 us, enough to hide the host's wake-up), two alone.
    if lookahead is None:  # profiles/r2_s5/newton_lookahead_ab.txt
        lookahead = 1 if (comm is not None and comm.world_size > 1) else 2
    depth = max(1, int(lookahead))
    # The chunk's last Newton update writes (seq << 1) | done straight into a mapped pinned word
    # (device address) and the host polls it: no D2H copy kernel and no event per check, whose
    # dependency gaps cost ~10 us each in the timeline (profiles/r2_s5).
    ws.prepare_flags(depth)
    flags, events, fdev = ws._flags, ws._events, ws._flag_dev

    def checked_loop(it: int):
        pending = []
        slot = 0
        while it < max_iter:
            ws._seq = (ws._seq + 1) & 0x3FFFFFFF
            it += enqueue_chunk(min(check_every, max_iter - it), fdev[slot], ws._seq)
            if not fdev[slot]:  # not a mapped allocation: copy the flag behind an event instead
                flags[slot].copy_(ws.done, non_blocking=True)
                events[slot].record()
            pending.append((slot, ws._seq))
            slot = (slot + 1) % (depth + 1)
            if not sync or len(pending) <= depth:
                continue
            c, seq = pending.pop(0)
            if fdev[c]:
                _await_flag(flags[c], seq, s)
            else:
                events[c].synchronize()
            if int(flags[c][0]) & 1:
                break

    if full_iters is not None and sync and fdev[0]:
        k = int(max(1, min(int(full_iters), max_iter)))
        ws._seq = (ws._seq + 1) & 0x3FFFFFFF
        seq0 = ws._seq
        enqueue_chunk(k, fdev[0], seq0)

        def verify() -> bool:
            _await_flag(flags[0], seq0, s)
            if int(flags[0][0]) & 1:
                return False  # converged (or max_iter) within the predicted iterations
            checked_loop(k)  # the prediction was short: finish the fit now
            return True
        return PendingFit(ws.state, verify=verify, warm_iters=warm)
    checked_loop(0)
    return PendingFit(ws.state, warm_iters=warm)


def _sgd_signature(n, d, C, lr, momentum, batch_rows, class_w, fit_intercept, comm):
    from ..utils.checkpoint import config_signature

    n_all = int(comm.all_reduce_scalar(float(n))) if (comm is not None and comm.world_size > 1) else n
    return config_signature(kind="sgd", n=n_all, d=d, C=C, lr=lr, momentum=momentum, batch_rows=batch_rows,
                            class_w=list(class_w), fit_intercept=fit_intercept)


def sgd_fit(rows: torch.Tensor, C: float = 1.0, lr: float = 0.5, momentum: float = 0.9, epochs: int = 5,
            batch_rows: int = 1 << 20, class_w=(1.0, 1.0), w0=None, d: int = 30, fit_intercept: bool = True,
            comm=None, fp8_scale: float = DEFAULT_FP8_SCALE, workspace: LRWorkspace | None = None,
            checkpoint=None, checkpoint_every: int = 0, affine: torch.Tensor | None = None) -> FitInfo:
    """Momentum minibatch SGD.  Each minibatch is a contiguous window of ``batch_rows`` rows of
    this rank's shard (rows are stored pre-shuffled); DP all-reduces the minibatch gradient.

    ``checkpoint`` (utils.checkpoint.CheckpointManager): every ``checkpoint_every`` minibatches
    (and at each epoch end) the solver state -- weights, velocity, objective, step counter -- and
    the data cursor (epoch, minibatch) are saved; a matching checkpoint is resumed from, giving
    the same result as an uninterrupted fit.

    ``affine``: [64] float64 (c | 1/sigma) for pivot-shifted rows (the fused scaler pass, as in
    newton_fit): the fit runs in standardized space, the update kernel maps each minibatch
    gradient and streams folded weights."""
    check_rows(rows)
    w0 = _default_w0(w0)
    n = rows.shape[0]
    if affine is not None and not rows.is_cuda:
        a = affine.cpu().double()
        rows = ((ref.rows_to_f32(rows, fp8_scale, d).double() - a[:32]) * a[32:]).float()
        affine = None
    aff = 0
    if affine is not None:
        if affine.dtype != torch.float64 or affine.numel() != 64 or affine.device != rows.device:
            raise ValueError("affine must be a [64] float64 tensor on the rows' device")
        aff = ptr(affine)
    sig = _sgd_signature(n, d, C, lr, momentum, batch_rows, class_w, fit_intercept, comm) if checkpoint else None
    got = checkpoint.latest(sig) if checkpoint is not None else None
    start = (0, 0)
    if not rows.is_cuda:
        return _sgd_fit_cpu(rows, C, lr, momentum, epochs, batch_rows, class_w, w0, d, fit_intercept, comm, fp8_scale,
                            checkpoint, checkpoint_every, sig, got)
    m = native()
    ws = workspace or LRWorkspace(rows.device)
    ws.reset(w0, class_w)
    s = stream_of(rows)
    if got is not None:
        st = got[0]["state"].to(torch.float64)
        ws.state.copy_(st.to(rows.device))
        w32 = st[S_W:S_W + 32].to(torch.float32)
        w32[LABEL_COL] = 0.0
        ws.w32.copy_(w32.to(rows.device))
        start = (int(got[1]["epoch"]), int(got[1]["batch"]))
    if aff:
        m.logreg_fold(ptr(ws.state), aff, ptr(ws.w32), s)  # the state is standardized-space
    nb = max(1, (n + batch_rows - 1) // batch_rows)
    if comm is not None and comm.world_size > 1:
        nb = int(comm.all_reduce_scalar(nb, op="max"))
    for ep in range(start[0], epochs):
        for b in range(start[1] if ep == start[0] else 0, nb):
            lo = min(b * batch_rows, n)
            hi = min(lo + batch_rows, n)
            _pass(m, rows, ws, False, lo, hi, fp8_scale, s, done=False)
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(ws.red[:GRAD_SLOTS])
            m.sgd_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), d, float(C), float(lr), float(momentum),
                         int(fit_intercept), s, aff)
            gstep = ep * nb + b + 1
            last = b + 1 == nb
            if checkpoint is not None and (last or (checkpoint_every and gstep % checkpoint_every == 0)):
                nxt = (ep + 1, 0) if last else (ep, b + 1)
                checkpoint.save(ep * nb + b + 1, {"state": ws.state},
                                {"signature": sig, "epoch": nxt[0], "batch": nxt[1], "kind": "sgd"})
    return _info_from_state(ws.state.cpu().numpy(), sgd=True)


def _info_from_state(st: np.ndarray, sgd: bool = False) -> FitInfo:
    return FitInfo(w=st[S_W:S_W + 32].copy(), n_iter=int(st[S_ITER]), n_newton_steps=int(st[S_NACC]),
                   converged=bool(st[S_CONV] > 0) if not sgd else True, objective=float(st[S_OBJ]),
                   grad_max=float(st[S_GMAX]))


# ------------------------------------------------------------------------------------------
# CPU execution path (same decisions as the device kernels, fp64)
# ------------------------------------------------------------------------------------------
def _reduced_cpu(R, w, class_w, hessian, comm):
    g, loss, wsum, H = ref.logreg_pass(R, w, class_w, hessian)
    red = ref.pack_reduced(g, loss, wsum, H)
    if comm is not None and comm.world_size > 1:
        red = comm.all_reduce(torch.from_numpy(red)).numpy()
    return red


def _newton_fit_cpu(rows, C, tol, max_iter, class_w, w0, d, fit_intercept, comm, fp8_scale) -> FitInfo:
    R = ref.rows_to_f32(rows, fp8_scale, d).double().numpy()
    st = ref.NewtonStateRef(w0)
    hist = []
    while not st.done:
        red = _reduced_cpu(R, st.w, class_w, True, comm)
        st.update(red, d, C, tol, max_iter, fit_intercept)
        hist.append(st.obj)
    return FitInfo(w=st.w.copy(), n_iter=st.iter, n_newton_steps=st.n_accepted, converged=st.converged,
                   objective=st.obj, grad_max=st.gmax, history=hist)


def _sgd_fit_cpu(rows, C, lr, momentum, epochs, batch_rows, class_w, w0, d, fit_intercept, comm, fp8_scale,
                 checkpoint=None, checkpoint_every=0, sig=None, got=None):
    R = ref.rows_to_f32(rows, fp8_scale, d).double().numpy()
    n = R.shape[0]
    w = w0.copy()
    v = np.zeros(32)
    nb = max(1, (n + batch_rows - 1) // batch_rows)
    if comm is not None and comm.world_size > 1:
        nb = int(comm.all_reduce_scalar(nb, op="max"))
    obj = np.inf
    it = 0
    start = (0, 0)
    if got is not None:
        st = got[0]["state"].numpy()
        w, v, obj, it = st[S_W:S_W + 32].copy(), st[S_VEL:S_VEL + 32].copy(), float(st[S_OBJ]), int(st[S_ITER])
        start = (int(got[1]["epoch"]), int(got[1]["batch"]))
    for ep in range(start[0], epochs):
        for b in range(start[1] if ep == start[0] else 0, nb):
            lo = min(b * batch_rows, n)
            hi = min(lo + batch_rows, n)
            red = _reduced_cpu(R[lo:hi], w, class_w, False, comm)
            S = red[33] if red[33] > 0 else 1.0
            reg = 1.0 / (C * S)
            grad = np.zeros(32)
            grad[:d] = red[:d] / S + reg * w[:d]
            if fit_intercept:
                grad[30] = red[30] / S
            v = momentum * v - lr * grad
            w = w + v
            obj = red[32] / S + 0.5 * reg * float(w[:d] @ w[:d])
            it += 1
            last = b + 1 == nb
            if checkpoint is not None and (last or (checkpoint_every and it % checkpoint_every == 0)):
                st = np.zeros(STATE_SIZE)
                st[S_W:S_W + 32], st[S_VEL:S_VEL + 32], st[S_OBJ], st[S_ITER] = w, v, obj, it
                nxt = (ep + 1, 0) if last else (ep, b + 1)
                checkpoint.save(ep * nb + b + 1, {"state": st},
                                {"signature": sig, "epoch": nxt[0], "batch": nxt[1], "kind": "sgd"})
    w[LABEL_COL] = 0.0
    return FitInfo(w=w, n_iter=it, n_newton_steps=0, converged=True, objective=obj, grad_max=float("nan"))
