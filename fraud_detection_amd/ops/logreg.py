"""K4 logistic-regression solvers over the padded device rows.

Solvers (all minimise sklearn's objective, ops/reference.py NewtonStateRef docstring):
  * ``newton``  full-batch (HBM-sized minibatch) Newton / IRLS: one fused pass per iteration
                (gradient + loss on VALU, Hessian on MFMA), deterministic reduce, on-device
                fp64 Cholesky step with backtracking.  Converges to sklearn-lbfgs parity in
                ~6-10 passes.  Data parallel: ONE all-reduce of 1088 doubles per iteration.
  * ``sgd``     curvature-normalised momentum minibatch SGD: every minibatch strides over the whole
                shard (row phase b of the pass grid's tile walk) plus 1/nb of the virtual SMOTE
                picks; epoch 0 = 4 steps over a quarter of the rows, Polyak averaging from the
                first full epoch; gradient-only passes with fixed-point sums.  One process: the whole schedule is ONE
                persistent launch (grid barrier per step); data parallel: pass -> one all-reduce of
                36 int64 -> update per step.

The device loop never synchronises with the host inside a chunk of iterations: a device-side
``done`` flag turns converged iterations into no-op launches.
"""
from __future__ import annotations

import os
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
    # persistent SGD: the fit ran on the one-block recovery launch (its grid barrier faulted because
    # not every block was resident -- another stream or process held CUs); bitwise the same fit
    recovered: bool = False


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
        mq, k = self.nbr.shape
        w = bucket_lambdas(mq, k, self.n_new, self.sample_offset, self.seed, self.counter_base, self.parents.device,
                           ws, stream_of(self.parents))
        return self.adopt(w)

    def adopt(self, w: "BucketWorkspace") -> "VirtualSmote":
        """Take the buckets of a bucket_lambdas call made for this draw (same picks, samples, seed)
        -- e.g. one enqueued on a side stream while the neighbour search ran."""
        mq, k = self.nbr.shape
        if getattr(w, "key", None) != (mq * k, int(self.n_new), int(self.sample_offset), int(self.seed),
                                       int(self.counter_base)):
            raise ValueError("bucket workspace was filled for another SMOTE draw")
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


def bucket_lambdas(mq: int, k: int, n_new: int, sample_offset: int, seed: int, counter_base: int, dev,
                   ws: "BucketWorkspace | None" = None, stream: int | None = None,
                   stages: tuple = (0, 1, 2)) -> "BucketWorkspace":
    """The samples' lambdas bucketed by pick (VirtualSmote.prepare).  Needs only the draw -- pick
    count mq x k, sample count, seed, counters -- not the neighbour table, so a pipeline enqueues
    it on a side stream while the k-NN runs (models/pipeline.py) and adopts the result."""
    m = native()
    R, n = int(mq) * int(k), int(n_new)
    s = int(stream) if stream is not None else int(torch.cuda.current_stream(dev).cuda_stream)
    w = ws or BucketWorkspace()
    if w.reserve(dev, mq, k, n_new):
        # fresh buffers come from the CURRENT stream's pool: another stream may only write them
        # after everything this stream has enqueued so far (the caller orders that: pipeline.py)
        if stream is not None and int(stream) != int(torch.cuda.current_stream(dev).cuda_stream):
            raise RuntimeError("bucket_lambdas: reserve the workspace before enqueueing on another stream")
    args = (int(mq), int(k), n, int(sample_offset), int(seed) & (2**64 - 1), int(counter_base) & (2**64 - 1))
    # stage 0 writes every table entry (no fill) and zeroes the bump allocator; stage 1 scans
    # each block's row in LDS (no global scan: a block's record run starts at a closed-form
    # offset) and scatters the coarse records; stage 2 assembles each pick's lambda run
    # ``stages``: a caller may enqueue the stages at different points of another stream's timeline
    if 0 in stages:
        m.smote_bucket(0, *args, ptr(w.table), 0, 0, 0, 0, 0, ptr(w.bump), s)        # counts [block][bin]
    if 1 in stages:
        m.smote_bucket(1, *args, ptr(w.table), ptr(w.rec), 0, 0, 0, 0, ptr(w.bump), s)  # prefix + records
    if 2 in stages:
        m.smote_bucket(2, *args, ptr(w.table), ptr(w.rec), ptr(w.tmp), ptr(w.off), ptr(w.cnt), ptr(w.lam),
                       ptr(w.bump), s)
        w.key = (R, n, int(sample_offset), int(seed), int(counter_base))
    return w


class BucketWorkspace:
    """Device buffers of VirtualSmote.prepare, grown on demand and reused fit to fit."""

    def __init__(self):
        self.cap, self.dev = None, None

    def reserve(self, dev, mq: int, k: int, n_new: int) -> bool:
        """Size the buffers for a draw of mq x k picks and n_new samples (on the current stream);
        True when they were (re)allocated -- a side stream must then wait for the current stream's
        present position, not an earlier one, before writing them."""
        m = native()
        R, n = int(mq) * int(k), int(n_new)
        nt = m.smote_bucket_bins(R, n) * m.smote_bucket_blocks(n)
        before = self.cap, self.dev
        self.get(dev, nt, n, R)
        return (self.cap, self.dev) != before

    def get(self, dev, nt: int, n: int, R: int) -> "BucketWorkspace":
        if self.cap is None or self.dev != dev or nt > self.cap[0] or n > self.cap[1] or R > self.cap[2]:
            i32 = torch.int32
            self.table = torch.empty(nt, dtype=i32, device=dev)
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

    def __init__(self, state_dev: torch.Tensor, sgd: bool = False, verify=None, warm_iters: int = 0,
                 keep: tuple = (), collective: bool = False, slot: int | None = None, exported: int = 0):
        cls = PendingFit
        if slot is None:
            slot = cls.reserve()
        cls._owners[slot] = self
        self._slot, self._sgd, self._info = slot, sgd, None
        self._stream = torch.cuda.current_stream(state_dev.device) if state_dev.is_cuda else None
        self._verify, self._state_dev, self.warm_iters = verify, state_dev, int(warm_iters)
        # the tensors a deferred continuation reads by device address (rows, affine map, virtual
        # SMOTE buffers): referenced here until verified, so the caching allocator cannot hand
        # their blocks to another fit meanwhile
        self._keep = tuple(keep) if verify is not None else ()
        # data parallel: the continuation holds gradient all-reduces, so only an explicit verify()
        # that every rank makes (DevicePipeline.settle, evaluate) may run it -- a field read on
        # one rank alone would enter the collectives alone and hang the job
        self._collective = bool(collective)
        self._export(exported)

    @classmethod
    def reserve(cls) -> int:
        """The next pinned slot, its previous owner materialised.  A fit that exports its own final
        state (the persistent SGD launch's recovery kernel stores it into ``slot_address``) reserves
        the slot before enqueueing, then wraps it with ``PendingFit(..., slot=, exported=stamp)``."""
        if not cls._pool:
            # word STATE_SIZE: the stamp (int64) an exporting launch stores after the state
            cls._pool = [torch.zeros(STATE_SIZE + 1, dtype=torch.float64, pin_memory=True) for _ in range(cls._POOL)]
            cls._stamps = [t.view(torch.int64).numpy()[STATE_SIZE:] for t in cls._pool]
            cls._owners = [None] * cls._POOL
            # device addresses of the mapped pinned slots: the export kernel stores into them
            cls._pool_dev = [int(native().host_device_pointer(t.data_ptr())) for t in cls._pool]
        slot = cls._next % cls._POOL
        cls._next += 1
        prev = cls._owners[slot]
        if prev is not None:
            # a program-order point every rank reaches at the same fit (slots rotate identically
            # on every rank): verifying a DP fit here is collective-safe
            prev._materialize(collective_ok=True)
        cls._owners[slot] = None
        return slot

    @classmethod
    def slot_address(cls, slot: int) -> int:
        return cls._pool_dev[slot]

    @classmethod
    def next_stamp(cls) -> int:
        """A fresh stamp (> every earlier one) for a launch that exports into a slot."""
        cls._seq = getattr(cls, "_seq", 0) + 1
        return cls._seq

    def _export(self, stamp: int = 0):
        """``stamp`` > 0: the fit's last kernel exports the state and then this stamp into the slot
        (sgd_persist(export_seq=)); the host polls the stamp, so no event is recorded behind it --
        each marker cost the command processor ~7 us at the fit boundary (profiles/r6_marker)."""
        cls, slot, st = PendingFit, self._slot, self._state_dev
        self._stamp, self._event = int(stamp), None
        if stamp:
            return
        if cls._pool_dev[slot] and st.numel() == STATE_SIZE:  # the export kernel stamps the slot too
            self._stamp = cls.next_stamp()
            native().logreg_export(ptr(st), cls._pool_dev[slot], stream_of(st), self._stamp)
        else:
            cls._pool[slot][:STATE_SIZE].copy_(st, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()

    SPIN_S = 0.05  # stamp polling, then a wait on the fit's stream (a faulted stream raises there)

    def _wait_stamp(self):
        view, t0 = PendingFit._stamps[self._slot], time.perf_counter()
        while int(view[0]) != self._stamp:
            if time.perf_counter() - t0 > self.SPIN_S:
                self._stream.synchronize()
                if int(view[0]) != self._stamp:
                    raise RuntimeError("PendingFit: state not exported after its stream drained")
                return

    def verify(self) -> "PendingFit":
        """Resolve a deferred convergence check (no-op for an already checked fit).  Under data
        parallelism every rank must call it at the same point of its program."""
        v, self._verify = self._verify, None
        if v is not None and v():
            self._export()  # the fit continued: export its final state again
        self._keep = ()
        return self

    @property
    def deferred(self) -> bool:
        return self._verify is not None

    def _materialize(self, collective_ok: bool = False) -> FitInfo:
        if self._info is None:
            if self._verify is not None and self._collective and not collective_ok:
                raise RuntimeError("data-parallel fit with a pending convergence check: settle it on every "
                                   "rank first (DevicePipeline.settle() or evaluate(...)), then read it")
            self.verify()
            if self._event is not None:
                self._event.synchronize()
            else:
                self._wait_stamp()
            self._info = _info_from_state(PendingFit._pool[self._slot][:STATE_SIZE].numpy().copy(), self._sgd)
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
        # the SGD pass grid (2 blocks per CU, 512 on MI355X): its waves define the minibatch partition
        self.sgd_blocks = nblocks or m.sgd_full_blocks()
        self.partial = torch.empty(max(self.nblocks, self.nblocks_fp8) * PART_STRIDE, device=device,
                                   dtype=torch.float32)
        self.red = torch.zeros(PART_STRIDE, device=device, dtype=torch.float64)
        # state (f64[256]) | w32 (f32[32]) | class_w (f32[2]) | done (i32): one device blob, so a
        # reset is ONE async copy from a pinned mirror of the same layout
        self._blob = torch.zeros(_BLOB_BYTES, device=device, dtype=torch.uint8)
        self.state, self.w32, self.class_w, self.done = _blob_views(self._blob)
        # fused SGD steps: 32 replicas x 36 int64 fixed-point accumulators + the arrival ticket;
        # zero between steps (every step's last block swaps them back to zero)
        self.sgd_acc = torch.zeros(SGD_ACC_WORDS + 8, device=device, dtype=torch.int64)
        # persistent SGD launch: barrier shards + 3 accumulator sets (zeroed by the launcher); the
        # data-parallel lean step's folded fixed-point sums (the all-reduced vector)
        self.sgd_persist = torch.zeros(int(m.SGD_PERSIST_WORDS), device=device, dtype=torch.int64)
        self.sgd_sums = torch.zeros(SGD_SLOTS, device=device, dtype=torch.int64)
        # fused Newton iterations: group tickets (zero, left zero) + fp64 group sums
        self.newton_fuse = torch.zeros(int(m.NEWTON_FUSE_WORDS), device=device, dtype=torch.int64)

    def prepare_flags(self, depth: int = 2):
        """The mapped pinned convergence-flag words newton_fit polls (pinned allocations cost tens
        of microseconds to milliseconds: made once per workspace, here or on first use)."""
        if getattr(self, "_flags", None) is None or len(self._flags) < depth + 1:
            m = native()
            self._flags = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(depth + 1)]
            self._flag_dev = [int(m.host_device_pointer(f.data_ptr())) for f in self._flags]
            self._events = [torch.cuda.Event() for _ in range(depth + 1)]
            self._seq = getattr(self, "_seq", 0)

    def reset(self, w0: np.ndarray, class_w=(1.0, 1.0), aff: int = 0, w0_dev: int = 0, persist: bool = False):
        """Initial state (w0 in the padded layout, class weights, done = 0) written by ONE kernel
        whose arguments carry the values -- no pinned staging and no H2D blit.  ``aff``: device
        address of the [64] affine map of pivot-shifted rows (w32 gets the folded weights).
        ``w0_dev``: device address of 32 fp64 standardized-space weights that replace ``w0`` (another
        fit's state: a warm start with no host round trip).  ``persist``: the same kernel also preps
        the persistent SGD workspace (zeroed barrier/accumulators, initial-state backup), so the
        persistent launch that follows needs no prep launch (sgd_persist(prepped=1))."""
        w = np.asarray(w0, dtype=np.float64).reshape(-1)
        native().logreg_init(ptr(self.state), ptr(self.w32), ptr(self.class_w), ptr(self.done), w.tolist(),
                             float(class_w[0]), float(class_w[1]), int(aff), stream_of(self.state), int(w0_dev),
                             ptr(self.sgd_persist) if persist else 0)


_BLOB_BYTES = 2304
SGD_ACC_WORDS = 32 * 36  # logreg.hip kSgdAccWords


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
        # (16, 3), (8, 1), (4, 1): one 1/4 iteration traded for a 1/8 one, same 2 full-data
        # iterations and AUC at the bench shape, 0.711 -> 0.690 ms per host-checked fit
        # (tools/sched_lab.py, profiles/r4_g/sched_lab.json)
        return [(16, 3), (8, 1), (4, 1)]
    if n_rows >= (2 << 20):
        return [(4, 3)]
    return []


def _pass(m, rows, ws: LRWorkspace, hessian: int, begin: int, end: int, fp8_scale: float, s: int, done=True,
          sub: int = 1, virtual: VirtualSmote | None = None, hole: tuple = (0, 0), update: tuple | None = None):
    """hessian: 0 = gradient/loss only; h >= 1 = Hessian from every h-th row tile (h = 1 exact).
    sub: visit a uniform 1/sub of the row tiles (progressive Newton warm-up).
    virtual: rows >= rows.shape[0] are virtual SMOTE rows (end may reach n_real + n_new).
    hole: (at, len) stored rows [at, at + len) the pass steps over (a CV fold's validation block);
    ``end`` counts logical rows (the hole excluded).
    update: (aff, C, tol, d, max_iter, fit_intercept, phase_start, done_host, seq) -- the Newton
    update after the pass.  Fused (FDX_NEWTON_FUSE=1): the pass's last blocks reduce the
    partials and apply it in the same launch (logreg.hip newton_fused_tail); else logreg_reduce +
    newton_update launches."""
    dptr = ptr(ws.done) if done else 0
    nf = None
    if update is not None and _newton_fuse() and done:
        aff, C, tol, d, max_iter, fi, phase_start, done_host, seq = update
        nf = (ptr(ws.red), ptr(ws.newton_fuse), ptr(ws.state), ptr(ws.w32), ptr(ws.done), int(aff), int(done_host),
              float(C), float(tol), int(d), int(max_iter), int(fi), int(phase_start), int(seq))
    h = int(hessian)
    ha, hl = int(hole[0]), int(hole[1])
    end += hl  # physical end
    if virtual is not None and virtual.n_new > 0:
        v = virtual
        mq, k = v.nbr.shape
        fp8 = storage_kind(rows) != "bf16"
        nb = ws.nblocks_fp8 if fp8 else ws.nblocks
        m.logreg_pass_virtual(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub),
                              ptr(ws.partial), nb, s, ptr(v.parents), ptr(v.nbr), ptr(v.lam), ptr(v.off),
                              ptr(v.cnt), int(rows.shape[0]), int(v.q_offset), int(mq), int(k),
                              float(fp8_scale) if fp8 else 0.0, 0, False, ha, hl, nf)
    elif storage_kind(rows) == "bf16":
        nb = ws.nblocks
        m.logreg_pass(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub), ptr(ws.partial),
                      nb, s, 0, False, ha, hl, nf)
    else:
        nb = ws.nblocks_fp8
        m.logreg_pass_fp8(ptr(rows), begin, end, ptr(ws.w32), ptr(ws.class_w), dptr, h, int(sub), float(fp8_scale),
                          ptr(ws.partial), nb, s, 0, False, ha, hl, nf)
    if nf is not None:
        return
    # gradient-only: reduce slots 0..33 and keep red[34] (weight of the rows behind the held H)
    m.logreg_reduce(ptr(ws.partial), nb, PART_STRIDE if h else GRAD_SLOTS, ptr(ws.red), dptr, s)
    if update is not None:
        aff, C, tol, d, max_iter, fi, phase_start, done_host, seq = update
        m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), int(d), float(C), float(tol),
                        int(max_iter), int(fi), int(phase_start), int(aff), s, int(done_host), int(seq))


def _newton_fuse() -> bool:
    """FDX_NEWTON_FUSE=1: the Newton update in the pass launch (newton_fused_tail); else the pass, logreg_reduce and newton_update launches."""
    return os.environ.get("FDX_NEWTON_FUSE", "0") == "1"


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


def _apply_hole(rows: torch.Tensor, hole):
    """(rows, (at, len)) for a device fit that steps over the block; a host fit gets the rows
    without it (one concatenation: the CPU path is the oracle, not the fast path)."""
    if not hole or int(hole[1]) == 0:
        return rows, (0, 0)
    at, ln = int(hole[0]), int(hole[1])
    if at < 0 or ln < 0 or at + ln > rows.shape[0]:
        raise ValueError(f"hole {hole} outside the {rows.shape[0]} stored rows")
    if rows.is_cuda:
        return rows, (at, ln)
    return torch.cat([rows[:at], rows[at + ln:]]), (0, 0)


def _default_w0(w0):
    if w0 is None:
        return np.zeros(NCOLS)
    w = np.asarray(w0, dtype=np.float64).copy()
    if w.shape != (NCOLS,):
        raise ValueError("w0 must be [32]")
    w[LABEL_COL] = 0.0
    return w


FLAG_WAITS: list = []  # host seconds spent in each _await_flag (diagnostics: tools/dp_scope_probe.py)


def _await_flag(flag: torch.Tensor, seq: int, stream: int, spin_s: float = 0.05):
    """Poll a mapped pinned flag word until the Newton update tagged ``seq`` has written it.
    After ``spin_s`` the host stops spinning and synchronises the stream instead (a stalled or
    faulted device then surfaces as the stream's error rather than a hang)."""
    t0 = time.perf_counter()
    try:
        _spin_flag(flag, seq, stream, spin_s, t0)
    finally:
        if len(FLAG_WAITS) < 4096:
            FLAG_WAITS.append(time.perf_counter() - t0)


def _spin_flag(flag: torch.Tensor, seq: int, stream: int, spin_s: float, t0: float):
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
               virtual: VirtualSmote | None = None, hole: tuple | None = None,
               w0_from: torch.Tensor | None = None) -> FitInfo:
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
    regenerated in every pass instead of stored (VirtualSmote; bf16 or fp8 device rows).  Its tensors,
    like the rows, must stay alive until a deferred fit is verified.
    ``hole``: (at, len) -- the fit's rows are ``rows`` without the block [at, at + len) (a
    cross-validation fold on the fold-sorted training table: no per-fold copy).
    ``w0_from``: another fit's device state (fp64 [>= 32], standardized-space weights first) whose
    weights start this fit -- read by the init kernel in stream order, so it may be a fit that is
    still enqueued (a CV fold warm-started from the previous one; device fits only)."""
    check_rows(rows)
    w0 = _default_w0(w0)
    rows, hole = _apply_hole(rows, hole)
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
    if w0_from is not None and (w0_from.dtype != torch.float64 or w0_from.numel() < NCOLS
                                or w0_from.device != rows.device):
        raise ValueError("w0_from must be a float64 device state of >= 32 entries on the rows' device")
    # w0 is standardized-space; w32 gets it folded for shifted rows
    ws.reset(w0, class_w, aff, ptr(w0_from) if w0_from is not None else 0)
    n = rows.shape[0] - hole[1] + (virtual.n_new if virtual is not None else 0)
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
            upd = (aff, C, 0.0, d, 1 << 30, int(fit_intercept), int(j == 0), 0, 0)
            if sync_warm:
                _pass(m, rows, ws, hs_w, 0, n, fp8_scale, s, sub=sub, virtual=virtual, hole=hole)
                comm.all_reduce_(ws.red)
                m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), d, float(C), 0.0, 1 << 30,
                                int(fit_intercept), int(j == 0), aff, s)
            else:  # the update in the pass's launch (fused) or right behind it
                _pass(m, rows, ws, hs_w, 0, n, fp8_scale, s, sub=sub, virtual=virtual, hole=hole, update=upd)
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
            dh = done_host if i == k - 1 else 0
            if comm is not None and comm.world_size > 1:
                _pass(m, rows, ws, hs if fresh else 0, 0, n, fp8_scale, s, virtual=virtual, hole=hole)
                # a gradient-only pass leaves the (already all-reduced) Hessian and its weight
                comm.all_reduce_(ws.red if fresh else ws.red[:GRAD_SLOTS])
                m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), d, float(C), float(tol),
                                int(max_iter + warm), int(fit_intercept), first[0], aff, s, dh, seq)
            else:
                _pass(m, rows, ws, hs if fresh else 0, 0, n, fp8_scale, s, virtual=virtual, hole=hole,
                      update=(aff, C, tol, d, max_iter + warm, int(fit_intercept), first[0], dh, seq))
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
        return PendingFit(ws.state, verify=verify, warm_iters=warm, keep=(rows, affine, virtual, ws),
                          collective=comm is not None and comm.world_size > 1)
    checked_loop(0)
    return PendingFit(ws.state, warm_iters=warm)


def _sgd_signature(n, d, C, lr, momentum, nb, epochs, average, tol, class_w, fit_intercept, comm, serpentine=False,
                   subs=None, nbs=None):
    from ..utils.checkpoint import config_signature

    n_all = int(comm.all_reduce_scalar(float(n))) if (comm is not None and comm.world_size > 1) else n
    extra = {"serpentine": True} if serpentine else {}
    if subs is not None and any(x != 1 for x in subs):
        extra["subsample"] = [int(x) for x in subs]
    if nbs is not None and any(x != nb for x in nbs):
        extra["epoch_batches"] = [int(x) for x in nbs]
    return config_signature(kind="sgd2", n=n_all, d=d, C=C, lr=list(lr), momentum=momentum, batches=nb,
                            epochs=epochs, average=bool(average), tol=tol, class_w=list(class_w),
                            fit_intercept=fit_intercept, **extra)


# Config 3's solver defaults (BASELINE.json: "SMOTE k-NN + logistic SGD").  Chosen on the bench
# distribution in fp64 simulation (8M raw rows -> 16M post-SMOTE rows, 3 data seeds plus a 4M-row
# shard): the Polyak-averaged last epoch lands within 2-3e-5 relative of the Newton optimum and the
# epoch gradient at 3-5e-4; a constant step instead of the curvature-normalised one needed > 48
# steps for 1e-3 (the curvature falls ~5x between w = 0 and the optimum).
SGD_BATCHES = 8
SGD_EPOCHS = 3
# per-epoch step scalar c (lr_t = c / mean s p (1 - p) of the minibatch); the 4th entry is the
# extra epoch's (SGD_EXTRA_EPOCHS)
SGD_LR = (0.6, 0.8, 0.8, 0.6)
# Per-epoch row sub-sample: epoch 0 visits 1/4 of the rows -- a growing-batch schedule: the first
# epoch only has to bring w near the optimum, so it needs no full pass (Smith et al., "Don't decay
# the learning rate, increase the batch size").  A sub-sampled epoch never decides convergence.
SGD_SUB = (4, 1, 1)
# Per-epoch minibatch counts: epoch 0 takes 4 steps of 1/16 of the rows (every 4th phase of a
# 16-minibatch grid), the full epochs 6 steps of 1/6.  fp64 simulation on the bench distribution
# (tools/sgd_schedule_lab.py "d66", 16M post-SMOTE rows, seven data seeds): every seed converges in
# the nominal 3 epochs (epoch gradient 3.8-8.4e-4, objective <= 4e-4 above Newton's); on the GPU at
# the bench shape bf16 and fp8 both end at 5.6e-4, the same as with 8-step full epochs, in 16 steps
# instead of 20: 1.050 vs 1.111 ms per bf16 fit, 0.997 vs 1.066 fp8 (profiles/r5_zz,
# tools/sgd_schedule_ab.py).  8 steps at c = 0.4 in epoch 0 ("sub4_avg2") ended at 4.5-9.8e-4 with 8
# more grid barriers; 4 steps over an eighth of the rows ran the extra epoch on some seeds.
# The extra epoch (4th entry) takes 3 minibatches at c = 0.6: the CV job's folds that miss tol after
# the nominal 16 steps end at the same epoch gradient (1.4-1.7e-3 vs 1.1-1.8e-3 after a 6-step extra
# epoch at c = 0.8 -- the statistic's noise level, tol is not reached either way) and the same AUCs
# in 19 steps instead of 22 (profiles/r6_sgd/extra_epoch_candidates_gpu.log: 2, 3 or 4 minibatches
# at c = 0.8, 0.4 or 0.3 ended at 1.8-8.6e-3).  Nominal fits never run it.
SGD_EPOCH_BATCHES = (4, 6, 6, 3)
# Epochs past SGD_EPOCHS that run only while the fit has not converged (the device `done` flag makes
# them no-ops otherwise; the persistent launch leaves its loop).  Each is averaged like the last
# nominal epoch, starting from that epoch's averaged iterate.  fp8 rows carry ~6% quantisation
# noise per feature, which slows the last digits of the epoch gradient (round 4: 1.4e-3 after 3
# epochs, profiles/r4_c); bf16 rows converge in the nominal 3 and never run it.
SGD_EXTRA_EPOCHS = 1
# First Polyak-averaged epoch (every later epoch is averaged too, each returning its own average
# started from the previous one): epoch 1, the first full epoch after the sub-sampled one.  fp64
# simulation (tools/sgd_schedule_lab.py): at 16M post-SMOTE rows the epoch gradient ends at 4.8e-4
# and the objective 9e-5 above Newton's; at 8M rows 9.0e-4 / 5.3e-4 -- where averaging only the
# last epoch ends at 1.5e-3 / 1.2e-3, short of tol even after an extra epoch (2.0e-3).
SGD_AVG_FROM = 1
SGD_MOMENTUM = 0.55
SGD_TOL = 1e-3                # on the epoch gradient max-norm (sklearn SGDClassifier's default tol)
SGD_SLOTS = 36


SGD_MAX_EPOCHS = 8  # launchers.h kSgdMaxEpochs (per-epoch step scalars of the persistent launch)


def _effective_subs(subs, n_stored: int, n_picks: int, nbs, blocks: int) -> list:
    """Sub-sample factors that keep every minibatch of an epoch's finer grid (nb_e x s) well populated
    (>= one grid's worth of row tiles and >= 2 pick tiles each); else that epoch visits every row."""
    groups = n_stored // (ref.ROW_TILE * ref.WAVES_PER_BLOCK * max(1, blocks))
    ptiles = -(-n_picks // ref.PICK_TILE)
    out = []
    for x, nb in zip(subs, nbs):
        ok = x > 1 and groups >= nb * x and (n_picks == 0 or ptiles >= 2 * nb * x)
        out.append(int(x) if ok else 1)
    return out


def _sgd_phase(pos: int, ep: int, nb: int, serpentine: bool) -> int:
    """Minibatch visited at position ``pos`` of epoch ``ep`` (logreg.hip sgd_persist_kernel phase_of)."""
    return nb - 1 - pos if (serpentine and ep % 2 == 1) else pos


def _persist_default() -> bool:
    import os
    return os.environ.get("FDX_SGD_PERSIST", "1") != "0"


def _epoch_lr(lr, ep: int) -> float:
    if np.ndim(lr) == 0:
        return float(lr)
    lr = list(lr)
    return float(lr[min(ep, len(lr) - 1)])


def sgd_fit(rows: torch.Tensor, C: float = 1.0, lr=SGD_LR, momentum: float = SGD_MOMENTUM,
            epochs: int = SGD_EPOCHS, batches: int = SGD_BATCHES, average: bool = True, tol: float = SGD_TOL,
            class_w=(1.0, 1.0), w0=None, d: int = 30, fit_intercept: bool = True, comm=None,
            fp8_scale: float = DEFAULT_FP8_SCALE, workspace: LRWorkspace | None = None, checkpoint=None,
            checkpoint_every: int = 0, affine: torch.Tensor | None = None, virtual: VirtualSmote | None = None,
            batch_rows: int | None = None, max_steps: int | None = None, hole: tuple | None = None,
            persistent: bool | None = None, serpentine: bool = False, subsample=SGD_SUB,
            extra_epochs: int = 0, avg_from: int | None = None, epoch_batches=None,
            _stamps: torch.Tensor | None = None, _fault_test: bool = False, _spin_limit: int = 0):
    """Minibatch SGD (BASELINE config 3) on sklearn's objective.

    Minibatches: an epoch is ``batches`` disjoint minibatches; minibatch b is the pass's row phase b
    -- the stored 64-row tiles t with t mod batches == b (every minibatch samples the whole shard,
    whatever the row order: a time-sorted or fold-sorted table included) plus the virtual-SMOTE pick tiles t mod batches == b
    (1/batches of the SMOTE samples, generated in the pass, never stored).  Each minibatch
    therefore holds both classes in the post-SMOTE proportion.  ``batch_rows`` (legacy) sets
    ``batches`` = ceil(rows / batch_rows).

    Step: heavy-ball momentum on the minibatch gradient, lr_t = lr[epoch] / dbar_t with dbar_t the
    minibatch's mean Gauss-Newton curvature s p (1 - p) (same pass, slot 35), Polyak-Ruppert
    averaging over the last epoch (``average``), and a device-side convergence state settled at
    every epoch end: the epoch gradient max-norm (FitInfo.grad_max) against ``tol``, the epoch's
    mean objective (FitInfo.objective), ``converged``; a converged fit turns its remaining passes
    into no-ops.  The whole fit is enqueued with no host synchronisation and returns a PendingFit.

    Data parallel: the minibatch sums (36 values) are all-reduced before every update (C4).
    ``checkpoint``: every ``checkpoint_every`` steps and at each epoch end the device state
    (weights, velocity, average, epoch sums) and the cursor (epoch, minibatch) are saved; a
    matching checkpoint is resumed from.  ``affine``: pivot-shifted rows (fused scaler pass), as in
    newton_fit.  ``virtual``: the SMOTE samples after ``rows`` (VirtualSmote).  ``max_steps``: stop
    after that many steps of the schedule (a simulated interruption for the resume tests).
    ``hole``: (at, len) stored rows the fit steps over (newton_fit).
    ``persistent``: one process, the whole schedule in ONE launch (logreg.hip sgd_persist_kernel:
    a grid barrier per step instead of a launch per step; bitwise the same fit).  Default on
    unless FDX_SGD_PERSIST=0.  It is a cooperative launch: a grid the occupancy query refuses runs
    on the per-step launches instead; a grid barrier that times out at run time (CUs held by another
    stream or process) hands the fit to the one-block recovery launch queued behind it, which
    re-runs it from the initial state -- bitwise the same fit, FitInfo.recovered set.
    ``_fault_test`` forces that path (test knob).  ``serpentine``: odd epochs visit the minibatches in reverse order
    (persistent launch only), so an epoch's first minibatches are the previous epoch's last ones
    -- still resident in the 256 MB Infinity Cache.  ``subsample``: per-epoch row sub-sample factors
    (SGD_SUB; an epoch with factor s visits 1/s of the rows in its nb minibatches).
    ``extra_epochs``: epochs after ``epochs`` that run only if the fit has not converged yet
    (the pipelines pass SGD_EXTRA_EPOCHS); with ``average`` each of them returns its own Polyak average, like the
    last nominal epoch.  ``avg_from``: first averaged epoch (None: the last nominal one; the
    pipelines pass SGD_AVG_FROM).  ``epoch_batches``: per-epoch minibatch counts (default
    ``batches`` for every epoch; the pass grid and its partition are sized for ``batches``)."""
    check_rows(rows)
    w0 = _default_w0(w0)
    rows, hole = _apply_hole(rows, hole)
    if virtual is not None and virtual.n_new == 0:
        virtual = None
    n_stored = rows.shape[0] - hole[1]
    n = n_stored + (virtual.n_new if virtual is not None else 0)
    if batch_rows:
        batches = max(1, -(-n // int(batch_rows)))
    nb = max(1, int(batches))
    if comm is not None and comm.world_size > 1:
        nb = int(comm.all_reduce_scalar(nb, op="max"))
    nominal = max(int(epochs), 1)
    epochs = nominal + max(0, int(extra_epochs))  # the schedule's length from here on
    # averaged epochs: avg_from (default the last nominal one) .. the extras
    avg_from = min(nominal - 1, max(0, int(avg_from))) if (average and avg_from is not None) else \
        (nominal - 1 if average else epochs)
    lrs = [_epoch_lr(lr, e) for e in range(epochs)]
    subs = [int(_epoch_lr(subsample, e)) if subsample is not None else 1 for e in range(epochs)]
    if any(x < 1 for x in subs):
        raise ValueError("sub-sample factors must be >= 1")
    nbs = [nb if epoch_batches is None else max(1, int(_epoch_lr(epoch_batches, e))) for e in range(epochs)]
    estart = np.concatenate([[0], np.cumsum(nbs)]).astype(int).tolist()  # first step of every epoch
    # a sub-sampled epoch only where every minibatch of its finer grid still holds row tiles of the
    # whole shard and SMOTE picks (small shards: every epoch full); one decision for all DP ranks
    n_picks = int(virtual.nbr.numel()) if virtual is not None else 0
    subs = _effective_subs(subs, n_stored, n_picks, nbs, ref.sgd_grid_blocks(n_stored, nb, ref.SGD_FULL_BLOCKS))
    if comm is not None and comm.world_size > 1:
        subs = [int(comm.all_reduce_scalar(float(x), op="min")) for x in subs]
    if affine is not None and not rows.is_cuda:
        a = affine.cpu().double()
        rows = ((ref.rows_to_f32(rows, fp8_scale, d).double() - a[:32]) * a[32:]).float()
        if virtual is not None:  # the samples interpolate shifted parents: map them the same way
            vr = ((virtual.rows_f32().double() - a[:32]) * a[32:]).float()
            vr[:, LABEL_COL] = virtual.label
            return _sgd_fit_cpu(rows, C, lrs, momentum, epochs, nb, avg_from, tol, class_w, w0, d, fit_intercept,
                                comm, fp8_scale, checkpoint, checkpoint_every, None, None, virtual=(virtual, vr),
                                max_steps=max_steps, serpentine=serpentine, subs=subs, nominal=nominal, nbs=nbs)
        affine = None
    aff = 0
    if affine is not None:
        if affine.dtype != torch.float64 or affine.numel() != 64 or affine.device != rows.device:
            raise ValueError("affine must be a [64] float64 tensor on the rows' device")
        aff = ptr(affine)
    sig = (_sgd_signature(n, d, C, lrs, momentum, nb, epochs, avg_from, tol, class_w, fit_intercept, comm, serpentine,
                          subs, nbs)
           if checkpoint else None)
    got = checkpoint.latest(sig) if checkpoint is not None else None
    start = (0, 0)
    if not rows.is_cuda:
        vv = (virtual, virtual.rows_f32()) if virtual is not None else None
        return _sgd_fit_cpu(rows, C, lrs, momentum, epochs, nb, avg_from, tol, class_w, w0, d, fit_intercept, comm,
                            fp8_scale, checkpoint, checkpoint_every, sig, got, virtual=vv, max_steps=max_steps,
                            serpentine=serpentine, subs=subs, nominal=nominal, nbs=nbs)
    if virtual is not None:
        virtual.check(rows)
        if class_w[1] > VIRTUAL_MAX_WEIGHT:
            raise ValueError(f"virtual SMOTE: positive class weight {class_w[1]} > {VIRTUAL_MAX_WEIGHT}")
        virtual.prepare()
    m = native()
    ws = workspace or LRWorkspace(rows.device)
    fp8 = storage_kind(rows) != "bf16"
    blocks = ref.sgd_grid_blocks(n_stored, nb, ws.sgd_blocks)
    dp = comm is not None and comm.world_size > 1
    persist = (persistent if persistent is not None else _persist_default()) and not dp
    persist = persist and epochs <= SGD_MAX_EPOCHS and m.sgd_persist_blocks(blocks) > 0
    # the one-launch path (no checkpoint, no DP): the init kernel preps the persistent workspace and
    # the recovery kernel exports the final state into a reserved pinned slot -- 2 launches fewer
    fused = persist and checkpoint is None and got is None
    ws.reset(w0, class_w, aff, persist=fused)
    s = stream_of(rows)
    if got is not None:
        ws.state.copy_(got[0]["state"].to(torch.float64).to(rows.device))
        if aff:
            m.logreg_fold(ptr(ws.state), aff, ptr(ws.w32), s)  # the state is standardized-space
        else:
            w32 = ws.state[S_W:S_W + 32].to(torch.float32)
            w32[LABEL_COL] = 0.0
            ws.w32.copy_(w32)
        start = (int(got[1]["epoch"]), int(got[1]["batch"]))
        # a fit that had converged before the checkpoint stays converged: its remaining passes and
        # updates are no-ops, as in the uninterrupted fit (reset() cleared the device flag)
        ws.done.fill_(int(float(got[0]["state"][S_CONV]) > 0))
    v = virtual
    mq, k = (v.nbr.shape if v is not None else (0, 1))

    vargs = (ptr(v.parents) if v else 0, ptr(v.nbr) if v else 0, ptr(v.lam) if v else 0,
             ptr(v.off) if v else 0, ptr(v.cnt) if v else 0, int(rows.shape[0]),
             int(v.q_offset) if v else 0, int(mq), int(k), int(hole[0]), int(hole[1]))

    def run_steps(s0: int, s1: int, prepped: bool = False, export_slot: int | None = None) -> int:
        """Steps [s0, s1) of the schedule: ONE persistent launch (a grid barrier per step, the
        update in every block), or one fused launch per step (FISH pass whose last block applies
        the update) -- bitwise the same fit.  Returns the stamp (> 0) when the persistent launch's
        recovery kernel exported the final state into ``export_slot``, else 0."""
        if s1 <= s0:
            return 0
        stamp = PendingFit.next_stamp() if (persist and export_slot is not None) else 0
        if persist:
            refused = m.sgd_persist(ptr(rows), int(fp8), float(fp8_scale), n + hole[1], ptr(ws.class_w), *vargs,
                                    ptr(ws.sgd_persist), ptr(ws.state), ptr(ws.w32), ptr(ws.done), aff, d, float(C),
                                    float(momentum), int(fit_intercept), float(tol), nb, int(epochs), int(avg_from),
                                    int(bool(serpentine)), [float(x) for x in lrs], int(s0), int(s1),
                                    4 * blocks, s, ptr(_stamps) if _stamps is not None else 0, subs, nbs,
                                    int(bool(_fault_test)), int(_spin_limit),
                                    PendingFit.slot_address(export_slot) if export_slot is not None else 0,
                                    int(bool(prepped)), stamp)
            if not refused:
                return stamp
            # the cooperative launch refused the grid: the per-step launches (bitwise the same fit)
        if serpentine:
            raise ValueError("serpentine minibatch order needs the persistent SGD launch")
        m.sgd_run(ptr(rows), int(fp8), float(fp8_scale), n + hole[1], ptr(ws.w32), ptr(ws.class_w), ptr(ws.done),
                  ptr(ws.partial), blocks, s, *vargs, ptr(ws.state), aff, d,
                  float(C), float(momentum), int(fit_intercept), float(tol), nb, int(epochs), int(avg_from),
                  [float(x) for x in lrs], int(s0), int(max(s0, s1)), ptr(ws.sgd_acc),
                  ptr(ws.sgd_acc[SGD_ACC_WORDS:]), subs, nbs)
        return 0

    if not dp and checkpoint is None:
        s0 = estart[start[0]] + start[1]
        slot = PendingFit.reserve() if fused else None
        exported = run_steps(s0, estart[epochs] if max_steps is None else min(estart[epochs], int(max_steps)),
                             prepped=fused, export_slot=slot)
        return PendingFit(ws.state, sgd=True, slot=slot, exported=exported)

    def dp_epochs(e0: int, e1: int, all_reduce):
        """Epochs [e0, e1) of the lean data-parallel schedule, enqueued with no host sync: per step
        the pass leaves its fixed-point sums (int64: the all-reduce is exact and order-free, every
        rank gets bitwise the same vector), one collective, the update.  A converged fit's passes
        and updates are no-ops (device `done`); its collectives still run on every rank.  The stream
        is queried here: under capture it is the capture stream."""
        s = stream_of(rows)
        for ep in range(e0, e1):
            c, nbe = lrs[ep], nbs[ep]
            for pos in range(nbe):
                b = _sgd_phase(pos, ep, nbe, serpentine)
                rsub, ph = nbe * subs[ep], b * subs[ep]
                m.sgd_pass_sums(ptr(rows), int(fp8), float(fp8_scale), n + hole[1], ptr(ws.w32), ptr(ws.class_w),
                                ptr(ws.done), rsub, ph, blocks, *vargs, ptr(ws.sgd_acc),
                                ptr(ws.sgd_acc[SGD_ACC_WORDS:]), ptr(ws.sgd_sums), aff, s)
                all_reduce(ws.sgd_sums)
                m.sgd_update_fixed(ptr(ws.sgd_sums), ptr(ws.state), ptr(ws.w32), ptr(ws.done), aff, d, float(C), c,
                                   float(momentum), int(fit_intercept), rsub, int(ep >= avg_from), int(pos + 1 == nbe),
                                   -1.0 if subs[ep] > 1 else float(tol), s)

    if dp and checkpoint is None and max_steps is None and start == (0, 0) and _dp_graph_ok(comm):
        # The whole DP schedule as hipGraph replays: the nominal epochs in one
        # graph, the extra epochs in another replayed only when the fit has not converged (the
        # same host check the eager loop makes).  Capture happens once per (buffers, schedule) key;
        # the graph holds the native RCCL all-reduces on the capture stream.
        key = (ptr(rows), int(rows.shape[0]), int(fp8), float(fp8_scale), n, tuple(hole), vargs, aff, d, float(C),
               float(momentum), int(fit_intercept), float(tol), tuple(lrs), tuple(subs), tuple(nbs), avg_from,
               bool(serpentine), blocks, nominal, epochs)
        # Captured natively (runtime/graphs.capture_native, one hipGraphLaunch per replay).  Opt-in:
        # on this ROCm build a launch of these graphs (kernels + RCCL nodes) returns only when the
        # device has run it -- with torch's CUDAGraph, natively, and alternating two instances alike
        # -- so the host enqueue per fit equals its device time (0.63 of 0.64 ms), where the eager
        # schedule enqueues in 0.25 ms and stays a fit ahead (profiles/r6_dpgraph).
        cache = ws.__dict__.setdefault("_dp_graphs", {})
        gs = cache.get(key)
        if gs is None:
            from ..runtime import graphs as rt_graphs

            nat = comm._native.all_reduce_
            gs = [rt_graphs.capture_native(lambda: dp_epochs(0, nominal, nat))]
            if epochs > nominal:
                gs.append(rt_graphs.capture_native(lambda: dp_epochs(nominal, epochs, nat)))
            if all(g is not None for g in gs):
                if len(cache) >= 4:  # a handful of shapes per workspace: drop the oldest
                    cache.pop(next(iter(cache)))
                cache[key] = gs
            else:
                gs = None
        if gs is not None:
            gs[0].replay()
            if len(gs) > 1 and not int(ws.done.item()):
                gs[1].replay()
            return PendingFit(ws.state, sgd=True)
    for ep in range(start[0], epochs):
        if ep >= nominal and int(ws.done.item()):  # converged: the extra epochs would be no-ops
            break
        c = lrs[ep]
        nbe = nbs[ep]
        for pos in range(start[1] if ep == start[0] else 0, nbe):
            if max_steps is not None and estart[ep] + pos >= max_steps:
                break
            b = _sgd_phase(pos, ep, nbe, serpentine)
            rsub, ph = nbe * subs[ep], b * subs[ep]
            avg = int(ep >= avg_from)
            last = pos + 1 == nbe
            if dp:
                # lean step: the pass leaves its fixed-point sums (int64: the all-reduce is exact and
                # order-free, every rank gets bitwise the same vector), one collective, the update
                m.sgd_pass_sums(ptr(rows), int(fp8), float(fp8_scale), n + hole[1], ptr(ws.w32), ptr(ws.class_w),
                                ptr(ws.done), rsub, ph, blocks, *vargs, ptr(ws.sgd_acc),
                                ptr(ws.sgd_acc[SGD_ACC_WORDS:]), ptr(ws.sgd_sums), aff, s)
                comm.all_reduce_(ws.sgd_sums)
                m.sgd_update_fixed(ptr(ws.sgd_sums), ptr(ws.state), ptr(ws.w32), ptr(ws.done), aff, d, float(C), c,
                                   float(momentum), int(fit_intercept), rsub, avg, int(last),
                                   -1.0 if subs[ep] > 1 else float(tol), s)
            else:  # the same kernels as the uninterrupted fit: checkpointed fits stay bit-identical
                run_steps(estart[ep] + pos, estart[ep] + pos + 1)
            gstep = estart[ep] + pos + 1
            if checkpoint is not None and (last or (checkpoint_every and gstep % checkpoint_every == 0)):
                nxt = (ep + 1, 0) if last else (ep, pos + 1)
                checkpoint.save(gstep, {"state": ws.state},
                                {"signature": sig, "epoch": nxt[0], "batch": nxt[1], "kind": "sgd"})
    return PendingFit(ws.state, sgd=True)


def _dp_graph_ok(comm) -> bool:
    """FDX_DP_GRAPH=1: the DP SGD schedule runs as hipGraph replays when its collectives are the
    native RCCL ones on the compute stream (default eager: see sgd_fit's measurement note)."""
    import os

    return getattr(comm, "_native", None) is not None and os.environ.get("FDX_DP_GRAPH", "0") == "1"


def _sgd_pass(m, rows, ws: LRWorkspace, n: int, fp8_scale: float, s: int, phase: int, nb: int, blocks: int,
              virtual: VirtualSmote | None, hole: tuple = (0, 0)):
    """Minibatch ``phase`` of ``nb``: the gradient + curvature-sum pass into ws.partial[:blocks]
    (``n`` logical rows: the hole excluded)."""
    dptr = ptr(ws.done)
    fp8 = storage_kind(rows) != "bf16"
    ha, hl = int(hole[0]), int(hole[1])
    end = n + hl
    if virtual is not None:
        v = virtual
        mq, k = v.nbr.shape
        m.logreg_pass_virtual(ptr(rows), 0, end, ptr(ws.w32), ptr(ws.class_w), dptr, 0, nb, ptr(ws.partial), blocks,
                              s, ptr(v.parents), ptr(v.nbr), ptr(v.lam), ptr(v.off), ptr(v.cnt), int(rows.shape[0]),
                              int(v.q_offset), int(mq), int(k), float(fp8_scale) if fp8 else 0.0, phase, True, ha, hl)
    elif not fp8:
        m.logreg_pass(ptr(rows), 0, end, ptr(ws.w32), ptr(ws.class_w), dptr, 0, nb, ptr(ws.partial), blocks, s,
                      phase, True, ha, hl)
    else:
        m.logreg_pass_fp8(ptr(rows), 0, end, ptr(ws.w32), ptr(ws.class_w), dptr, 0, nb, float(fp8_scale),
                          ptr(ws.partial), blocks, s, phase, True, ha, hl)


def sgd_minibatch_sums(rows: torch.Tensor, w: torch.Tensor, nb: int, phase: int, class_w=(1.0, 1.0),
                       fp8_scale: float = DEFAULT_FP8_SCALE, virtual: VirtualSmote | None = None,
                       blocks: int | None = None) -> dict:
    """One SGD minibatch pass, reduced (test / diagnostic API): gradient, loss, weight and
    curvature sums of minibatch ``phase`` of ``nb`` at weights ``w`` on the device."""
    m = native()
    ws = LRWorkspace(rows.device)
    ws.reset(w.cpu().double().numpy(), class_w)
    n = rows.shape[0]
    if virtual is not None:
        virtual.check(rows)
        virtual.prepare()
        n += virtual.n_new
    fp8 = storage_kind(rows) != "bf16"
    blocks = blocks or ref.sgd_grid_blocks(rows.shape[0], nb, ws.sgd_blocks)
    s = stream_of(rows)
    _sgd_pass(m, rows, ws, n, fp8_scale, s, phase, nb, blocks, virtual)
    m.logreg_reduce(ptr(ws.partial), blocks, SGD_SLOTS, ptr(ws.red), 0, s)
    red = ws.red[:SGD_SLOTS].cpu().numpy()
    return {"grad": red[:32].copy(), "loss": float(red[32]), "wsum": float(red[33]), "dsum": float(red[35]),
            "blocks": blocks}


S_SGD_FAULT = 229  # logreg.hip kSgdFault: 2 = the persistent SGD fit ran on its recovery launch


def _info_from_state(st: np.ndarray, sgd: bool = False) -> FitInfo:
    if sgd and st[S_SGD_FAULT] not in (0.0, 2.0):
        raise RuntimeError(f"persistent SGD launch: unexpected fault state {st[S_SGD_FAULT]}")
    return FitInfo(w=st[S_W:S_W + 32].copy(), n_iter=int(st[S_ITER]), n_newton_steps=0 if sgd else int(st[S_NACC]),
                   converged=bool(st[S_CONV] > 0), objective=float(st[S_OBJ]), grad_max=float(st[S_GMAX]),
                   recovered=bool(sgd and st[S_SGD_FAULT] == 2.0))


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


def _sgd_fit_cpu(rows, C, lrs, momentum, epochs, nb, avg_from, tol, class_w, w0, d, fit_intercept, comm, fp8_scale,
                 checkpoint=None, checkpoint_every=0, sig=None, got=None, virtual=None, max_steps=None,
                 serpentine=False, subs=None, nominal=None, nbs=None):
    """The device SGD's algorithm in fp64 (ref.SgdStateRef) over the same minibatch partition:
    stored row tiles by the pass grid's strided walk (the full SGD grid of a 256-CU part,
    ref.SGD_FULL_BLOCKS, shrunk for small shards like the device), virtual samples by their pick tile."""
    R = ref.rows_to_f32(rows, fp8_scale, d).double().numpy()
    n_stored = R.shape[0]
    subs = list(subs) if subs is not None else [1] * max(epochs, 1)
    nbs = list(nbs) if nbs is not None else [nb] * max(epochs, 1)
    estart = np.concatenate([[0], np.cumsum(nbs)]).astype(int).tolist()
    blocks = ref.sgd_grid_blocks(n_stored, nb, ref.SGD_FULL_BLOCKS)
    parts = [R]
    pick = None
    if virtual is not None:
        v, vr = virtual
        mq, k = v.nbr.shape
        pick, _ = ref.smote_pick_draws(int(mq), int(k), int(v.n_new), int(v.seed), int(v.counter_base),
                                       int(v.sample_offset))
        parts.append(np.asarray(vr, dtype=np.float64))
    R = np.concatenate(parts)
    members_of = {}

    def members(rsub: int, ph: int):
        """Rows of phase ph of a grid of rsub minibatches (an epoch with sub-sample s: rsub = nb s)."""
        if rsub not in members_of:
            bs = [ref.sgd_row_batches(n_stored, rsub, blocks)]
            if pick is not None:
                bs.append(ref.sgd_pick_batches(mq * k, rsub, ref.PICK_TILE)[pick.astype(np.int64)])
            batch_of = np.concatenate(bs)
            members_of[rsub] = [np.nonzero(batch_of == b)[0] for b in range(rsub)]
        return members_of[rsub][ph]

    st = ref.SgdStateRef(w0)
    start = (0, 0)
    if got is not None:
        sv = got[0]["state"].numpy()
        st.w, st.v = sv[S_W:S_W + 32].copy(), sv[S_VEL:S_VEL + 32].copy()
        st.avg, st.ep_g = sv[160:192].copy(), sv[192:224].copy()
        st.ep_loss, st.ep_w, st.n_avg, st.iter = float(sv[224]), float(sv[225]), int(sv[226]), int(sv[S_ITER])
        st.gmax, st.obj, st.converged = float(sv[S_GMAX]), float(sv[S_OBJ]), bool(sv[S_CONV] > 0)
        st.done = st.converged
        start = (int(got[1]["epoch"]), int(got[1]["batch"]))
    for ep in range(start[0], epochs):
        if nominal is not None and ep >= nominal and st.done:  # converged: extra epochs are no-ops
            break
        nbe = nbs[ep]
        for pos in range(start[1] if ep == start[0] else 0, nbe):
            if max_steps is not None and estart[ep] + pos >= max_steps:
                break
            b = _sgd_phase(pos, ep, nbe, serpentine)
            Rb = R[members(nbe * subs[ep], b * subs[ep])]
            g, loss, wsum, _ = ref.logreg_pass(Rb, st.w, class_w, False)
            X = Rb.copy()
            X[:, LABEL_COL] = 0.0
            wv = st.w.copy()
            wv[LABEL_COL] = 0.0
            p = ref.sigmoid(X @ wv)
            sw = np.where(Rb[:, LABEL_COL] > 0.5, class_w[1], class_w[0])
            red = np.concatenate([g, [loss, wsum, 0.0, float(np.sum(sw * p * (1 - p)))]])
            if comm is not None and comm.world_size > 1:
                red = comm.all_reduce(torch.from_numpy(red)).numpy()
            last = pos + 1 == nbe
            st.step(red[:32], red[32], red[33], red[35], d, C, lrs[ep], momentum, nbe * subs[ep],
                    ep >= avg_from, last, -1.0 if subs[ep] > 1 else tol, fit_intercept)
            gstep = estart[ep] + pos + 1
            if checkpoint is not None and (last or (checkpoint_every and gstep % checkpoint_every == 0)):
                sv = np.zeros(STATE_SIZE)
                sv[S_W:S_W + 32], sv[S_VEL:S_VEL + 32], sv[160:192], sv[192:224] = st.w, st.v, st.avg, st.ep_g
                sv[224], sv[225], sv[226], sv[S_ITER] = st.ep_loss, st.ep_w, st.n_avg, st.iter
                sv[S_GMAX], sv[S_OBJ], sv[S_CONV] = st.gmax, st.obj, float(st.converged)
                nxt = (ep + 1, 0) if last else (ep, pos + 1)
                checkpoint.save(gstep, {"state": sv},
                                {"signature": sig, "epoch": nxt[0], "batch": nxt[1], "kind": "sgd"})
    w = st.w.copy()
    w[LABEL_COL] = 0.0
    return FitInfo(w=w, n_iter=st.iter, n_newton_steps=0, converged=st.converged, objective=st.obj,
                   grad_max=st.gmax)
