"""K1 scaler statistics / K2 standardize+pad+cast / stable label compaction."""
from __future__ import annotations

import time

from dataclasses import dataclass

import numpy as np
import torch

from . import reference as ref
from .layout import DEFAULT_FP8_SCALE, DTYPE_KIND, NCOLS, NFEAT_MAX, TORCH_STORAGE
from .native import native, ptr, stream_of

_SCALER_BLOCKS = 2048  # 8 resident blocks per CU x 256 CUs


@dataclass
class ScalerStats:
    """StandardScaler parameters; fp64 for sklearn export, fp32 copies feed the kernels.
    ``n`` may be given as a device tensor (the all-reduced count): it is read on first use."""

    n_src: object          # float, or a 1-element device tensor holding the row count
    d: int
    mean64: torch.Tensor   # [32] float64
    var64: torch.Tensor    # [32] float64
    scale64: torch.Tensor  # [32] float64
    mean32: torch.Tensor   # [32] float32
    inv32: torch.Tensor    # [32] float32 (0 beyond d)
    # set by scaler_fit_cast: [64] float64 (c | 1/sigma) mapping pivot-shifted rows s = x - pivot
    # to standardized ones, z = (s - c) / sigma (identity beyond d)
    aff: torch.Tensor | None = None

    @property
    def n(self) -> float:
        if isinstance(self.n_src, torch.Tensor):
            self.n_src = float(self.n_src.item())
        return float(self.n_src)

    def to(self, device) -> "ScalerStats":
        return ScalerStats(self.n_src, self.d, *(t.to(device) for t in
                                             (self.mean64, self.var64, self.scale64, self.mean32, self.inv32)),
                           aff=None if self.aff is None else self.aff.to(device))

    def shifted_to_standard(self, rows_f32: torch.Tensor) -> torch.Tensor:
        """z rows from pivot-shifted fp32 rows [m, 32] (affine map on the feature columns)."""
        a = self.aff.to(rows_f32.device, torch.float32)
        return (rows_f32 - a[:32]) * a[32:]

    def standard_to_shifted(self, rows_f32: torch.Tensor) -> torch.Tensor:
        """Pivot-shifted fp32 rows from standardized ones (inverse of shifted_to_standard)."""
        a = self.aff.to(rows_f32.device, torch.float64)
        return torch.addcmul(a[:32].float(), rows_f32, (1.0 / a[32:]).float())

    def numpy(self):
        d = self.d
        return (self.mean64[:d].cpu().numpy(), self.var64[:d].cpu().numpy(), self.scale64[:d].cpu().numpy())


def _check_X(X: torch.Tensor) -> None:
    if X.dim() != 2 or X.dtype != torch.float32:
        raise ValueError(f"X must be 2-D float32, got {X.dtype} {tuple(X.shape)}")
    if X.shape[1] > NFEAT_MAX:
        raise ValueError(f"at most {NFEAT_MAX} features supported, got {X.shape[1]}")
    if X.stride(1) != 1:
        raise ValueError("X must be row-major with unit column stride")


def _pivot_dev(pivot: torch.Tensor, d: int, dev) -> torch.Tensor:
    """The kernels read pivot[c] for c < d only: a contiguous fp32 device row is used in place."""
    if pivot.is_cuda and pivot.device == dev and pivot.dtype == torch.float32 and pivot.is_contiguous() \
            and pivot.numel() >= d:
        return pivot
    piv = torch.zeros(NCOLS, device=dev, dtype=torch.float32)
    piv[:d] = pivot[:d].to(dev, torch.float32)
    return piv


def scaler_partial_sums(X: torch.Tensor, pivot: torch.Tensor) -> torch.Tensor:
    """Shifted fp64 sums [64] = (sum(x - pivot) | sum((x - pivot)^2)) over the rows of X."""
    _check_X(X)
    n, d = X.shape
    if not X.is_cuda:
        return torch.from_numpy(ref.scaler_sums(X.numpy(), pivot.cpu().numpy()))
    m = native()
    piv = _pivot_dev(pivot, d, X.device)
    nb = min(_SCALER_BLOCKS, max(1, (n + 255) // 256))
    partial = torch.empty((nb + m.scaler_reduce_scratch_rows(nb)) * 64, device=X.device, dtype=torch.float64)
    sums = torch.empty(64, device=X.device, dtype=torch.float64)
    s = stream_of(X)
    m.scaler_partial(ptr(X), n, X.stride(0), d, ptr(piv), ptr(partial), nb, s)
    m.scaler_reduce(ptr(partial), nb, ptr(sums), s)
    return sums


def _aff_cpu(sums: np.ndarray, n: float, scale: np.ndarray, d: int) -> torch.Tensor:
    aff = np.zeros(64)
    aff[32:] = 1.0
    aff[:d] = sums[:d] / n
    aff[32:32 + d] = 1.0 / scale[:d]
    return torch.from_numpy(aff)


def scaler_finalize(sums: torch.Tensor, n_total, pivot: torch.Tensor, d: int, want_aff: bool = False,
                    colscale: torch.Tensor | None = None, nparts: int = 1) -> ScalerStats:
    """``n_total`` None: the count is in sums[31] (device) -- see scaler_fit.  ``colscale`` (fp8
    rows, [d] float32): the stored values are v = s * colscale, folded into ``aff``.  ``nparts``
    (device): ``sums`` is [nparts][64] first-level reduce rows, summed in order by the kernel."""
    dev = sums.device
    if n_total is None and not sums.is_cuda:
        n_total = float(sums[31])
    if not sums.is_cuda:
        mean, var, scale, m32, i32 = ref.scaler_finalize(sums.numpy(), float(n_total), pivot.cpu().numpy(), d)
        aff = _aff_cpu(sums.numpy(), float(n_total), scale, d) if want_aff else None
        if aff is not None and colscale is not None:
            k = torch.ones(32, dtype=torch.float64)
            k[:d] = colscale[:d].cpu().to(torch.float64)
            aff = torch.cat([aff[:32] * k, aff[32:] / k])
        return ScalerStats(float(n_total), d, torch.from_numpy(mean), torch.from_numpy(var),
                           torch.from_numpy(scale), torch.from_numpy(m32), torch.from_numpy(i32), aff=aff)
    m = native()
    piv = _pivot_dev(pivot, d, dev)
    mean64 = torch.empty(32, device=dev, dtype=torch.float64)
    var64 = torch.empty_like(mean64)
    scale64 = torch.empty_like(mean64)
    mean32 = torch.empty(32, device=dev, dtype=torch.float32)
    inv32 = torch.empty_like(mean32)
    aff = torch.empty(64, device=dev, dtype=torch.float64) if want_aff else None
    m.scaler_finalize(ptr(sums), -1.0 if n_total is None else float(n_total), ptr(piv), d, ptr(mean64), ptr(var64),
                      ptr(scale64), ptr(mean32), ptr(inv32), ptr(aff), stream_of(sums),
                      ptr(colscale if (want_aff and colscale is not None) else None), int(nparts))
    n_src = sums[31:32] if n_total is None else float(n_total)
    return ScalerStats(n_src, d, mean64, var64, scale64, mean32, inv32, aff=aff)


def scaler_fit(X: torch.Tensor, comm=None, pivot: torch.Tensor | None = None) -> ScalerStats:
    """StandardScaler.fit on device.  With ``comm`` (parallel.comm.Communicator) the shifted sums
    and row counts are all-reduced so every rank gets the global statistics (collective C1)."""
    _check_X(X)
    n, d = X.shape
    if pivot is None:
        if comm is not None and comm.world_size > 1:
            pivot = X[0].clone() if n > 0 else torch.zeros(d, device=X.device)
            pivot = comm.broadcast(pivot.contiguous(), src=0)
        else:
            pivot = X[0] if n > 0 else torch.zeros(d, device=X.device)  # a view: no copy kernel
    sums = scaler_partial_sums(X, pivot)
    if comm is not None and comm.world_size > 1:
        # count rides in the unused slot 31 (d <= 30): one all-reduce, no host sync
        sums[31:32].fill_(float(n))
        sums = comm.all_reduce(sums)
        return scaler_finalize(sums, None, pivot, d)
    return scaler_finalize(sums, float(n), pivot, d)


_GRID_CACHE: dict = {}


def _stats_cast_grid(m, dev, fp8: bool = False) -> int:
    """Every block of the fused pass resident at once (occupancy-derived, per row format).
    Leaving block slots free for the side-stream count kernels was measured no faster
    (profiles/r2_s6, reserveab)."""
    key = (dev.index, bool(fp8))
    if key not in _GRID_CACHE:
        _GRID_CACHE[key] = int(m.scaler_stats_cast_blocks(int(bool(fp8))))
    return _GRID_CACHE[key]


def fused_cast_ok(X: torch.Tensor) -> bool:
    """The fused K1+K2 kernel reads contiguous 16-byte aligned [n, d <= 30] fp32 rows."""
    return (not X.is_cuda) or (X.is_contiguous() and X.data_ptr() % 16 == 0 and X.shape[1] <= 30)


def fp8_fused_prescale(X: torch.Tensor, comm=None, sample_rows: int = 65536):
    """(pivot [d], colscale [d]) float32 for the fp8 fused cast: mean and 1/std of ``sample_rows``
    rows strided over the shard (rank 0's under DP, broadcast), so the stored e4m3 values are
    ~z * scale.
    Only a prescale: the exact statistics of the same pass define the solver's affine map."""
    n, d = X.shape
    if comm is not None and comm.world_size > 1:
        buf = torch.zeros(2 * d, device=X.device, dtype=torch.float32)
        if comm.rank == 0:
            buf.copy_(torch.cat(_sample_moments(X, sample_rows)))
        buf = comm.broadcast(buf, src=0)
        return buf[:d].contiguous(), buf[d:].contiguous()
    return _sample_moments(X, sample_rows)


def _sample_moments(X: torch.Tensor, sample_rows: int):
    # strided over the whole shard: tables are often ordered (the creditcard Time column is
    # sorted), so the first rows are not a sample
    stride = max(1, X.shape[0] // max(1, sample_rows))
    if X.is_cuda and X.is_contiguous() and X.shape[0] > 0:
        # three small launches (sample partials -> fixed-order reduce -> mean, 1/std) instead of
        # ~10 torch ops (gather, cast, mean, std, where: ~0.25 ms of launches on the fit's path)
        m = native()
        n, d = X.shape
        ns = min(sample_rows, (n - 1) // stride + 1)
        nb = m.fp8_prescale_blocks()
        ws = torch.empty((nb + m.scaler_reduce_scratch_rows(nb)) * 64 + 64, device=X.device, dtype=torch.float64)
        out = torch.empty(2 * d, device=X.device, dtype=torch.float32)
        m.fp8_prescale(ptr(X), n, d, ns, stride, ptr(ws), ptr(ws[-64:]), ptr(out), ptr(out[d:]), stream_of(X))
        return out[:d], out[d:]
    smp = X[::stride][:sample_rows].double()
    mu = smp.mean(0)
    sd = smp.std(0, unbiased=False)
    k = torch.where(sd > 0, 1.0 / sd, torch.ones_like(sd))
    return mu.float().contiguous(), k.float().contiguous()


def scaler_fit_cast(X: torch.Tensor, labels: torch.Tensor | None, out: torch.Tensor, comm=None,
                    pivot: torch.Tensor | None = None, bias_value: float = 1.0,
                    fp8_scale: float = DEFAULT_FP8_SCALE, out_idx: torch.Tensor | None = None) -> ScalerStats:
    """StandardScaler.fit fused with the row cast: ONE read of X yields the (all-reduced)
    statistics and the training rows in ``out`` [n, 32] (col 30 = bias_value, col 31 = label):
      * bf16: pivot-shifted rows s = x - pivot;
      * fp8 (uint8 out): e4m3 of s' = (x - p) * k * fp8_scale with a sample prescale (p ~ mean,
        k ~ 1/sigma: fp8_fused_prescale) -- 32 B rows, half the bf16 bytes.
    The returned stats carry ``aff`` mapping the stored feature values (fp8: after dividing by
    fp8_scale) to standardized ones, z = (v - c) * inv, which the Newton solver applies as an exact
    affine map of its sums (ops/logreg.newton_fit(affine=...)): same model, half the raw-matrix
    traffic of scaler_fit + scale_cast.
    ``out_idx`` (int64 [n] destination rows, a permutation, device): scatter form -- row i of X is
    written to out[out_idx[i]], e.g. the fold-sorted training table of a CV job straight from the
    raw table.  X is still read in order (a gather of the 120-byte raw rows ran at a third of the
    streaming rate: 772 vs 256 us at 8M rows, profiles/r4_i/timeline_cv_job.txt); the statistics are
    those of the in-order pass."""
    _check_X(X)
    idx = out_idx
    if idx is not None:
        if idx.dtype != torch.int64 or idx.shape != (X.shape[0],) or idx.device != X.device:
            raise ValueError("out_idx must be an int64 [n] tensor on X's device")
    n = X.shape[0]
    d = X.shape[1]
    fp8 = out.dtype == torch.uint8
    if out.shape != (n, NCOLS) or out.dtype not in (torch.bfloat16, torch.uint8) or not out.is_contiguous():
        raise ValueError(f"bad output buffer {tuple(out.shape)} {out.dtype}")
    if labels is not None and (labels.dtype != torch.uint8 or labels.shape[0] != X.shape[0]):
        raise ValueError("labels must be uint8 [n] aligned with X")
    dist = comm is not None and comm.world_size > 1
    colscale = None
    if fp8:
        pivot_fp8, colscale = fp8_fused_prescale(X, comm)  # a sample of X: any order of its rows
        pivot = pivot_fp8 if pivot is None else pivot
    if pivot is None:
        if dist:
            pivot = X[0].clone() if n > 0 else torch.zeros(d, device=X.device)
            pivot = comm.broadcast(pivot.contiguous(), src=0)
        else:
            pivot = X[0] if n > 0 else torch.zeros(d, device=X.device)
    if not X.is_cuda:
        sums = torch.from_numpy(ref.scaler_sums(X.numpy(), pivot.cpu().numpy()))
        o = torch.zeros((n, NCOLS), dtype=torch.float32)
        o[:, :d] = X - pivot[:d].to(torch.float32)
        if fp8:
            o[:, :d] *= colscale[:d] * fp8_scale
        o[:, 30] = bias_value
        if labels is not None:
            o[:, 31] = labels.to(torch.float32)
        cast = torch.from_numpy(ref.fp8_encode(o.numpy())) if fp8 else o.to(torch.bfloat16)
        if idx is None:
            out.copy_(cast)
        else:
            out[idx] = cast
    else:
        if not fused_cast_ok(X) or out.data_ptr() % 16:
            raise ValueError("scaler_fit_cast: X must be contiguous and 16-byte aligned with d <= 30")
        m = native()
        piv = _pivot_dev(pivot, d, X.device)
        # all blocks resident at once (occupancy-derived), never more than the tiles
        nb = max(1, min(_stats_cast_grid(m, X.device, fp8), (n + 127) // 128))
        # block partials, then >= 1 row for the first-level reduce output
        partial = torch.empty((nb + max(1, m.scaler_reduce_scratch_rows(nb))) * 64, device=X.device,
                              dtype=torch.float64)
        sums = torch.empty(64, device=X.device, dtype=torch.float64)
        s = stream_of(X)
        nparts = 1
        if n > 0:
            m.scaler_stats_cast(ptr(X), n, d, ptr(piv), ptr(labels), float(bias_value), ptr(out), ptr(partial), nb, s,
                                ptr(colscale), float(fp8_scale) if fp8 else 1.0, ptr(idx))
            if dist:  # the all-reduce needs the one [64] sums vector
                m.scaler_reduce(ptr(partial), nb, ptr(sums), s)
            else:  # first level only: the finalize kernel sums its rows (one launch fewer)
                mid = partial[nb * 64:]
                nparts = int(m.scaler_reduce_level1(ptr(partial), nb, ptr(mid), s))
                sums = mid[: nparts * 64]
        else:
            sums.zero_()
    if dist:
        sums[31:32].fill_(float(n))
        sums = comm.all_reduce(sums)
        st = scaler_finalize(sums, None, pivot, d, want_aff=True, colscale=colscale)
    else:
        st = scaler_finalize(sums, float(n), pivot, d, want_aff=True, colscale=colscale,
                             nparts=nparts if X.is_cuda else 1)
    # fp8: stored v = s * k  ->  z = (s - c) * inv = (v - k c) * (inv / k), folded in the finalize
    return st


def scale_cast(X: torch.Tensor, stats: ScalerStats, labels: torch.Tensor | None = None,
               out_dtype: str = "bf16", out: torch.Tensor | None = None, idx: torch.Tensor | None = None,
               bias_value: float = 1.0, fp8_scale: float = DEFAULT_FP8_SCALE) -> torch.Tensor:
    """Standardize raw fp32 rows into the padded 32-column device layout (K2)."""
    _check_X(X)
    n_out = X.shape[0] if idx is None else idx.shape[0]
    d = X.shape[1]
    if labels is not None and (labels.dtype != torch.uint8 or labels.shape[0] != X.shape[0]):
        raise ValueError("labels must be uint8 [n] aligned with X")
    if out is None:
        out = torch.empty((n_out, NCOLS), device=X.device, dtype=TORCH_STORAGE[out_dtype])
    if out.shape != (n_out, NCOLS) or out.dtype != TORCH_STORAGE[out_dtype] or not out.is_contiguous():
        raise ValueError(f"bad output buffer {tuple(out.shape)} {out.dtype}")
    if not X.is_cuda:
        r = ref.scale_cast(X.numpy(), stats.mean32.cpu().numpy(), stats.inv32.cpu().numpy(),
                           None if labels is None else labels.numpy(), bias_value, out_dtype, fp8_scale,
                           None if idx is None else idx.numpy())
        out.copy_(r)
        return out
    if idx is not None:
        if idx.dtype != torch.int64 or not idx.is_cuda:
            raise ValueError("idx must be a device int64 tensor")
    if out.data_ptr() % 16:
        raise ValueError("output rows must be 16-byte aligned")
    m = native()
    m.scale_cast(ptr(X), X.shape[0] if idx is None else n_out, X.stride(0), d, ptr(idx),
                 ptr(stats.mean32), ptr(stats.inv32), ptr(labels), float(bias_value), float(fp8_scale),
                 DTYPE_KIND[out_dtype], ptr(out), stream_of(X))
    return out


class PendingCompaction:
    """Count/scan kernels enqueued; the scan also stores the total into a mapped pinned word.
    ``result()`` spins on that word (it lands a few microseconds after the scan, with no D2H
    copy kernel and no event wake-up on the path), then enqueues the write of the stable index
    list.  Work enqueued after the scan keeps the GPU busy meanwhile."""

    _pool: list = []  # rotating pinned slots (pinned allocation costs tens of microseconds)
    _views: list = []  # numpy views of the slots (host reads/writes without torch dispatch)
    _dev: list = []  # device addresses of the slots (0: not mapped -> D2H copy + event)
    _owners: list = []  # the pending compaction whose count each slot still holds
    _next = 0
    _POOL = 8
    SPIN_S = 0.05  # then fall back to the event (a stalled or faulted stream surfaces as its error)

    @classmethod
    def take_slot(cls):
        """A free pinned slot, reset to -1 (the scan writes a count >= 0).  A ninth compaction in
        flight settles the slot's previous owner first."""
        if not cls._pool:
            cls._pool = [torch.empty(1, dtype=torch.int64, pin_memory=True) for _ in range(cls._POOL)]
            cls._views = [t.numpy() for t in cls._pool]
            cls._dev = [int(native().host_device_pointer(t.data_ptr())) for t in cls._pool]
            cls._owners = [None] * cls._POOL
        slot = cls._next % cls._POOL
        cls._next += 1
        prev = cls._owners[slot]
        if prev is not None:
            prev.result()
        cls._owners[slot] = None
        cls._views[slot][0] = -1
        return slot, cls._dev[slot]

    def __init__(self, labels, target, nb, counts, total, slot: int, side: bool = False, home=None):
        cls = PendingCompaction
        self.labels, self.target, self.nb, self.counts = labels, target, nb, counts
        # the stream the index list belongs to (its consumers run there): result() enqueues the
        # write there whichever stream is current when it is called -- e.g. when a later
        # compaction settles this one from inside its side-stream context
        self.home = home if home is not None else torch.cuda.current_stream(labels.device)
        # a side-stream count writes `total` concurrently with the compute stream: hold it until
        # result() has waited for that stream, or the caching allocator hands its block to a
        # compute-stream tensor while the scan may still write it
        self.side, self.total = side, total
        cls._owners[slot] = self
        self._slot = slot
        self.host = cls._pool[slot]
        if not cls._dev[slot]:
            self.host.copy_(total, non_blocking=True)
        # the scan stores the count into the mapped slot itself: then no event is recorded behind
        # it (a marker costs the command processor ~6 us in front of the scaler pass,
        # profiles/r6_marker); the spin's fallback waits on the stream instead
        self.event = None
        if side or not cls._dev[slot]:
            self.event = torch.cuda.Event()
            self.event.record()
        self._out = None

    def _drain(self):
        if self.event is not None:
            self.event.synchronize()
        else:
            self.home.synchronize()

    def _count(self) -> int:
        v = PendingCompaction._views[self._slot]
        if PendingCompaction._dev[self._slot]:
            t0 = time.perf_counter()
            while v[0] < 0:
                if time.perf_counter() - t0 > self.SPIN_S:
                    self._drain()
                    if v[0] < 0:
                        raise RuntimeError("compaction: count not written after its stream drained")
                    break
        else:
            self._drain()
        return int(v[0])

    def result(self) -> torch.Tensor:
        if self._out is None:
            cnt = self._count()
            with torch.cuda.stream(self.home):
                if self.side:  # counts were written on the side stream
                    self.home.wait_event(self.event)
                if PendingCompaction._owners[self._slot] is self:
                    PendingCompaction._owners[self._slot] = None
                self.total = None
                out = torch.empty(cnt, device=self.labels.device, dtype=torch.int64)
                if cnt:
                    native().compact_write(ptr(self.labels), self.labels.shape[0], self.target, ptr(self.counts),
                                           ptr(out), self.nb, self.home.cuda_stream)
                self._out = out
        return self._out


class _Ready:
    def __init__(self, out):
        self._out = out

    def result(self):
        return self._out


def compact_indices_async(labels: torch.Tensor, target: int = 1, nblocks: int = 512,
                          side=None, ready=None):
    """Stable indices of rows whose label == target, as a pending result (see PendingCompaction).

    ``side`` (torch.cuda.Stream) runs the count/scan kernels and the count's copy to the host on
    that stream, after ``ready`` (a torch.cuda.Event recorded on the current stream once the labels
    are written): the caller can enqueue its big kernel on the current stream first and the count
    runs beside it instead of in front of it (pipeline.fit: the fused scaler pass starts ~30 us
    sooner at the fit boundary, profiles/r2_s6).  ``result()`` orders the current stream after the
    side stream's kernels before it writes the index list."""
    if labels.dtype != torch.uint8 or labels.dim() != 1:
        raise ValueError("labels must be 1-D uint8")
    n = labels.shape[0]
    if not labels.is_cuda:
        return _Ready(torch.nonzero(labels == target, as_tuple=False).reshape(-1).to(torch.int64))
    m = native()
    nb = int(max(1, min(nblocks, (n + 255) // 256)))
    if side is None:
        counts = torch.empty(nb, device=labels.device, dtype=torch.int64)
        total = torch.empty(1, device=labels.device, dtype=torch.int64)
        s = stream_of(labels)
        slot, hdev = PendingCompaction.take_slot()
        m.compact_count(ptr(labels), n, target, ptr(counts), nb, s)
        m.exclusive_scan_small(ptr(counts), nb, ptr(total), s, hdev)
        return PendingCompaction(labels, target, nb, counts, total, slot)
    compute = torch.cuda.current_stream(labels.device)
    if ready is not None:
        side.wait_event(ready)
    with torch.cuda.stream(side):
        # scratch from the SIDE stream's pool: a block from the compute stream's pool may have
        # been freed by a tensor whose compute-stream kernels are still queued (e.g. the scaler
        # pass's partial sums), which is safe only for compute-stream reuse
        counts = torch.empty(nb, device=labels.device, dtype=torch.int64)
        total = torch.empty(1, device=labels.device, dtype=torch.int64)
        slot, hdev = PendingCompaction.take_slot()
        m.compact_count(ptr(labels), n, target, ptr(counts), nb, side.cuda_stream)
        m.exclusive_scan_small(ptr(counts), nb, ptr(total), side.cuda_stream, hdev)
        pend = PendingCompaction(labels, target, nb, counts, total, slot, side=True, home=compute)
    counts.record_stream(compute)  # result() launches the index write on the compute stream
    return pend


def compact_indices(labels: torch.Tensor, target: int = 1, nblocks: int = 512) -> torch.Tensor:
    """Stable indices of rows whose label == target (device: 3 deterministic kernels)."""
    return compact_indices_async(labels, target, nblocks).result()


def stats_from_numpy(mean: np.ndarray, scale: np.ndarray, n: float = 0.0, var=None, device="cpu") -> ScalerStats:
    """Build kernel-ready stats from an existing (e.g. sklearn) scaler's mean_/scale_."""
    d = len(mean)
    mean64 = np.zeros(32)
    scale64 = np.ones(32)
    var64 = np.zeros(32)
    mean64[:d] = mean
    scale64[:d] = scale
    var64[:d] = scale ** 2 if var is None else var
    inv32 = np.zeros(32, dtype=np.float32)
    inv32[:d] = (1.0 / np.asarray(scale, dtype=np.float64)).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    return ScalerStats(float(n), d, t(mean64), t(var64), t(scale64), t(mean64.astype(np.float32)), t(inv32))
