"""Communicator for data-parallel training (SURVEY.md §2.4 collectives C1-C9).

One process per GPU.  Backends:
  * ``nccl``  torch.distributed over RCCL (on ROCm the "nccl" backend IS RCCL) across xGMI;
  * ``rccl``  the native communicator in csrc/comm/rccl_comm.cpp (ncclCommInitRank on our own
              unique id, collectives enqueued on the compute stream: no ProcessGroup work
              objects, capturable in hipGraphs) -- used for the hot all-reduces whenever every
              rank loads it and passes a known all-reduce (FDX_COMM=auto, the default;
              FDX_COMM=torch forces the ProcessGroup, FDX_COMM=rccl makes failure fatal);
  * ``gloo``  CPU tensors (tests, world_size > 1 without GPUs; CUDA tensors are host-staged,
              so several ranks can share one GPU in tests).

All payloads in this framework are tiny (<= 8.5 KB per Newton iteration) except the SMOTE
minority all-gather, so the API is shaped for latency: one fused buffer per step, in-place
all-reduce on the current stream.

Ordering contract between the two communicators on one GPU (torch ProcessGroup for barriers and
device scalars; the native RCCL communicator for every device all-reduce and row all-gather): both are only
ever driven from this class, in program order, from one host thread per rank.  The native
collectives run on the current compute stream; a ProcessGroup collective waits for the current
stream before it starts and (synchronous ops) makes the current stream wait for its completion.
So on every rank the device executes ONE total order of collectives -- the program order -- and
since every rank runs the same control flow, all ranks issue the same sequence: no cross-
communicator deadlock is possible.  Host-value exchanges (``all_gather_ints``,
``all_reduce_scalar``) go over a third, CPU-only gloo group: they never wait for the device
stream (a DP fit's row/minority-count exchange used to block the host behind the ~280 us fused
scaler pass, leaving the GPU idle while the host then enqueued the k-NN), and they only ever wait
on other ranks' HOSTS, which have already enqueued every earlier device collective -- so they
cannot close a cycle with the device order either.  ``FDX_COMM_TRACE=1`` records that sequence per rank
(``trace``), and tests/test_distributed.py asserts it is identical on every rank.

Every collective is timed (HIP events on the stream it runs on, host clock for gloo) and
observed in ``fdx_allreduce_seconds{op}``; ``collective_summary()`` gives the per-op breakdown
bench.py reports under DP.
"""
from __future__ import annotations

import contextlib
import os
import time
from datetime import timedelta

import torch
import torch.distributed as dist


_SHM_DTYPES = (torch.float32, torch.float64, torch.int32, torch.int64)


class CollectiveStats:
    """Per-op count / bytes / total and max seconds.  Device-timed entries are resolved lazily
    (their events complete asynchronously); ``summary()`` synchronises and resolves them."""

    def __init__(self):
        self.pending = []
        self.acc: dict = {}

    def _add(self, op: str, nbytes: int, sec: float):
        a = self.acc.setdefault(op, [0, 0, 0.0, 0.0])
        a[0] += 1
        a[1] += nbytes
        a[2] += sec
        a[3] = max(a[3], sec)
        try:
            from ..obs.metrics import train_metrics

            train_metrics().allreduce_seconds.labels(op).observe(sec)
        except Exception:  # noqa: BLE001 - metrics are best effort
            pass

    def count(self, op: str, nbytes: int):
        """An untimed collective: count and bytes only."""
        a = self.acc.setdefault(op, [0, 0, 0.0, 0.0])
        a[0] += 1
        a[1] += nbytes

    def resolve(self, block: bool = False):
        keep = []
        for op, nbytes, e0, e1 in self.pending:
            if block or e1.query():
                self._add(op, nbytes, e0.elapsed_time(e1) / 1e3)
            else:
                keep.append((op, nbytes, e0, e1))
        self.pending = keep

    def summary(self) -> dict:
        if self.pending:
            torch.cuda.synchronize()
            self.resolve(block=True)
        return {op: {"count": a[0], "bytes": a[1], "total_ms": round(a[2] * 1e3, 4),
                     "mean_us": round(a[2] / max(a[0], 1) * 1e6, 2), "max_us": round(a[3] * 1e6, 2)}
                for op, a in sorted(self.acc.items())}

    def reset(self):
        self.pending, self.acc = [], {}


def _single_node_gloo_iface():
    """Every rank of a single-node job whose rendezvous is on the loopback address reaches the
    others over loopback: pin gloo's TCP device to `lo` instead of resolving the host name (which
    may not resolve in a container) unless the user chose an interface."""
    if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost") and os.path.exists("/sys/class/net/lo"):
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")


class Communicator:
    def __init__(self, backend: str | None = None, device: torch.device | None = None):
        self.initialized_here = False
        _single_node_gloo_iface()
        if dist.is_available() and dist.is_initialized():
            self.world_size = dist.get_world_size()
            self.rank = dist.get_rank()
            self.backend = dist.get_backend()
        elif int(os.environ.get("WORLD_SIZE", "1")) > 1:
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl" and device is not None and device.type == "cuda":
                kw["device_id"] = device
            dist.init_process_group(backend=backend, timeout=timedelta(seconds=int(os.environ.get("FDX_DIST_TIMEOUT", "600"))), **kw)
            self.initialized_here = True
            self.world_size = dist.get_world_size()
            self.rank = dist.get_rank()
            self.backend = backend
        else:
            self.world_size = 1
            self.rank = 0
            self.backend = "single"
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.stats = CollectiveStats()
        # per-collective hipEvent timing is opt-in (FDX_COMM_TIMING=1): two events and list
        # bookkeeping around every collective of a timed fit otherwise; counts and
        # bytes are always kept
        self._timing = os.environ.get("FDX_COMM_TIMING", "0") == "1"
        self.trace = [] if os.environ.get("FDX_COMM_TRACE", "0") == "1" else None
        self._native = None
        self._shm = None  # host-staged sums over shared memory (lazy, collective; False: off)
        mode = os.environ.get("FDX_COMM", "auto")  # auto | rccl | torch
        if self.world_size > 1 and self.backend == "nccl" and mode in ("auto", "rccl") and torch.cuda.is_available():
            self._native = self._try_native(strict=(mode == "rccl"))
        # CPU gloo group for host-int exchanges (created collectively: every rank, same point)
        self._host_pg = None
        hp = os.environ.get("FDX_HOST_PG", "1")  # 1 (nccl only) | 0 | force (also under gloo: tests)
        if self.world_size > 1 and ((self.backend != "gloo" and hp == "1") or hp == "force"):
            try:
                self._host_pg = dist.new_group(backend="gloo")
            except Exception as e:  # noqa: BLE001 - no gloo transport: host values ride the device PG
                import logging

                logging.getLogger(__name__).warning("CPU gloo group unavailable (%s): host exchanges use %s",
                                                    e, self.backend)
                self._host_pg = None

    def _try_native(self, strict: bool):
        """Bring up the native RCCL communicator and verify it with a known all-reduce; every
        rank must pass, otherwise all ranks keep using the ProcessGroup (collective decision)."""
        dev = torch.device("cuda", torch.cuda.current_device())

        def agree(ok: int) -> bool:
            flag = torch.tensor([ok], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            return int(flag.item()) == 1

        # 1) every rank can load the module -- agreed BEFORE the collective init, so a rank that
        #    fails early can never leave the others blocked inside ncclCommInitRank
        try:
            from .rccl import NativeRCCL, available

            ok = int(available())
        except Exception:  # noqa: BLE001
            if strict:
                raise
            ok = 0
        if not agree(ok):
            if strict:
                raise RuntimeError("native RCCL unavailable on some rank")
            return None
        # 2) init on all ranks, 3) known all-reduce, agreed again
        nat, ok = None, 1
        try:
            nat = NativeRCCL(self.rank, self.world_size, self.local_rank)
            ok = int(nat.verify())
        except Exception:  # noqa: BLE001
            if strict:
                raise
            ok = 0
        if agree(ok):
            return nat
        if nat is not None:
            nat.close()
        if strict:
            raise RuntimeError("native RCCL verification failed on some rank")
        return None

    @property
    def native_rccl(self) -> bool:
        return self._native is not None

    # ---- instrumentation ---------------------------------------------------------------
    @contextlib.contextmanager
    def _timed(self, op: str, t: torch.Tensor | None = None, path: str = ""):
        nbytes = 0 if t is None else t.numel() * t.element_size()
        if self.trace is not None:
            self.trace.append((op, path, nbytes))
        if not self._timing or self.world_size == 1:
            yield
            if self.world_size > 1:
                self.stats.count(op, nbytes)
            return
        if t is not None and t.is_cuda and path in ("rccl", "nccl"):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            yield
            e1.record()
            self.stats.pending.append((op, nbytes, e0, e1))
            if len(self.stats.pending) > 1024:
                self.stats.resolve()
        else:
            t0 = time.perf_counter()
            yield
            self.stats._add(op, nbytes, time.perf_counter() - t0)

    def collective_summary(self) -> dict:
        return self.stats.summary()

    # ---- basic collectives -------------------------------------------------------------
    def barrier(self):
        if self.world_size > 1:
            with self._timed("barrier", None, self.backend):
                if self.backend == "nccl" and torch.cuda.is_available():
                    dist.barrier(device_ids=[torch.cuda.current_device()])
                else:
                    dist.barrier()

    def _host_staged(self, t: torch.Tensor) -> bool:
        # gloo moves CUDA tensors through host memory (tests run several ranks on one GPU)
        return self.backend == "gloo" and t.is_cuda

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world_size == 1:
            return t
        if self._native is not None and t.is_cuda and op == "sum":
            path = "rccl"
        elif self._host_staged(t):
            path = "gloo-staged"
        else:
            path = self.backend
        with self._timed(f"all_reduce_{op}", t, path):
            if self._native is not None and t.is_cuda and op == "sum":
                self._native.all_reduce_(t)
                return t
            if self._host_staged(t):
                h = self._stage_d2h(t)
                # the shared-memory sums take numpy dtypes only (bf16 / fp16 stay on gloo: ADVICE r5)
                shm = self._shm_group() if (op == "sum" and h.dtype in _SHM_DTYPES) else None
                if shm is not None and shm.fits(h.numpy()):  # same size on every rank: same branch
                    shm.all_reduce_(h.numpy())
                else:
                    dist.all_reduce(h, op=_op(op))
                t.copy_(h)
                return t
            dist.all_reduce(t, op=_op(op))
            return t

    def _shm_group(self):
        """The shared-memory sum all-reduce of the host-staged path (parallel/shm_reduce.py), set up
        at the first staged sum -- a point every rank reaches together -- when all ranks share one
        host (torchrun's LOCAL_WORLD_SIZE == WORLD_SIZE).  FDX_COMM_SHM=0 keeps gloo."""
        if self._shm is None:
            self._shm = False
            if (os.environ.get("FDX_COMM_SHM", "1") == "1"
                    and int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == self.world_size):
                from .shm_reduce import ShmAllReduce

                cap = int(os.environ.get("FDX_COMM_SHM_BYTES", str(4 << 20)))
                tmo = float(os.environ.get("FDX_DIST_TIMEOUT", "600"))
                obj = ShmAllReduce(0, self.world_size, cap, timeout_s=tmo) if self.rank == 0 else None
                name = [obj.name if obj is not None else None]
                dist.broadcast_object_list(name, src=0)
                if obj is None:
                    obj = ShmAllReduce(self.rank, self.world_size, cap, name=name[0], timeout_s=tmo)
                self._shm = obj
        return self._shm or None

    def _stage_d2h(self, t: torch.Tensor) -> torch.Tensor:
        """Device -> host copy of a gloo-staged collective's operand into a reused pinned buffer
        (a pageable copy goes through the runtime's staging path on every call).  Timed on its own
        ("stage_d2h"): the wait for the device work that produces ``t`` shows up here, apart from
        the collective's wait for the other ranks."""
        key = (tuple(t.shape), t.dtype)
        pool = self.__dict__.setdefault("_pinned", {})
        h = pool.get(key)
        if h is None:
            h = pool[key] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        t0 = time.perf_counter()
        h.copy_(t)  # synchronous: waits for the stream's work that writes t
        if self._timing:  # stats only (not a collective: the trace does not list it)
            self.stats._add("stage_d2h", t.numel() * t.element_size(), time.perf_counter() - t0)
        return h

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        return self.all_reduce_(t.clone(), op)

    def all_reduce_scalar(self, x: float, op: str = "sum") -> float:
        if self.world_size == 1:
            return x
        if self._host_pg is not None:
            t = torch.tensor([float(x)], dtype=torch.float64)
            with self._timed(f"all_reduce_scalar_{op}", None, "gloo-host"):
                dist.all_reduce(t, op=_op(op), group=self._host_pg)
                return float(t.item())
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        with self._timed(f"all_reduce_scalar_{op}", None, self.backend):
            dist.all_reduce(t, op=_op(op))
            return float(t.item())

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            t = t.contiguous()
            with self._timed("broadcast", t, "gloo-staged" if self._host_staged(t) else self.backend):
                if self._host_staged(t):
                    h = self._stage_d2h(t)
                    dist.broadcast(h, src=src)
                    t.copy_(h)
                else:
                    dist.broadcast(t, src=src)
        return t

    def all_gather_ints(self, vals) -> list:
        """All-gather a short list of ints from every rank (one small collective + one sync)."""
        if self.world_size == 1:
            return [list(vals)]
        host = self._host_pg is not None
        dev = torch.device("cuda", torch.cuda.current_device()) if (self.backend == "nccl" and not host) \
            else torch.device("cpu")
        t = torch.tensor(list(vals), dtype=torch.int64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        if host:
            with self._timed("all_gather_ints", None, "gloo-host"):
                dist.all_gather(out, t, group=self._host_pg)
                return torch.stack(out).tolist()
        with self._timed("all_gather_ints", None, self.backend):
            dist.all_gather(out, t)
            return torch.stack(out).cpu().tolist()

    def all_gather_rows(self, x: torch.Tensor, counts: list | None = None):
        """Variable-length all-gather along dim 0 (collective C3, SMOTE minority rows).
        Returns (concatenated tensor, list of per-rank row counts).  ``counts``: the per-rank row
        counts when the caller already exchanged them (saves a collective and a host sync)."""
        if self.world_size == 1:
            return x, [x.shape[0]]
        if self._native is not None and x.is_cuda:
            if counts is None:
                counts = [int(c[0]) for c in self.all_gather_ints([x.shape[0]])]
            with self._timed("all_gather_rows", x, "rccl"):
                return self._native_gather(x, counts)
        if self._host_staged(x):
            with self._timed("all_gather_rows_staged", x, "gloo-staged"):
                return self._staged_gather(x, counts)
        with self._timed("all_gather_rows", x, self.backend):
            return self._all_gather_rows(x, counts)

    def _native_gather(self, x: torch.Tensor, counts: list):
        """C3 on the native communicator: grouped xGMI send/recv straight into the compact
        [sum(counts), ...] output on the compute stream (csrc/comm/rccl_comm.cpp all_gatherv)."""
        counts = [int(c) for c in counts]
        return self._native.all_gatherv(x.contiguous(), counts), counts

    def _staged_gather(self, x: torch.Tensor, counts: list | None):
        """gloo rehearsal of C3 for CUDA rows: one D2H copy into a padded host buffer, the gloo
        all-gather, and one H2D copy per rank straight into the compact device output -- no CPU
        tensor compute (a CPU zero-fill / cat here ran on the OpenMP pool and stalled 5-49 ms per
        call beside the other rank's threads: profiles/r4_a/dpscope.log)."""
        if counts is None:
            counts = [int(c[0]) for c in self.all_gather_ints([x.shape[0]])]
        counts = [int(c) for c in counts]
        mx = max(counts)
        pad = torch.empty((mx,) + tuple(x.shape[1:]), dtype=x.dtype)  # rows past x.shape[0] never read
        if x.shape[0]:
            pad[: x.shape[0]].copy_(x)
        outs = [torch.empty_like(pad) for _ in range(self.world_size)]
        dist.all_gather(outs, pad)
        out = torch.empty((sum(counts),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        o0 = 0
        for o, c in zip(outs, counts):
            if c:
                out[o0:o0 + c].copy_(o[:c])
            o0 += c
        return out, counts

    def _all_gather_rows(self, x: torch.Tensor, counts: list | None):
        dev = x.device
        if counts is None:
            n = torch.tensor([x.shape[0]], dtype=torch.int64, device=dev)
            cl = [torch.zeros_like(n) for _ in range(self.world_size)]
            dist.all_gather(cl, n)
            counts = [int(c.item()) for c in cl]
        counts = [int(c) for c in counts]
        mx = max(counts)
        pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
        pad[: x.shape[0]] = x
        outs = [torch.empty_like(pad) for _ in range(self.world_size)]
        dist.all_gather(outs, pad)
        return torch.cat([o[:c] for o, c in zip(outs, counts)], 0), counts

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def max_over_ranks(self, x: float) -> float:
        return self.all_reduce_scalar(x, op="max")

    def close(self):
        if self._native is not None:
            self._native.close()
            self._native = None
        if self._shm:
            self.barrier()  # no rank may still be reading the segment when the creator unlinks it
            self._shm.close()
            self._shm = None
        self._host_pg = None
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized_here = False


def _op(op: str):
    return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]


_SINGLE = None


def single() -> Communicator:
    global _SINGLE
    if _SINGLE is None:
        c = Communicator.__new__(Communicator)
        c.world_size, c.rank, c.local_rank, c.backend, c._native, c.initialized_here = 1, 0, 0, "single", None, False
        c.stats, c._timing, c.trace = CollectiveStats(), False, None
        _SINGLE = c
    return _SINGLE
