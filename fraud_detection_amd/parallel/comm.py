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
"""
from __future__ import annotations

import os
from datetime import timedelta

import torch
import torch.distributed as dist


class Communicator:
    def __init__(self, backend: str | None = None, device: torch.device | None = None):
        self.initialized_here = False
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
        self._native = None
        mode = os.environ.get("FDX_COMM", "auto")  # auto | rccl | torch
        if self.world_size > 1 and self.backend == "nccl" and mode in ("auto", "rccl") and torch.cuda.is_available():
            self._native = self._try_native(strict=(mode == "rccl"))

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

    # ---- basic collectives -------------------------------------------------------------
    def barrier(self):
        if self.world_size > 1:
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
            self._native.all_reduce_(t)
            return t
        if self._host_staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=_op(op))
            t.copy_(h)
            return t
        dist.all_reduce(t, op=_op(op))
        return t

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        return self.all_reduce_(t.clone(), op)

    def all_reduce_scalar(self, x: float, op: str = "sum") -> float:
        if self.world_size == 1:
            return x
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=_op(op))
        return float(t.item())

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            t = t.contiguous()
            if self._host_staged(t):
                h = t.cpu()
                dist.broadcast(h, src=src)
                t.copy_(h)
            else:
                dist.broadcast(t, src=src)
        return t

    def all_gather_ints(self, vals) -> list:
        """All-gather a short list of ints from every rank (one small collective + one sync)."""
        if self.world_size == 1:
            return [list(vals)]
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor(list(vals), dtype=torch.int64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t)
        return torch.stack(out).cpu().tolist()

    def all_gather_rows(self, x: torch.Tensor, counts: list | None = None):
        """Variable-length all-gather along dim 0 (collective C3, SMOTE minority rows).
        Returns (concatenated tensor, list of per-rank row counts).  ``counts``: the per-rank row
        counts when the caller already exchanged them (saves a collective and a host sync)."""
        if self.world_size == 1:
            return x, [x.shape[0]]
        if self._host_staged(x):
            out, c = self.all_gather_rows(x.cpu(), counts)
            return out.to(x.device), c
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
        _SINGLE = c
    return _SINGLE
