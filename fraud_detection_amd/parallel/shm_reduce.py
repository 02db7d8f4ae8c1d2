"""Sum all-reduce of small host vectors among the ranks of ONE host through shared memory.

The host-staged gloo path of a single-host job (the one-GPU multi-process rehearsal, whose CUDA
tensors are staged through host memory; CPU-tensor collectives go straight to gloo and do not come
here, nor do dtypes numpy lacks, e.g. bf16) pays a TCP-loopback round trip per collective: ~200 us
for a 1.1 KB SGD step vector in `profiles/r5_ze` -- 24 of them per SGD fit.  Here every rank
writes its vector into its own slot of a shared segment and publishes a sequence number; each rank
then sums the W slots itself in rank order (the same fixed order on every rank, so every rank gets
bitwise the same result, and int64 fixed-point sums stay exact) and acknowledges.  Two slot sets
alternate by sequence parity, so a rank only waits for the others' acknowledgement of the
collective before the previous one.

Ordering relies on x86-64's total store order (a rank's data stores are visible before its
sequence store; a reader's sequence load precedes its data loads; loads are not reordered with
later stores) -- the container and the GPU boxes are x86-64.  A rank that stops participating
(killed, hung) makes the others raise after ``timeout_s`` instead of waiting forever.

Multi-GPU jobs on RCCL never come here (parallel/comm.py uses this only for host-staged gloo
collectives of ranks that share a host).
"""
from __future__ import annotations

import time
import uuid

import numpy as np

_CTRL = 16  # int64 words per rank: [0] published sequence, [1] acknowledged sequence


class ShmAllReduce:
    def __init__(self, rank: int, world: int, cap_bytes: int, name: str | None = None,
                 timeout_s: float = 600.0):
        from multiprocessing import resource_tracker, shared_memory

        self.rank, self.world, self.cap = int(rank), int(world), int(cap_bytes + 63) // 64 * 64
        self.timeout_s = float(timeout_s)
        size = self.world * _CTRL * 8 + 2 * self.world * self.cap
        if name is None:  # the creator (rank 0)
            self.shm = shared_memory.SharedMemory(name=f"fdx_ar_{uuid.uuid4().hex[:16]}", create=True, size=size)
            self.owner = True
            np.frombuffer(self.shm.buf, dtype=np.int64, count=self.world * _CTRL)[:] = 0
        else:
            self.shm = shared_memory.SharedMemory(name=name, create=False)
            self.owner = False
            # Python < 3.13 registers an attached segment with this process's resource tracker,
            # which would unlink it when THIS process exits; only the creator owns it
            try:
                resource_tracker.unregister(self.shm._name, "shared_memory")  # noqa: SLF001
            except Exception:  # noqa: BLE001
                pass
        self.name = self.shm.name
        self.ctrl = np.frombuffer(self.shm.buf, dtype=np.int64, count=self.world * _CTRL).reshape(self.world, _CTRL)
        self._data_off = self.world * _CTRL * 8
        self.seq = 0

    def _slot(self, par: int, r: int, dtype, count: int) -> np.ndarray:
        off = self._data_off + (par * self.world + r) * self.cap
        return np.frombuffer(self.shm.buf, dtype=dtype, count=count, offset=off)

    def _wait(self, col: int, target: int):
        c = self.ctrl[:, col]
        spins = 0
        t0 = None
        while int(c.min()) < target:
            spins += 1
            if spins > 2000:
                if t0 is None:
                    t0 = time.monotonic()
                elif time.monotonic() - t0 > self.timeout_s:
                    raise RuntimeError(f"shm all-reduce: a rank stopped participating (waited {self.timeout_s:.0f} s "
                                       f"for sequence {target})")
                time.sleep(0)  # yield: another rank may share this CPU

    def fits(self, a: np.ndarray) -> bool:
        return a.nbytes <= self.cap

    def all_reduce_(self, a: np.ndarray) -> np.ndarray:
        """In place: a = sum over ranks of a (every rank calls with the same shape and dtype)."""
        if a.nbytes > self.cap:
            raise ValueError(f"shm all-reduce: {a.nbytes} bytes > capacity {self.cap}")
        flat = a.reshape(-1)
        s = self.seq + 1
        par = s & 1
        if s > 2:
            self._wait(1, s - 2)  # every rank has read this parity's previous contents
        self._slot(par, self.rank, flat.dtype, flat.size)[:] = flat
        self.ctrl[self.rank, 0] = s  # publish after the data (TSO: stores stay in order)
        self._wait(0, s)
        acc = self._slot(par, 0, flat.dtype, flat.size).copy()
        for r in range(1, self.world):  # fixed rank order on every rank
            acc += self._slot(par, r, flat.dtype, flat.size)
        self.ctrl[self.rank, 1] = s  # done reading (loads are not reordered with later stores)
        flat[:] = acc
        self.seq = s
        return a

    def close(self):
        try:
            del self.ctrl
            self.shm.close()
            if self.owner:
                self.shm.unlink()
        except Exception:  # noqa: BLE001
            pass
