"""HBM planner: size a fit to the device memory actually free (SURVEY.md §5.7 "long row axis",
BASELINE config 5 "288 GB HBM per-GPU minibatch sizing").

The reference loads everything into host memory (preprocess.py:32-49, train_model.py:22).  Here a
rank's raw shard is fp32 [n, 30] (120 B/row) and the training rows are 64 B (bf16) or 32 B (fp8)
plus SMOTE's synthetic rows, so three regimes exist:

  * ``resident``   -- raw shard + training rows + workspaces fit in the budget: upload once, the
                      fused one-read scaler+cast pass (the fast path; 10-100M rows on MI355X);
  * ``stream_raw`` -- only the training rows fit: the raw shard stays in host memory and is
                      streamed through two pinned staging buffers (pass 1: exact fp64 statistics,
                      pass 2: standardize+cast into the device-resident rows), H2D copies on a
                      side stream overlapped with the previous chunk's kernels;
  * infeasible     -- the training rows themselves exceed the budget: raise with the numbers (a
                      rank count or fp8 storage that makes it fit is reported).

The budget is the device's free memory (hipMemGetInfo) minus a reserve, or ``FDX_HBM_BUDGET``
(bytes) / ``budget=`` to plan as if the device were smaller (tests exercise streaming that way).
``sgd_batch_rows`` is the largest power-of-two minibatch whose per-step traffic stays within 1/64
of the budget (bounded by the shard); the SGD solver clips its configured minibatch to it.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

ROW_BYTES = {"bf16": 64, "fp8": 32, "f32": 128}
RESERVE_FRAC = 0.08          # allocator slack, RCCL buffers, other tenants
RESERVE_MIN = 1 << 30


@dataclass
class HbmPlan:
    mode: str                 # resident | stream_raw
    budget: int               # bytes usable by this fit
    n_rows: int
    d: int
    storage: str
    raw_bytes: int            # fp32 raw shard on device (resident mode)
    rows_bytes: int           # training buffer incl. SMOTE capacity
    work_bytes: int           # minority rows, k-NN, solver workspaces
    chunk_rows: int           # streaming chunk (stream_raw)
    sgd_batch_rows: int

    @property
    def device_bytes(self) -> int:
        return self.rows_bytes + self.work_bytes + (self.raw_bytes if self.mode == "resident" else
                                                     2 * self.chunk_rows * (4 * self.d + 1))

    def as_dict(self) -> dict:
        return dict(mode=self.mode, budget=self.budget, n_rows=self.n_rows, storage=self.storage,
                    device_bytes=self.device_bytes, raw_bytes=self.raw_bytes, rows_bytes=self.rows_bytes,
                    chunk_rows=self.chunk_rows, sgd_batch_rows=self.sgd_batch_rows)


def free_bytes(dev: torch.device) -> tuple[int, int]:
    """(free, total) device bytes; CPU devices report host-sized numbers (planning only)."""
    if dev.type == "cuda":
        free, total = torch.cuda.mem_get_info(dev)
        return int(free), int(total)
    import psutil

    vm = psutil.virtual_memory()
    return int(vm.available), int(vm.total)


def budget_for(dev: torch.device, budget: int | None = None) -> int:
    if budget is None and os.environ.get("FDX_HBM_BUDGET"):
        budget = int(float(os.environ["FDX_HBM_BUDGET"]))
    if budget is not None:
        return int(budget)
    free, total = free_bytes(dev)
    return max(0, free - max(RESERVE_MIN, int(RESERVE_FRAC * total)))


def plan_fit(n_rows: int, d: int, storage: str = "bf16", smote: bool = True, sampling_ratio: float = 1.0,
             minority_frac: float = 0.02, dev: torch.device | str = "cpu", budget: int | None = None,
             chunk_rows: int | None = None) -> HbmPlan:
    dev = torch.device(dev)
    B = budget_for(dev, budget)
    rb = ROW_BYTES[storage]
    cap = n_rows + (int(n_rows * max(sampling_ratio, 1.0)) + 128 if smote else 0)
    rows_bytes = cap * rb
    n_min = int(n_rows * minority_frac) + 1
    # fp32 minority rows (+ gathered copy), k-NN scratch, solver workspace (~16 MB), labels
    work = 3 * n_min * 128 + n_rows + (16 << 20)
    raw = n_rows * 4 * d
    if raw + rows_bytes + work <= B:
        mode, chunk = "resident", 0
    else:
        mode = "stream_raw"
        left = B - rows_bytes - work
        per_row = 2 * (4 * d + 1)          # two staging slots: fp32 row + label
        if left < per_row * 4096:
            need = rows_bytes + work + per_row * 4096
            need8 = cap * ROW_BYTES["fp8"] + work + per_row * 4096
            alt = "" if storage == "fp8" else f"; fp8 rows would need {need8 / 2**30:.2f} GiB"
            raise MemoryError(f"training rows alone need {need / 2**30:.2f} GiB > budget {B / 2**30:.2f} GiB"
                              f" for {n_rows} rows ({storage}){alt}: shard over more ranks")
        chunk = chunk_rows or min(1 << 22, max(4096, (left // per_row) // 4096 * 4096))
    sgd = 1 << 22
    while sgd * 2 <= min(cap, 1 << 26) and sgd * 2 * 64 <= B // 64:
        sgd *= 2
    return HbmPlan(mode, B, n_rows, d, storage, raw, rows_bytes, work, int(chunk), int(min(sgd, max(cap, 1))))


def observe_hbm(dev: torch.device) -> int:
    """fdx_hbm_used_bytes <- device memory in use (torch's allocator, which also holds every
    buffer of the native kernels)."""
    used = int(torch.cuda.memory_allocated(dev)) if dev.type == "cuda" else 0
    try:
        from ..obs.metrics import train_metrics

        train_metrics().hbm_used_bytes.set(used)
    except Exception:  # noqa: BLE001
        pass
    return used
