"""K8 k-nearest neighbours (SMOTE) and K9 SMOTE sample generation."""
from __future__ import annotations

import os

import numpy as np
import torch

from . import reference as ref
from .layout import DEFAULT_FP8_SCALE, DTYPE_KIND, NCOLS, check_rows, storage_kind
from .native import native, ptr, stream_of


def _pad32(n: int) -> int:
    return max(32, (n + 31) // 32 * 32)


def _padded(X: torch.Tensor, n_pad: int) -> torch.Tensor:
    if X.shape[0] == n_pad and X.is_contiguous():
        return X
    out = torch.zeros((n_pad, NCOLS), device=X.device, dtype=torch.float32)
    out[: X.shape[0]] = X
    return out


# Engines (all exact fp32 rankings, tests/test_kernels_gpu.py):
#   fp32    one-wave workgroups (32 queries) streaming candidate tiles from L2 / Infinity Cache
#           through a 16 x v_mfma_f32_32x32x2_f32 chain per 32x32 tile;
#   fp32lds 4-wave workgroups (128 queries) sharing double-buffered LDS-staged candidate chunks
#           (4x fewer streamed bytes, half the occupancy);
#   bf16x3  hi.hi + hi.lo + lo.hi bf16 MFMA filter (5.3x fewer MFMA cycles) + exact re-score.
#   bf16x3r the same filter with no fp32 work in the tile loop: passing candidates are appended to
#           per-lane lists under a provable lower-bound threshold, and a second kernel re-scores
#           the listed candidates exactly (8 lanes per query) -- knn.hip knn_collect_kernel.
#   b3top   the bf16x3 score with register top-8 APPROXIMATE lists (no lists in memory, no fp32 work
#           in the tile loop, seeded slices so ~6 waves fill every SIMD); one merge kernel re-scores
#           each query's 8 best exactly and proves the exact top-k from the error margin (else an
#           exact scan of that query) -- knn.hip knn_b3top_kernel.
# Measured on MI355X from 13.6k to 170k minority rows (profiles/r2_s3i/knn_engines.jsonl): fp32
# beat fp32lds (0.66-0.99x) and bf16x3 (0.86-0.96x) at every size.  bf16x3r (round 5,
# profiles/r5_k, r5_o): at the DP=8 global-scope rank (13.6k queries x 108.8k candidates) 0.78 ms
# against 1.07.  At the bench's DP=1 self-search the lab had it at 0.194 vs 0.209 ms, but inside
# the pipeline's step its collect + re-rank took 199 us against the fp32 engine's ~200 us
# (profiles/r5_x timeline): no gain.  Round 6 (profiles/r6_knn): with a quad-max pre-test in the
# append path and the pair-interleaved MFMA chains the lab has bf16x3r at 0.184 ms vs fp32's 0.217
# at DP=1, and in the pipeline's step (quick SGD benches, two runs each) 1.006 / 1.015 ms medians
# against 1.037 / 1.035.  auto = bf16x3r from 8k candidates, fp32 below; FDX_KNN selects an engine.
KNN_BF16X3_MIN_CANDIDATES = 1 << 13


def knn_engine(mq: int, mc: int, engine: str | None = None) -> str:
    e = engine or os.environ.get("FDX_KNN", "auto")
    if e == "auto":
        return "bf16x3r" if mc >= KNN_BF16X3_MIN_CANDIDATES else "fp32"
    if e not in ("fp32", "fp32lds", "bf16x3", "bf16x3r", "b3top"):
        raise ValueError(f"unknown k-NN engine {e!r}")
    return e


def _check_parents(parents: torch.Tensor | None, C: torch.Tensor, affine: torch.Tensor | None) -> int:
    if parents is None:
        if affine is not None:
            raise ValueError("parents_affine without parents")
        return 0
    if parents.dtype != torch.bfloat16 or tuple(parents.shape) != (C.shape[0], NCOLS) or \
            not parents.is_contiguous() or parents.device != C.device:
        raise ValueError("parents must be a contiguous bf16 [mc, 32] tensor on C's device")
    if affine is not None and (affine.dtype != torch.float64 or affine.numel() < 64 or affine.device != C.device):
        raise ValueError("parents_affine must be ScalerStats.aff (float64 [64]) on C's device")
    return ptr(parents)


def knn_topk(Q: torch.Tensor, C: torch.Tensor, k: int = 5, self_offset: int = -1, want_dist: bool = False,
             nsplit: int | None = None, engine: str | None = None, parents: torch.Tensor | None = None,
             parents_affine: torch.Tensor | None = None, _diag: dict | None = None):
    """k nearest candidates (squared L2 over the 30 feature columns) of each query row.

    Q [mq, 32] / C [mc, 32] fp32 padded rows (columns 30/31, intercept and label, are ignored).  If ``self_offset >= 0``, query row q is candidate
    row ``self_offset + q`` and is excluded (SMOTE's self-match removal).  Returns int32 [mq, k]
    (ascending distance, ties -> smaller index) and optionally squared distances.
    ``nsplit``: candidate slices searched by separate workgroups and merged (None = auto).
    ``engine``: "fp32" = exact fp32 MFMA chain over every candidate (16 x 32x32x2 f32 per tile);
    "bf16x3" = hi.hi + hi.lo + lo.hi bf16 MFMA filter (6 x 32x32x16 bf16 per tile) with a provable
    margin and exact fp32 re-scoring of the survivors; None/"auto" (FDX_KNN env) picks by size.
    Both return the exact fp32 ranking.
    ``parents`` (bf16 [mc, 32], optional): also filled with ``smote_parents(C, parents_affine)``
    by the operand-prep launch that already reads C (one launch fewer on the SMOTE path).
    """
    for t, nm in ((Q, "Q"), (C, "C")):
        if t.dim() != 2 or t.shape[1] != NCOLS or t.dtype != torch.float32:
            raise ValueError(f"{nm} must be fp32 [m, 32]")
    mq, mc = Q.shape[0], C.shape[0]
    if not 1 <= k <= 8:
        raise ValueError("k must be in [1, 8]")
    n_valid = mc - (1 if self_offset >= 0 else 0)
    if n_valid < k:
        raise ValueError(f"need at least k={k} candidates besides self, have {n_valid}")
    if self_offset >= 0 and self_offset + mq > mc:
        raise ValueError("self_offset + mq exceeds the candidate set")
    if not Q.is_cuda:
        if _check_parents(parents, C, parents_affine):
            parents.copy_(smote_parents(C, parents_affine))
        idx, d2 = ref.knn_topk(Q.numpy(), C.numpy(), k, self_offset)
        idx_t = torch.from_numpy(idx)
        return (idx_t, torch.from_numpy(d2.astype(np.float32))) if want_dist else idx_t
    m = native()
    s = stream_of(Q)
    eng = knn_engine(mq, mc, engine)
    mq_pad, mc_pad = _pad32(mq), _pad32(mc)
    if eng == "fp32lds":
        mq_pad = (mq_pad + 127) // 128 * 128  # 4 query blocks of 32 per workgroup
    Qc, Cc = Q.contiguous(), C.contiguous()
    # GEMM-ready rows: the -0.5||c||^2 term rides in column 30 (see knn.hip knn_prep_kernel)
    Qp = torch.empty((mq_pad, NCOLS), device=Q.device, dtype=torch.float32)
    Cp = torch.empty((mc_pad, NCOLS), device=C.device, dtype=torch.float32)
    pp = _check_parents(parents, Cc, parents_affine)
    self_search = Qc.data_ptr() == Cc.data_ptr() and mq == mc and mq_pad == mc_pad
    split_done = False
    if eng in ("bf16x3r", "b3top"):  # their hi/lo bf16 operands (+ per-tile candidate norm bound)
        Qhl = torch.empty((mq_pad, 64), device=Q.device, dtype=torch.bfloat16)
        Chl = torch.empty((mc_pad, 64), device=C.device, dtype=torch.bfloat16)
        tmax = torch.empty(mc_pad // 32, device=C.device, dtype=torch.float32)
    if self_search:
        # SMOTE self-search: one launch reads the rows once and writes both operands (+ parents, and
        # for the bf16x3 engines that stream candidate tiles, their hi/lo split)
        fuse = eng in ("bf16x3r", "b3top")
        m.knn_prep(ptr(Cc), mc, mc_pad, 2, ptr(Cp), s, ptr(Qp), ptr(parents_affine), pp,
                   ptr(Chl) if fuse else 0, ptr(Qhl) if fuse else 0, ptr(tmax) if fuse else 0)
        split_done = fuse
    else:
        m.knn_prep(ptr(Cc), mc, mc_pad, 0, ptr(Cp), s, 0, ptr(parents_affine), pp)
        m.knn_prep(ptr(Qc), mq, mq_pad, 1, ptr(Qp), s)
    idx = torch.empty((mq, k), device=Q.device, dtype=torch.int32)
    score = torch.empty((mq, k), device=Q.device, dtype=torch.float32) if want_dist else None
    if nsplit is not None:
        ns = max(1, int(nsplit))
    else:
        ns = {"fp32": m.knn_splits, "fp32lds": m.knn_lds_splits, "bf16x3": m.knn3_splits,
              "bf16x3r": m.knn3r_splits, "b3top": m.knn_b3top_splits}[eng](mq_pad, mc_pad)
    ws_s = ws_i = None
    if ns > 1 and eng not in ("bf16x3r", "b3top"):
        ws_s = torch.empty((ns, mq, k), device=Q.device, dtype=torch.float32)
        ws_i = torch.empty((ns, mq, k), device=Q.device, dtype=torch.int32)
    if eng == "fp32":
        m.knn_topk(ptr(Qp), mq_pad, mq, ptr(Cp), mc_pad, mc, int(self_offset), int(k), ptr(idx),
                   ptr(score), ptr(ws_s), ptr(ws_i), ns, s)
    elif eng == "fp32lds":
        m.knn_topk_lds(ptr(Qp), mq_pad, mq, ptr(Cp), mc_pad, mc, int(self_offset), int(k), ptr(idx),
                       ptr(score), ptr(ws_s), ptr(ws_i), ns, s)
    elif not split_done:
        # hi/lo bf16 split of both operands (+ per-tile candidate norm bound) for the filter
        if eng == "bf16x3":
            Qhl = torch.empty((mq_pad, 64), device=Q.device, dtype=torch.bfloat16)
            Chl = torch.empty((mc_pad, 64), device=C.device, dtype=torch.bfloat16)
            tmax = torch.empty(mc_pad // 32, device=C.device, dtype=torch.float32)
        # 2: fragment order (b3top and the bf16x3r collect stream candidate tiles; bf16x3 reads rows)
        m.knn_split(ptr(Cp), mc_pad, 2 if eng in ("b3top", "bf16x3r") else 0, ptr(Chl), ptr(tmax), s)
        m.knn_split(ptr(Qp), mq_pad, 1, ptr(Qhl), 0, s)
    if eng == "b3top":
        ns = min(ns, 32)
        ws_s = torch.empty((ns, mq, 8), device=Q.device, dtype=torch.float32)
        ws_i = torch.empty((ns, mq, 8), device=Q.device, dtype=torch.int32)
        ws_m = torch.empty((ns, mq, 2), device=Q.device, dtype=torch.float32)
        fail = torch.empty(1 + mq, device=Q.device, dtype=torch.int32)  # count, then failed query ids
        m.knn_b3top(ptr(Qp), ptr(Qhl), mq_pad, mq, ptr(Cp), ptr(Chl), ptr(tmax), mc_pad, mc, int(self_offset),
                    int(k), ptr(idx), ptr(score), ptr(ws_s), ptr(ws_i), ptr(ws_m), ptr(fail), ns, s)
        if _diag is not None:  # queries answered by the exact scan (diagnostics; synchronises)
            _diag.update(nsplit=ns, exact_scans=int(fail[0].item()))
    elif eng == "bf16x3r":
        nb = ns * (mq_pad // 32) * 64
        lists = torch.empty(nb * m.KNN3R_LIST_CAP * 2, device=Q.device, dtype=torch.int32)  # (lb, index)
        # list lengths, then each lane's final threshold and largest margin (knn_collect_kernel)
        counts = torch.empty(3 * nb, device=Q.device, dtype=torch.int32)
        m.knn_topk3r(ptr(Qp), ptr(Qhl), mq_pad, mq, ptr(Cp), ptr(Chl), ptr(tmax), mc_pad, mc, int(self_offset),
                     int(k), ptr(idx), ptr(score), ptr(lists), ptr(counts), ns, s)
        if _diag is not None:  # list lengths (diagnostics; synchronises)
            c = counts[:nb].float()
            _diag.update(nsplit=ns, list_cap=int(m.KNN3R_LIST_CAP), mean=float(c.mean()), max=int(c.max()),
                         p99=float(torch.quantile(c[: min(c.numel(), 1 << 24)], 0.99)),
                         over_cap=int((c > m.KNN3R_LIST_CAP).sum()), counts=counts[:nb].view(ns, mq_pad // 32, 64))
    elif eng == "bf16x3":
        m.knn_topk3(ptr(Qp), ptr(Qhl), mq_pad, mq, ptr(Cp), ptr(Chl), ptr(tmax), mc_pad, mc, int(self_offset),
                    int(k), ptr(idx), ptr(score), ptr(ws_s), ptr(ws_i), ns, s)
    if want_dist:
        qn = (Q[:, :30].double() ** 2).sum(1, keepdim=True)
        return idx, (qn - 2.0 * score.double()).float()
    return idx


def smote_parents(C: torch.Tensor, affine: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [m, 32] SMOTE parents in the training rows' space: bf16(z * sigma + c) on the feature
    columns with ``affine`` (ScalerStats.aff, pivot-shifted rows), bf16(z) without; columns 30/31
    copied.  Sampling from them halves the gather bytes and drops the per-sample affine map."""
    if C.dtype != torch.float32 or C.dim() != 2 or C.shape[1] != NCOLS:
        raise ValueError("C must be fp32 [m, 32]")
    C = C.contiguous()
    if not C.is_cuda:
        v = C.numpy().copy()
        if affine is not None:
            a = affine.cpu().numpy()
            v[:, :30] = (v[:, :30] * (1.0 / a[32:62]).astype(np.float32)) + a[:30].astype(np.float32)
        return torch.from_numpy(v).to(torch.bfloat16)
    P = torch.empty((C.shape[0], NCOLS), dtype=torch.bfloat16, device=C.device)
    native().smote_parents(ptr(C), C.shape[0], ptr(affine), ptr(P), stream_of(C))
    return P


def smote_generate(C: torch.Tensor, nbr: torch.Tensor, q_offset: int, n_new: int, out: torch.Tensor,
                   seed: int = 42, counter_base: int = 0, label: float = 1.0,
                   fp8_scale: float = DEFAULT_FP8_SCALE, affine: torch.Tensor | None = None,
                   sample_offset: int = 0) -> torch.Tensor:
    """Write ``n_new`` synthetic rows into ``out`` (a [n_new, 32] bf16/fp32/fp8 view, e.g. the tail of
    the training buffer).  Sample s interpolates minority row (q_offset + i) toward neighbour
    nbr[i, kk] with Philox draws keyed by (seed, s, counter_base).  C: fp32 standardized parents,
    or bf16 parents from smote_parents (already in the output space; ``affine`` must be None).
    ``affine`` ([64] float64, ScalerStats.aff) with fp32 parents: ``out`` holds pivot-shifted rows
    -- each feature is written as z * sigma + c.  ``sample_offset`` (multiple of 128): these are
    samples [sample_offset, sample_offset + n_new) of one global draw sequence (DP ranks)."""
    if C.dtype not in (torch.float32, torch.bfloat16) or C.dim() != 2 or C.shape[1] != NCOLS:
        raise ValueError("C must be fp32 or bf16 [m, 32]")
    pb = C.dtype == torch.bfloat16
    if pb and affine is not None:
        raise ValueError("bf16 parents are already in the output space (smote_parents): no affine")
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError("nbr must be int32 [mq, k]")
    mq, k = nbr.shape
    if q_offset < 0 or q_offset + mq > C.shape[0]:
        raise ValueError("query rows out of range of C")
    ref.smote_check_ranges(C.shape[0], mq, k)
    if sample_offset < 0 or sample_offset % 128:
        raise ValueError("sample_offset must be a non-negative multiple of 128")
    check_rows(out, "out")
    if out.shape[0] != n_new:
        raise ValueError("out must have n_new rows")
    kind = storage_kind(out)
    if n_new == 0:
        return out
    if not C.is_cuda:
        nb = nbr.numpy()
        if nb.min() < 0 or nb.max() >= C.shape[0]:
            raise ValueError("neighbour index out of range")
        rows = ref.smote_generate(C.float().numpy(), nb, q_offset, n_new, seed, counter_base, label,
                                  sample_offset=sample_offset)
        if affine is not None:
            a = affine.cpu().numpy()
            sig = (1.0 / a[32:62]).astype(np.float32)
            rows[:, :30] = rows[:, :30] * sig + a[:30].astype(np.float32)
        if kind == "bf16":
            out.copy_(torch.from_numpy(rows).to(torch.bfloat16))
        elif kind == "f32":
            out.copy_(torch.from_numpy(rows))
        else:
            r2 = rows.copy()
            r2[:, :30] *= fp8_scale
            out.copy_(torch.from_numpy(ref.fp8_encode(r2)))
        return out
    m = native()
    m.smote_generate(ptr(C), int(pb), ptr(nbr), mq, k, int(q_offset), int(n_new), int(sample_offset),
                     int(seed) & (2**64 - 1),
                     int(counter_base) & (2**64 - 1), float(label), DTYPE_KIND[kind], float(fp8_scale),
                     ptr(affine), ptr(out), stream_of(C))
    return out
