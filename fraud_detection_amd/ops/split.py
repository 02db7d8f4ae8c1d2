"""K3 stratified train/test split + K-fold assignment (csrc/kernels/split.hip).

Reference: ``train_test_split(stratify=y, test_size=0.2, random_state=42)`` followed by
``StratifiedKFold(5, shuffle=True, random_state=42)`` on the train part (train_model.py:31-33,
49,58).  The device version keeps the contract -- per-class shuffles, a round(frac * n_c) test
share per class, K folds per class whose sizes differ by at most one -- but draws the shuffle
from a keyed Feistel permutation instead of numpy's Mersenne Twister, so it needs no sort and
no host round trip.  ``data/io.py`` keeps the sklearn-identical split for reference-exact runs;
``train.py --split device`` (auto for large tables on a GPU) uses this one.

Codes: 255 = test, 0..K-1 = CV fold of a train row.  ``assign_numpy`` is the bit-identical oracle.
"""
from __future__ import annotations

import numpy as np
import torch

from .native import native, ptr, stream_of

TEST = 255


def _fmix32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x85EBCA6B)
    x ^= x >> np.uint32(13)
    x *= np.uint32(0xC2B2AE35)
    x ^= x >> np.uint32(16)
    return x


def _class_codes(rank: np.ndarray, n_c: int, seed: int, cls: int, test_frac: float, k: int) -> np.ndarray:
    ntest = min(int(np.floor(test_frac * float(n_c) + 0.5)), n_c)
    m = n_c - ntest
    kk = k if k > 1 else 1
    q, r = m // kk, m % kk
    b = 2
    while b < 64 and (1 << b) < n_c:
        b += 1
    h = (b + 1) >> 1
    mask = np.uint64((1 << h) - 1)
    with np.errstate(over="ignore"):
        keys = [int(_fmix32(np.uint32(seed) ^ _fmix32(np.uint32((0x9E3779B9 * (2 * cls + 1) + i) & 0xFFFFFFFF))))
                for i in range(4)]
        x = rank.astype(np.uint64)
        todo = np.ones(x.shape, bool)
        while todo.any():
            xs = x[todo]
            L, R = xs >> np.uint64(h), xs & mask
            for kv in keys:
                f = _fmix32((R ^ np.uint64(kv)).astype(np.uint32)).astype(np.uint64) & mask
                L, R = R, L ^ f
            xs = (L << np.uint64(h)) | R
            x[todo] = xs
            todo[todo] = xs >= np.uint64(n_c)
    pos = x.astype(np.int64)
    out = np.full(pos.shape, TEST, np.uint8)
    tr = pos >= ntest
    if k <= 1:
        out[tr] = 0
        return out
    p = pos[tr] - ntest
    big = r * (q + 1)
    out[tr] = np.where(p < big, p // (q + 1), r + (p - big) // max(q, 1)).astype(np.uint8)
    return out


def assign_numpy(labels: np.ndarray, test_frac: float = 0.2, n_folds: int = 5, seed: int = 42) -> np.ndarray:
    """Oracle of the device kernel (same permutation, same codes)."""
    y = np.asarray(labels).astype(np.uint8).reshape(-1)
    pos = y == 1
    out = np.empty(y.shape[0], np.uint8)
    for cls, sel in ((0, ~pos), (1, pos)):
        n_c = int(sel.sum())
        if n_c:
            out[sel] = _class_codes(np.arange(n_c), n_c, seed, cls, test_frac, n_folds)
    return out


def assign(labels: torch.Tensor, test_frac: float = 0.2, n_folds: int = 5, seed: int = 42,
           nblocks: int = 512) -> torch.Tensor:
    """Per-row codes (uint8): 255 = test, 0..n_folds-1 = fold.  Device: 3 kernels, no host sync."""
    if labels.dim() != 1:
        raise ValueError("labels must be 1-D")
    if not 0 <= n_folds <= 254:
        raise ValueError("0 <= n_folds <= 254")
    if not 0.0 <= test_frac <= 1.0:
        raise ValueError("test_frac must be in [0, 1]")
    y = labels.to(torch.uint8) if labels.dtype != torch.uint8 else labels
    if not y.is_cuda:
        return torch.from_numpy(assign_numpy(y.numpy(), test_frac, n_folds, seed))
    if y.data_ptr() % 16:
        y = y.clone()
    n = y.shape[0]
    m = native()
    s = stream_of(y)
    nb = int(max(1, min(nblocks, (n + 255) // 256)))
    counts = torch.empty(nb, device=y.device, dtype=torch.int64)
    total = torch.empty(1, device=y.device, dtype=torch.int64)
    out = torch.empty(n, device=y.device, dtype=torch.uint8)
    if n == 0:
        return out
    m.compact_count(ptr(y), n, 1, ptr(counts), nb, s)
    m.exclusive_scan_small(ptr(counts), nb, ptr(total), s)
    m.strat_assign(ptr(y), n, ptr(counts), ptr(total), int(seed) & 0xFFFFFFFF, float(test_frac), int(n_folds),
                   ptr(out), nb, s)
    return out


def split_indices(codes: torch.Tensor, n_folds: int):
    """(train_idx, test_idx, [(fold_train_idx, fold_val_idx)] * n_folds) as int64 row indices of
    the full table, all in ascending row order."""
    ar = torch.arange(codes.shape[0], device=codes.device)
    test = ar[codes == TEST]
    train = ar[codes != TEST]
    folds = []
    for f in range(n_folds if n_folds > 1 else 0):
        folds.append((ar[(codes != f) & (codes != TEST)], ar[codes == f]))
    return train, test, folds


__all__ = ["TEST", "assign", "assign_numpy", "split_indices"]
