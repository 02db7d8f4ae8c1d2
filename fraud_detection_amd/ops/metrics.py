"""K10 exact ROC-AUC and confusion counts."""
from __future__ import annotations

import numpy as np
import torch

from . import reference as ref
from .native import native, ptr, stream_of

_CHUNK = 16384


def _check(scores: torch.Tensor, labels: torch.Tensor):
    if scores.dtype != torch.float32 or scores.dim() != 1:
        raise ValueError("scores must be 1-D float32")
    if labels.dtype != torch.uint8 or labels.shape != scores.shape:
        raise ValueError("labels must be uint8 aligned with scores")


def auc_pair_counts(scores: torch.Tensor, labels: torch.Tensor):
    """(twice_pairs, P, N): twice_pairs = 2 #{s_p > s_n} + #{s_p == s_n}.  Exact integers, so
    data-parallel shards combine by all-gathering positives (see parallel/dp.py)."""
    _check(scores, labels)
    n = scores.shape[0]
    if not scores.is_cuda:
        y = labels.numpy().astype(bool)
        P, N = int(y.sum()), int(n - y.sum())
        auc = ref.roc_auc(scores.numpy(), y) if P and N else float("nan")
        return (int(round(auc * 2 * P * N)) if P and N else 0), P, N
    m = native()
    s = stream_of(scores)
    counter = torch.zeros(1, device=scores.device, dtype=torch.int64)
    pos = torch.empty(max(n, 1), device=scores.device, dtype=torch.float32)
    m.auc_compact(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), s)
    P = int(counter.item())
    N = n - P
    if P == 0 or N == 0:
        return 0, P, N
    nchunks = (P + _CHUNK - 1) // _CHUNK
    m.sort_chunks(ptr(pos), n, ptr(counter), _CHUNK, nchunks, s)
    out = torch.zeros(1, device=scores.device, dtype=torch.int64)
    m.auc_count(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), _CHUNK, nchunks, ptr(out), s)
    return int(out.item()), P, N


def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """Exact ROC-AUC (ties averaged), equal to sklearn.metrics.roc_auc_score."""
    twice, P, N = auc_pair_counts(scores, labels)
    if P == 0 or N == 0:
        return float("nan")
    return twice / (2.0 * P * N)


def confusion_counts(scores: torch.Tensor, labels: torch.Tensor, threshold: float = 0.0) -> np.ndarray:
    """[tn, fp, fn, tp] with prediction = score > threshold (threshold 0 on logits == p > 0.5)."""
    _check(scores, labels)
    if not scores.is_cuda:
        return ref.confusion(scores.numpy(), labels.numpy(), threshold)
    m = native()
    out = torch.zeros(4, device=scores.device, dtype=torch.int64)
    m.confusion(ptr(scores), ptr(labels), scores.shape[0], float(threshold), ptr(out), stream_of(scores))
    return out.cpu().numpy()
