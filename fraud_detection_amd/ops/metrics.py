"""K10 exact ROC-AUC and confusion counts."""
from __future__ import annotations

import numpy as np
import torch

from . import reference as ref
from .native import native, ptr, stream_of

_CHUNK = 16384
# above this many positives the sorted-positive-chunk count (~N log(chunk) per 16384 positives)
# loses to the native radix sort + one counting pass
SORT_PATH_POSITIVES = 100_000
# from this many scores on, the radix path runs straight away (no positive-count read-back)
RADIX_ROWS = 8_000_000


def _radix_ws(dev, nbytes: int) -> torch.Tensor:
    """Sort scratch from the caching allocator, per call: its block is stream-ordered, so two AUC
    calls on different streams or threads never share keys / labels / counters (a module-level
    buffer reused by every call raced between concurrent evaluations -- ADVICE r3)."""
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)


def auc_radix(scores: torch.Tensor, labels: torch.Tensor):
    """Exact AUC on device with no host synchronisation: native stable LSD radix sort of
    (score key, label) + one counting pass (csrc/kernels/auc.hip).  Returns (auc float64 0-dim
    device tensor, int64 [3] device tensor = (twice_pairs, P, N))."""
    _check(scores, labels)
    n = scores.shape[0]
    m = native()
    dev = scores.device
    ws = _radix_ws(dev, int(m.auc_radix_workspace_bytes(n)))
    res = torch.empty(3, dtype=torch.int64, device=dev)
    auc = torch.empty((), dtype=torch.float64, device=dev)
    m.auc_radix(ptr(scores), ptr(labels), n, ptr(ws), ptr(res), ptr(auc), stream_of(scores))
    return auc, res


def auc_known_positives(scores: torch.Tensor, labels: torch.Tensor, n_pos: int):
    """Exact AUC on device with no host synchronisation when the caller knows the positive count
    (e.g. a CV fold, whose class counts the fold assignment already produced): the positives are
    compacted and chunk-sorted in LDS and every score counts the positives below it by binary search
    (~N log P) -- a handful of kernels instead of the 5-pass radix sort.  Returns (auc float64 0-dim
    device tensor, twice_pairs int64 0-dim device tensor)."""
    _check(scores, labels)
    n = scores.shape[0]
    P = int(n_pos)
    N = n - P
    dev = scores.device
    if P <= 0 or N <= 0:
        return torch.full((), float("nan"), dtype=torch.float64, device=dev), torch.zeros((), dtype=torch.int64, device=dev)
    if P > SORT_PATH_POSITIVES:
        auc, res = auc_radix(scores, labels)
        return auc, res[0]
    m = native()
    s = stream_of(scores)
    counter = torch.zeros(1, device=dev, dtype=torch.int64)
    pos = torch.empty(max(n, 1), device=dev, dtype=torch.float32)
    m.auc_compact(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), s)
    # the smallest power-of-two chunk that holds the positives: the one-block bitonic sort's
    # stages and the count's LDS fill scale with it (a fixed 16384 for ~3.4k fold positives cost
    # more than the radix path it replaced)
    chunk = min(_CHUNK, max(64, 1 << (P - 1).bit_length()))
    nchunks = (P + chunk - 1) // chunk
    m.sort_chunks(ptr(pos), n, ptr(counter), chunk, nchunks, s)
    out = torch.zeros(1, device=dev, dtype=torch.int64)
    m.auc_count(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), chunk, nchunks, ptr(out), s)
    twice = out[0]
    return twice.double() / (2.0 * P * N), twice


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
    if n >= RADIX_ROWS:
        _, res = auc_radix(scores, labels)
        twice, P, N = (int(v) for v in res.cpu())
        return twice, P, N
    m = native()
    s = stream_of(scores)
    counter = torch.zeros(1, device=scores.device, dtype=torch.int64)
    pos = torch.empty(max(n, 1), device=scores.device, dtype=torch.float32)
    m.auc_compact(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), s)
    P = int(counter.item())
    N = n - P
    if P == 0 or N == 0:
        return 0, P, N
    if min(P, N) > SORT_PATH_POSITIVES:
        _, res = auc_radix(scores, labels)
        return int(res[0].item()), P, N
    nchunks = (P + _CHUNK - 1) // _CHUNK
    m.sort_chunks(ptr(pos), n, ptr(counter), _CHUNK, nchunks, s)
    out = torch.zeros(1, device=scores.device, dtype=torch.int64)
    m.auc_count(ptr(scores), ptr(labels), n, ptr(pos), ptr(counter), _CHUNK, nchunks, ptr(out), s)
    return int(out.item()), P, N


def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """Exact ROC-AUC (ties averaged), equal to sklearn.metrics.roc_auc_score.  Large inputs on a
    GPU take the sync-free radix path and read the result once."""
    if scores.is_cuda and scores.shape[0] >= RADIX_ROWS:
        _check(scores, labels)
        auc, _ = auc_radix(scores, labels)
        return float(auc.item())
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


# ---- histogram AUC (K10 `auc_hist`): mergeable across ranks by summing histograms ------------
def _order_key_np(scores: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(scores, dtype=np.float32).view(np.uint32)
    b = np.where(b == np.uint32(0x80000000), np.uint32(0), b)  # -0 == +0
    return np.where(b & np.uint32(0x80000000), ~b, b | np.uint32(0x80000000)).astype(np.uint32)


def score_histogram(scores: torch.Tensor, labels: torch.Tensor, bits: int = 20) -> torch.Tensor:
    """int32 [2, 2^bits] counts of (negative, positive) scores per bin of the order-preserving key."""
    _check(scores, labels)
    nb = 1 << bits
    if not scores.is_cuda:
        key = _order_key_np(scores.numpy()) >> np.uint32(32 - bits)
        lab = labels.numpy() != 0
        h = np.stack([np.bincount(key[~lab], minlength=nb), np.bincount(key[lab], minlength=nb)]).astype(np.int32)
        return torch.from_numpy(h)
    hist = torch.zeros(2 * nb, dtype=torch.int32, device=scores.device)
    native().auc_hist(ptr(scores), ptr(labels), scores.shape[0], bits, ptr(hist), stream_of(scores))
    return hist.view(2, nb)


def auc_from_histogram(hist: torch.Tensor) -> tuple[int, int, int]:
    """(twice_pairs, P, N) with bins as tie classes: sum_b P_b (2 N_<b + N_b), exact integers."""
    nb = hist.shape[1]
    bits = nb.bit_length() - 1
    if not hist.is_cuda:
        h = hist.numpy().astype(np.int64)
        nbefore = np.concatenate([[0], np.cumsum(h[0])[:-1]])
        twice = int(np.sum(h[1] * (2 * nbefore + h[0])))
        return twice, int(h[1].sum()), int(h[0].sum())
    out = torch.zeros(3, dtype=torch.int64, device=hist.device)
    native().auc_hist_reduce(ptr(hist), bits, ptr(out), stream_of(hist))
    twice, P, N = (int(v) for v in out.cpu())
    return twice, P, N


def roc_auc_hist(scores: torch.Tensor, labels: torch.Tensor, bits: int = 20, comm=None) -> float:
    """ROC-AUC from score histograms (scores in one bin count as ties).  With ``comm`` the
    histograms of all ranks are summed (one fixed-size all-reduce, collective C6) instead of
    gathering every score; 2^20 bins resolve float32 scores to ~2^-11 relative."""
    hist = score_histogram(scores, labels, bits)
    if comm is not None and comm.world_size > 1:
        hist = comm.all_reduce_(hist.contiguous())
    twice, P, N = auc_from_histogram(hist)
    if P == 0 or N == 0:
        return float("nan")
    return twice / (2.0 * P * N)


def roc_curve_hist(scores: torch.Tensor, labels: torch.Tensor, bits: int = 16, comm=None):
    """(fpr, tpr) at every bin edge, descending threshold -- the evaluate_model.py ROC plot."""
    hist = score_histogram(scores, labels, bits)
    if comm is not None and comm.world_size > 1:
        hist = comm.all_reduce_(hist.contiguous())
    h = hist.cpu().numpy().astype(np.int64)[:, ::-1]
    tp, fp = np.cumsum(h[1]), np.cumsum(h[0])
    P, N = max(tp[-1], 1), max(fp[-1], 1)
    keep = np.r_[True, (np.diff(tp) + np.diff(fp)) > 0]
    return np.r_[0.0, fp[keep] / N], np.r_[0.0, tp[keep] / P]
