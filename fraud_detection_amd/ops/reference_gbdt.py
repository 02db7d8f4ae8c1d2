"""Numpy oracle of the K11 GBDT kernels (csrc/kernels/gbdt.hip), also the CPU execution path.

Same algorithm, same fixed-point quantisation, same fp64 operation order in the split gain,
same tie rules, so a device fit given the same quantised gradients builds bit-identical trees:

* cuts: per feature, sample quantiles at i*m//B (i = 1..B-1) of the sorted sample, deduplicated,
  values <= the sample minimum dropped, +inf appended (bin(x) = #cuts <= x, bins [0, nb-1]);
* split "bins <= b go left" <=> x < cuts[b]; gain = (GL^2/(HL+l) + GR^2/(HR+l)) - G^2/(H+l),
  valid when HL, HR >= min_child_weight; argmax over (feature, bin), ties -> lowest feature,
  then lowest bin; split iff gain > 1e-6 and not gain < gamma (xgboost kRtEps / pruner);
* complete heap trees of depth D; a non-split node passes every row to its left child;
* leaf = float32(eta * (-G/(H+l))) (0 when H < min_child_weight or H <= 0).

xgboost itself is not installed in this image, so parity with xgboost is "unpinned"; the
semantics above follow xgboost's hist updater (train_model.py:69-80 uses XGBClassifier).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

MAX_BIN = 256
ROW_BYTES = 32


def quantile_cuts(sample: np.ndarray, max_bin: int = MAX_BIN):
    """sample: [m, d] float32.  Returns (cuts [d, 256] float32 padded with +inf, nbins [d] int32)."""
    sample = np.asarray(sample, dtype=np.float32)
    m, d = sample.shape
    if max_bin < 2 or max_bin > MAX_BIN:
        raise ValueError("max_bin must be in [2, 256]")
    cuts = np.full((d, MAX_BIN), np.inf, dtype=np.float32)
    nbins = np.zeros(d, dtype=np.int32)
    if m == 0:
        nbins[:] = 1
        return cuts, nbins
    idx = (np.arange(1, max_bin, dtype=np.int64) * m) // max_bin
    srt = np.sort(sample, axis=0)
    return cuts_from_sorted_picks(srt[idx], srt[0], max_bin)


def cuts_from_sorted_picks(picks: np.ndarray, vmin: np.ndarray, max_bin: int = MAX_BIN):
    """picks [max_bin-1, d]: sample values at the quantile positions; vmin [d]: sample minimum."""
    picks = np.asarray(picks, dtype=np.float32)
    d = picks.shape[1]
    cuts = np.full((d, MAX_BIN), np.inf, dtype=np.float32)
    nbins = np.zeros(d, dtype=np.int32)
    for f in range(d):
        c = np.unique(picks[:, f])
        c = c[c > vmin[f]][: max_bin - 1]
        cuts[f, : len(c)] = c
        nbins[f] = len(c) + 1  # + the +inf cut
    return cuts, nbins


def bin_rows(X: np.ndarray, cuts: np.ndarray, nbins: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float32)
    n, d = X.shape
    out = np.zeros((n, ROW_BYTES), dtype=np.uint8)
    for f in range(d):
        nb = int(nbins[f])
        out[:, f] = np.searchsorted(cuts[f, :nb], X[:, f], side="right").clip(0, nb - 1)
    return out


GRAD_BITS = 14  # |g_q|, h_q <= 2^14: the device packs (h, g) of a row into one 64-bit LDS atomic


def grad_scales(scale_pos_weight: float):
    """Power-of-two fixed-point scales with |g * gscale| <= 2^14 and h * hscale <= 2^14
    (h = p (1 - p) w <= w / 4): 2^16 rows of packed (h << 32) + g sum exactly in 64 bits."""
    wmax = max(float(scale_pos_weight), 1.0)
    gscale = float(2.0 ** np.floor(np.log2((2.0 ** GRAD_BITS) / wmax)))
    return gscale, 4.0 * gscale


def gradients(margin: np.ndarray, y: np.ndarray, spw: float, gscale: float, hscale: float) -> np.ndarray:
    """int32 [n, 2] quantised (g, h) of the logistic loss (fp64 arithmetic on fp32 margins)."""
    m = np.asarray(margin, dtype=np.float32).astype(np.float64)
    p = 1.0 / (1.0 + np.exp(-m))
    pos = np.asarray(y) != 0
    w = np.where(pos, float(np.float32(spw)), 1.0)
    g = (p - pos.astype(np.float64)) * w
    h = np.maximum(p * (1.0 - p), 1e-16) * w
    return np.stack([np.rint(g * gscale), np.rint(h * hscale)], 1).astype(np.int32)


def _hist(bins: np.ndarray, q: np.ndarray, node: np.ndarray, nn: int, d: int) -> np.ndarray:
    """int64 [nn, d, 256, 2] exact histograms (float64 bincount of integers in < 2^53 chunks)."""
    out = np.zeros((nn, d, MAX_BIN, 2), dtype=np.int64)
    n = bins.shape[0]
    step = max(1, int(2 ** 52 // (2 ** 31 + 1)) // 2)
    keys_f = (np.arange(d, dtype=np.int64) * MAX_BIN)[None, :]
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        k = (node[lo:hi, None].astype(np.int64) * (d * MAX_BIN) + keys_f + bins[lo:hi, :d]).ravel()
        for c in range(2):
            w = np.repeat(q[lo:hi, c].astype(np.float64), d)
            out[..., c] += np.bincount(k, weights=w, minlength=nn * d * MAX_BIN).astype(np.int64).reshape(nn, d, MAX_BIN)
    return out


@dataclass
class TreeArrays:
    feat: np.ndarray   # [ni] int32, -1 = pass-through
    bin: np.ndarray    # [ni] int32
    thr: np.ndarray    # [ni] float32 (+inf when not split)
    gain: np.ndarray   # [ni] float64
    leaf: np.ndarray   # [nl] float32


def best_split(H: np.ndarray, nbins: np.ndarray, ginv: float, hinv: float, lam: float, mcw: float):
    """H: int64 [d, 256, 2] of one node.  Returns (gain, feature, bin, GLq, HLq, Gq, Hq)."""
    d = H.shape[0]
    cg = np.cumsum(H[:, :, 0], axis=1)
    chs = np.cumsum(H[:, :, 1], axis=1)
    Gq, Hq = int(cg[0, -1]), int(chs[0, -1])
    G, Hs = float(Gq) * ginv, float(Hq) * hinv
    root = G * G / (Hs + lam)
    GL = cg.astype(np.float64) * ginv
    HL = chs.astype(np.float64) * hinv
    GR = (Gq - cg).astype(np.float64) * ginv
    HR = (Hq - chs).astype(np.float64) * hinv
    with np.errstate(all="ignore"):
        gain = (GL * GL / (HL + lam) + GR * GR / (HR + lam)) - root
    b = np.arange(MAX_BIN)[None, :]
    valid = (b < (nbins[:d, None] - 1)) & (HL >= mcw) & (HR >= mcw)
    gain = np.where(valid, gain, -np.inf)
    flat = int(np.argmax(gain))
    f, bb = divmod(flat, MAX_BIN)
    return float(gain[f, bb]), f, bb, int(cg[f, bb]), int(chs[f, bb]), Gq, Hq


def build_tree(bins: np.ndarray, q: np.ndarray, cuts: np.ndarray, nbins: np.ndarray, depth: int, lam: float,
               mcw: float, gamma: float, eta: float, gscale: float, hscale: float, comm=None):
    """Grow one depth-`depth` heap tree.  Returns (TreeArrays, leaf index per row [n])."""
    n = bins.shape[0]
    d = int(len(nbins))
    ginv, hinv = 1.0 / gscale, 1.0 / hscale
    ni, nl = (1 << depth) - 1, 1 << depth
    feat = np.full(ni, -1, np.int32)
    binv = np.full(ni, 255, np.int32)
    thr = np.full(ni, np.inf, np.float32)
    gain = np.zeros(ni, np.float64)
    ng = np.zeros(2 * nl - 1, np.int64)
    nh = np.zeros(2 * nl - 1, np.int64)
    node = np.zeros(n, np.int64)  # index within the level
    for level in range(depth):
        nn = 1 << level
        Hl = _hist(bins, q, node, nn, d)
        if comm is not None and comm.world_size > 1:
            import torch

            Hl = comm.all_reduce(torch.from_numpy(Hl)).numpy()
        h0 = nn - 1
        right = np.zeros(n, bool)
        for k in range(nn):
            hid = h0 + k
            g_, f, b, GLq, HLq, Gq, Hq = best_split(Hl[k], nbins, ginv, hinv, lam, mcw)
            if hid == 0:
                ng[0], nh[0] = Gq, Hq
            split = np.isfinite(g_) and g_ > 1e-6 and not (g_ < gamma)
            lc, rc = 2 * hid + 1, 2 * hid + 2
            if split:
                feat[hid], binv[hid], thr[hid], gain[hid] = f, b, cuts[f, b], g_
                ng[lc], nh[lc], ng[rc], nh[rc] = GLq, HLq, Gq - GLq, Hq - HLq
                sel = node == k
                right |= sel & (bins[:, f] > b)
            else:
                ng[lc], nh[lc], ng[rc], nh[rc] = Gq, Hq, 0, 0
        node = 2 * node + right.astype(np.int64)
    leaf = np.zeros(nl, np.float32)
    for i in range(nl):
        G, H = float(ng[ni + i]) * ginv, float(nh[ni + i]) * hinv
        w = 0.0 if (H < mcw or H <= 0.0) else -G / (H + lam)
        leaf[i] = np.float32(eta * w)
    return TreeArrays(feat, binv, thr, gain, leaf), node


def predict_margin(X: np.ndarray, feat: np.ndarray, thr: np.ndarray, leaf: np.ndarray, depth: int,
                   base_margin: float = 0.0) -> np.ndarray:
    """X [n, d] float32; feat/thr [T, ni]; leaf [T, nl].  float32 margins (sum in tree order)."""
    X = np.asarray(X, dtype=np.float32)
    n = X.shape[0]
    out = np.full(n, np.float32(base_margin), dtype=np.float32)
    rows = np.arange(n)
    for t in range(feat.shape[0]):
        node = np.zeros(n, np.int64)
        for _ in range(depth):
            f = feat[t][node]
            xv = X[rows, np.maximum(f, 0)]
            right = (f >= 0) & ~(xv < thr[t][node])
            node = 2 * node + 1 + right
        out = (out + leaf[t][node - ((1 << depth) - 1)]).astype(np.float32)
    return out


def predict_margin_bins(bins: np.ndarray, feat: np.ndarray, binv: np.ndarray, leaf: np.ndarray, depth: int,
                        base_margin: float = 0.0) -> np.ndarray:
    """The device margin walk (gbdt.hip gbdt_margin_kernel) on binned rows: a row goes right at a
    node when its bin of the node's feature exceeds the split bin.  float32, summed in tree order."""
    bins = np.asarray(bins)
    n = bins.shape[0]
    out = np.full(n, np.float32(base_margin), dtype=np.float32)
    rows = np.arange(n)
    for t in range(feat.shape[0]):
        node = np.zeros(n, np.int64)
        for _ in range(depth):
            f = feat[t][node]
            bv = bins[rows, np.maximum(f, 0)].astype(np.int64)
            right = (f >= 0) & (bv > binv[t][node])
            node = 2 * node + 1 + right
        out = (out + leaf[t][node - ((1 << depth) - 1)]).astype(np.float32)
    return out
