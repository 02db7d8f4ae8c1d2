"""CPU oracles for every HIP kernel (SURVEY.md §7.5 "CPU oracles first").

These are the semantics the kernels implement, written plainly in numpy/torch (fp64 unless the
kernel's storage format says otherwise).  GPU tests compare the kernels against these; CPU
tensors run through them, so the whole framework is exercisable without a GPU.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .layout import BIAS_COL, LABEL_COL, NCOLS

# ------------------------------------------------------------------------------------------
# Philox4x32-10 (bit-exact with common.h philox4x32_10)
# ------------------------------------------------------------------------------------------
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    c0 = np.asarray(c0, dtype=np.uint32).copy()
    c1 = np.asarray(c1, dtype=np.uint32).copy()
    c2 = np.asarray(c2, dtype=np.uint32).copy()
    c3 = np.asarray(c3, dtype=np.uint32).copy()
    k0 = np.uint32(k0 & 0xFFFFFFFF)
    k1 = np.uint32(k1 & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return c0, c1, c2, c3


def u32_to_unit(v):
    return (np.asarray(v, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def u32_range(v, n: int):
    return ((np.asarray(v, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


# ------------------------------------------------------------------------------------------
# storage codecs
# ------------------------------------------------------------------------------------------
def bf16_round(x: np.ndarray) -> np.ndarray:
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16).float().numpy()


def fp8_decode(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, dtype=np.uint8).astype(np.int64)
    s = (b >> 7) & 1
    e = (b >> 3) & 0xF
    m = b & 7
    sub = m.astype(np.float64) * 2.0 ** -9
    nor = (1.0 + m / 8.0) * np.exp2(e - 7.0)
    out = np.where(e == 0, sub, nor)
    out = np.where((e == 15) & (m == 7), np.nan, out)
    return np.where(s == 1, -out, out).astype(np.float32)


def fp8_encode(x: np.ndarray) -> np.ndarray:
    """RNE, saturating to +-448 (OCP e4m3fn satfinite); mirrors common.h f32_to_fp8e4m3."""
    x = np.asarray(x, dtype=np.float32)
    out = np.zeros(x.shape, dtype=np.uint8)
    flat_x = x.reshape(-1)
    flat_o = out.reshape(-1)
    for i, v in enumerate(flat_x):  # small arrays only (tests)
        flat_o[i] = _fp8_encode_scalar(float(v))
    return out


def _fp8_encode_scalar(f: float) -> int:
    sign = 0x80 if math.copysign(1.0, f) < 0 else 0
    a = abs(f)
    if a != a:
        return 0x7F
    if a >= 464.0:
        return sign | 0x7E
    if a < 2.0 ** -10:
        return sign
    fr, e = math.frexp(a)
    be = e - 1 + 7
    if be <= 0:
        r = _rint(a * 512.0)
        return sign | int(r)
    mant = (fr * 2.0 - 1.0) * 8.0
    r = _rint(mant)
    if r >= 8.0:
        r = 0.0
        be += 1
    if be > 15 or (be == 15 and r >= 7.0):
        return sign | 0x7E
    return sign | (be << 3) | int(r)


def _rint(v: float) -> float:
    return float(np.rint(np.float32(v)))


def rows_to_f32(rows: torch.Tensor, fp8_scale: float = 4.0, d: int = 30) -> torch.Tensor:
    """Decode a padded row buffer (bf16 / f32 / fp8-as-uint8) to fp32 [n, 32] in model space."""
    if rows.dtype == torch.bfloat16:
        return rows.float()
    if rows.dtype == torch.float32:
        return rows
    if rows.dtype == torch.uint8:
        v = torch.from_numpy(fp8_decode(rows.cpu().numpy()))
        v[:, :d] /= fp8_scale
        return v
    raise ValueError(rows.dtype)


# ------------------------------------------------------------------------------------------
# K1 / K2 scaler
# ------------------------------------------------------------------------------------------
def scaler_sums(X: np.ndarray, pivot: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float32)
    d = X.shape[1]
    D = X.astype(np.float64) - np.asarray(pivot, dtype=np.float32).astype(np.float64)[None, :d]
    out = np.zeros(64)
    out[:d] = D.sum(0)
    out[32 : 32 + d] = (D * D).sum(0)
    return out


def scaler_finalize(sums: np.ndarray, n: float, pivot: np.ndarray, d: int):
    eps = np.finfo(np.float64).eps
    mean = np.zeros(32)
    var = np.zeros(32)
    scale = np.ones(32)
    m = sums[:d] / n
    mean[:d] = np.asarray(pivot[:d], dtype=np.float32).astype(np.float64) + m
    v = np.maximum(sums[32 : 32 + d] / n - m * m, 0.0)
    var[:d] = v
    ub = n * eps * v + (n * mean[:d] * eps) ** 2
    scale[:d] = np.where(v <= ub, 1.0, np.sqrt(v))
    mean32 = mean.astype(np.float32)
    inv32 = np.zeros(32, dtype=np.float32)
    inv32[:d] = (1.0 / scale[:d]).astype(np.float32)
    return mean, var, scale, mean32, inv32


def scale_cast(X, mean32, inv32, labels=None, bias_value=1.0, out_kind="bf16", fp8_scale=4.0, idx=None):
    X = np.asarray(X, dtype=np.float32)
    if idx is not None:
        X = X[np.asarray(idx)]
        if labels is not None:
            labels = np.asarray(labels)[np.asarray(idx)]
    n, d = X.shape
    out = np.zeros((n, NCOLS), dtype=np.float32)
    out[:, :d] = (X - mean32[None, :d]) * inv32[None, :d]
    out[:, BIAS_COL] = bias_value
    if labels is not None:
        out[:, LABEL_COL] = np.asarray(labels, dtype=np.float32)
    if out_kind == "bf16":
        return torch.from_numpy(out).to(torch.bfloat16)
    if out_kind == "f32":
        return torch.from_numpy(out)
    if out_kind == "fp8":
        scaled = out.copy()
        scaled[:, :d] *= fp8_scale
        return torch.from_numpy(fp8_encode(scaled))
    raise ValueError(out_kind)


# ------------------------------------------------------------------------------------------
# K5 / K6 predict + linear SHAP
# ------------------------------------------------------------------------------------------
def sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def predict_rows(rows_f32: np.ndarray, w: np.ndarray):
    w = np.asarray(w, dtype=np.float64).copy()
    w[LABEL_COL] = 0.0
    z = np.asarray(rows_f32, dtype=np.float64) @ w
    return sigmoid(z), z


def predict_shap(X: np.ndarray, a: np.ndarray, c: np.ndarray, bias: float, dz: int, dphi: int):
    X = np.asarray(X, dtype=np.float64)
    a = np.asarray(a, dtype=np.float64)
    c = np.asarray(c, dtype=np.float64)
    z = X[:, :dz] @ a[:dz] + bias
    phi = a[None, :dphi] * (X[:, :dphi] - c[None, :dphi])
    return sigmoid(z), z, phi


# ------------------------------------------------------------------------------------------
# K4 logistic regression
# ------------------------------------------------------------------------------------------
def logreg_pass(rows_f32: np.ndarray, w: np.ndarray, class_w=(1.0, 1.0), hessian=True):
    R = np.asarray(rows_f32, dtype=np.float64)
    y = R[:, LABEL_COL].copy()
    X = R.copy()
    X[:, LABEL_COL] = 0.0
    w = np.asarray(w, dtype=np.float64).copy()
    w[LABEL_COL] = 0.0
    z = X @ w
    p = sigmoid(z)
    s = np.where(y > 0.5, class_w[1], class_w[0])
    r = s * (p - y)
    g = X.T @ r
    loss = float(np.sum(s * (np.logaddexp(0.0, z) - y * z)))
    wsum = float(s.sum())
    H = (X * (s * p * (1 - p))[:, None]).T @ X if hessian else None
    return g, loss, wsum, H


def pack_reduced(g, loss, wsum, H) -> np.ndarray:
    red = np.zeros(1088)
    red[:32] = g
    red[32] = loss
    red[33] = wsum
    if H is not None:
        red[64:] = np.asarray(H).reshape(-1)
    return red


class NewtonStateRef:
    """Mirror of logreg.hip newton_update_kernel (same decisions, fp64)."""

    def __init__(self, w0: np.ndarray):
        self.w = np.asarray(w0, dtype=np.float64).copy()
        self.w_prev = self.w.copy()
        self.step = np.zeros(32)
        self.vel = np.zeros(32)
        self.obj_prev = np.inf
        self.iter = 0
        self.backtracks = 0
        self.gmax = np.inf
        self.obj = np.inf
        self.n_accepted = 0
        self.converged = False
        self.done = False

    def update(self, red, d, C, tol, max_iter, fit_intercept=True):
        if self.done:
            return
        S = red[33] if red[33] > 0 else 1.0
        reg = 1.0 / (C * S)
        idx = list(range(d)) + ([BIAS_COL] if fit_intercept else [])
        grad = np.zeros(32)
        grad[:d] = red[:d] / S + reg * self.w[:d]
        if fit_intercept:
            grad[BIAS_COL] = red[BIAS_COL] / S
        obj = red[32] / S + 0.5 * reg * float(np.dot(self.w[:d], self.w[:d]))
        gmax = float(np.max(np.abs(grad[idx])))
        self.obj = obj
        if self.iter > 0 and obj > self.obj_prev + 1e-6 * abs(self.obj_prev) and self.backtracks < 40:
            self.step *= 0.5
            self.w = self.w_prev + self.step
            self.backtracks += 1
            dec = 1
        elif gmax <= tol:
            self.gmax = gmax
            self.converged = True
            self.done = True
            dec = 2
        else:
            self.gmax = gmax
            Hf = np.asarray(red[64:]).reshape(32, 32)
            SH = red[34] if red[34] > 0 else S  # weight of the rows behind H (device: slot 34)
            A = Hf[np.ix_(idx, idx)] / SH
            for k, j in enumerate(idx):
                if j < d:
                    A[k, k] += reg
            L = np.linalg.cholesky(A)
            st = np.linalg.solve(L.T, np.linalg.solve(L, -grad[idx]))
            self.w_prev = self.w.copy()
            self.step = np.zeros(32)
            self.step[idx] = st
            self.w = self.w_prev + self.step
            self.obj_prev = obj
            self.backtracks = 0
            self.n_accepted += 1
            dec = 0
        self.iter += 1
        if dec != 2 and self.iter >= max_iter:
            self.done = True


WAVES_PER_BLOCK = 4     # logreg.hip kThreads / 64
ROW_TILE = 64           # rows per wave tile
PICK_TILE = 16          # virtual-SMOTE picks per wave tile (bf16 and fp8 passes: 4 lanes per pick)
PICK_TILE_BF16 = PICK_TILE
SGD_MIN_SPAN = 4        # every SGD minibatch spans >= 4 strided blocks of row tiles
SGD_FULL_BLOCKS = 512   # the SGD pass grid of a 256-CU MI355X (logreg.hip sgd_full_blocks: 2 per CU)


def sgd_grid_blocks(n_stored: int, nb: int, full_blocks: int) -> int:
    """Blocks of the SGD pass grid: the full resident grid, shrunk for small shards so that every
    minibatch spans >= SGD_MIN_SPAN strided blocks of G = 4 * blocks row tiles (its rows then come
    from the whole shard, not from one contiguous window)."""
    want = int(n_stored) // (ROW_TILE * WAVES_PER_BLOCK * max(1, int(nb)) * SGD_MIN_SPAN)
    return int(max(1, min(int(full_blocks), want)))


def sgd_row_batches(n_stored: int, nb: int, blocks: int | None = None) -> np.ndarray:
    """Minibatch of every stored row (logreg.hip bf16_wave_pass row_phase walk): row tile
    t = row // 64 belongs to minibatch t mod nb (tile-interleaved: every minibatch samples the whole
    shard at 64-row granularity; the grid size ``blocks`` no longer enters)."""
    return (np.arange(int(n_stored), dtype=np.int64) // ROW_TILE) % int(nb)


def sgd_pick_batches(n_picks: int, nb: int, pick_tile: int = PICK_TILE_BF16) -> np.ndarray:
    """Minibatch of every virtual-SMOTE pick: pick tile t = pick // pick_tile belongs to t mod nb
    (all samples of a pick land in the pick's minibatch)."""
    return (np.arange(int(n_picks), dtype=np.int64) // int(pick_tile)) % int(nb)


SGD_DBAR_FLOOR = 1e-3


class SgdStateRef:
    """Mirror of logreg.hip sgd_apply (fp64): heavy-ball momentum SGD with the step normalised by
    the minibatch's mean curvature, Polyak averaging, epoch-end convergence state."""

    def __init__(self, w0: np.ndarray):
        self.w = np.asarray(w0, dtype=np.float64).copy()
        self.v = np.zeros(32)
        self.avg = np.zeros(32)
        self.n_avg = 0
        self.ep_g = np.zeros(32)
        self.ep_loss = 0.0
        self.ep_w = 0.0
        self.iter = 0
        self.gmax = np.inf
        self.obj = np.inf
        self.converged = False
        self.done = False

    def step(self, g_raw, loss, wsum, dsum, d, C, c, mom, nb, avg, epoch_end, tol, fit_intercept=True):
        if self.done:
            return
        S = wsum if wsum > 0 else 1.0
        reg = 1.0 / (C * S * nb)
        lr = c / max(dsum / S, SGD_DBAR_FLOOR)
        g = np.zeros(32)
        g[:d] = g_raw[:d] / S + reg * self.w[:d]
        if fit_intercept:
            g[BIAS_COL] = g_raw[BIAS_COL] / S
        self.v = mom * self.v - lr * g
        self.w = self.w + self.v
        self.ep_g += np.asarray(g_raw[:32], dtype=np.float64)
        self.ep_loss += loss
        self.ep_w += wsum
        if avg:
            self.avg += self.w
            self.n_avg += 1
        self.iter += 1
        if epoch_end:
            Sw = self.ep_w if self.ep_w > 0 else 1.0
            if self.n_avg > 0:
                self.w = self.avg / self.n_avg
            G = np.zeros(32)
            G[:d] = self.ep_g[:d] / Sw + self.w[:d] / (C * Sw)
            if fit_intercept:
                G[BIAS_COL] = self.ep_g[BIAS_COL] / Sw
            self.gmax = float(np.abs(G).max())
            self.obj = self.ep_loss / Sw + 0.5 * float(self.w[:d] @ self.w[:d]) / (C * Sw)
            self.ep_g[:] = 0.0
            self.avg[:] = 0.0
            self.ep_loss = self.ep_w = 0.0
            self.n_avg = 0
            if self.gmax <= tol:
                self.converged = self.done = True


# ------------------------------------------------------------------------------------------
# K8 / K9 SMOTE
# ------------------------------------------------------------------------------------------
def knn_topk(Q: np.ndarray, C: np.ndarray, k: int, self_offset: int = -1):
    """Exact k nearest neighbours (squared L2 over the 30 feature columns; columns 30/31 of the
    padded layout -- intercept and label -- are not features) with the kernel's tie rule."""
    Q = np.asarray(Q, dtype=np.float64)[:, :30]
    C = np.asarray(C, dtype=np.float64)[:, :30]
    score = Q @ C.T - 0.5 * np.sum(C * C, axis=1)[None, :]
    if self_offset >= 0:
        rows = np.arange(Q.shape[0])
        score[rows, self_offset + rows] = -np.inf
    order = np.lexsort((np.broadcast_to(np.arange(C.shape[0]), score.shape), -score), axis=1)
    idx = order[:, :k].astype(np.int32)
    d2 = np.sum(Q * Q, 1)[:, None] - 2.0 * np.take_along_axis(score, idx.astype(np.int64), 1)
    return idx, d2


SMOTE_MAX_ROWS = 1 << 24  # i / j are packed into 24 bits of a draw (common.h smote_pack_draw)


def smote_check_ranges(n_parents: int, mq: int, k: int) -> None:
    """The packed draw holds i and j in 24 bits and the Lemire pick ranges over mq*k in 32 bits:
    refuse sizes that would silently wrap.  Shard the SMOTE query set above this."""
    if n_parents >= SMOTE_MAX_ROWS:
        raise ValueError(f"SMOTE parent set has {n_parents} rows; the packed draw indexes < 2^24 "
                         f"({SMOTE_MAX_ROWS}) rows -- use smote_scope='shard' or subsample the minority class")
    if mq * k >= 1 << 32:
        raise ValueError(f"SMOTE pick range mq*k = {mq}*{k} does not fit 32 bits")


def smote_plan(nbr: np.ndarray, n_new: int, seed: int, counter_base: int, sample_offset: int = 0) -> np.ndarray:
    """uint32 [n_new, 2] SMOTE draws {i | lam_hi << 24, j | lam_lo << 24} (common.h
    smote_pack_draw): one Philox call per pair of samples -- in 128-sample block m, counter
    64 m + L serves sample 128 m + L with words (x, y) and sample 128 m + 64 + L with (z, w); query
    row i and neighbour slot from one Lemire pick over mq*k, lam = (word >> 16) / 2^16."""
    nbr = np.asarray(nbr)
    mq, k = nbr.shape
    smote_check_ranges(mq, mq, k)
    pick, lam = smote_pick_draws(mq, k, n_new, seed, counter_base, sample_offset)
    i = (pick // k).astype(np.uint32)
    j = nbr[i, pick % k].astype(np.uint32)
    return np.stack([i | ((lam >> np.uint32(8)) << np.uint32(24)), j | ((lam & np.uint32(0xFF)) << np.uint32(24))], 1)


def smote_pick_draws(mq: int, k: int, n_new: int, seed: int, counter_base: int, sample_offset: int = 0):
    """(pick = query row * k + neighbour slot, lam * 2^16) of each sample, uint32 (smote_plan's
    draws before the neighbour lookup; the virtual-SMOTE buckets group samples by pick)."""
    s = np.arange(n_new, dtype=np.uint64) + np.uint64(sample_offset)
    c = (s // np.uint64(128)) * np.uint64(64) + (s % np.uint64(64))
    half = ((s % np.uint64(128)) // np.uint64(64)).astype(bool)
    r = philox4x32_10((c & _MASK32).astype(np.uint32), (c >> np.uint64(32)).astype(np.uint32),
                      np.full(n_new, counter_base & 0xFFFFFFFF, np.uint32),
                      np.full(n_new, (counter_base >> 32) & 0xFFFFFFFF, np.uint32),
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    wp = np.where(half, r[2], r[0])
    wl = np.where(half, r[3], r[1])
    return u32_range(wp, mq * k).astype(np.uint32), wl.astype(np.uint32) >> np.uint32(16)


def smote_draws_decode(plan: np.ndarray):
    """(i, j, lam float32) from smote_plan words."""
    p = np.asarray(plan, dtype=np.uint32)
    lam16 = ((p[:, 0] >> np.uint32(24)) << np.uint32(8)) | (p[:, 1] >> np.uint32(24))
    mask = np.uint32(0xFFFFFF)
    return ((p[:, 0] & mask).astype(np.int64), (p[:, 1] & mask).astype(np.int64),
            lam16.astype(np.float32) * np.float32(1.0 / 65536.0))


def smote_generate(C: np.ndarray, nbr: np.ndarray, q_offset: int, n_new: int, seed: int,
                   counter_base: int, label: float = 1.0, sample_offset: int = 0) -> np.ndarray:
    """fp32 synthetic rows (before bf16/fp8 rounding), bit-exact Philox draws."""
    C = np.asarray(C, dtype=np.float32)
    nbr = np.asarray(nbr)
    i, j, lam = smote_draws_decode(smote_plan(nbr, n_new, seed, counter_base, sample_offset))
    lam = lam[:, None]
    xi = C[q_offset + i]
    xj = C[j]
    out = (xi + lam * (xj - xi)).astype(np.float32)
    out[:, BIAS_COL] = 1.0
    out[:, LABEL_COL] = label
    return out


# ------------------------------------------------------------------------------------------
# K10 metrics
# ------------------------------------------------------------------------------------------
def roc_auc(scores: np.ndarray, labels: np.ndarray) -> float:
    """Exact ROC-AUC with averaged ties (== sklearn.metrics.roc_auc_score)."""
    s = np.asarray(scores, dtype=np.float64)
    y = np.asarray(labels).astype(bool)
    P, N = int(y.sum()), int((~y).sum())
    if P == 0 or N == 0:
        return float("nan")
    order = np.argsort(s, kind="mergesort")
    ss = s[order]
    ranks = np.empty(len(s))
    # average ranks over ties
    i = 0
    n = len(ss)
    bounds = np.flatnonzero(np.diff(ss)) + 1
    starts = np.concatenate([[0], bounds])
    ends = np.concatenate([bounds, [n]])
    avg = (starts + ends + 1) / 2.0
    ranks_sorted = np.repeat(avg, ends - starts)
    ranks[order] = ranks_sorted
    del i
    return float((ranks[y].sum() - P * (P + 1) / 2.0) / (P * N))


def confusion(scores, labels, thr: float):
    s = np.asarray(scores)
    y = np.asarray(labels).astype(bool)
    p = s > thr
    return np.array([np.sum(~y & ~p), np.sum(~y & p), np.sum(y & ~p), np.sum(y & p)], dtype=np.int64)
