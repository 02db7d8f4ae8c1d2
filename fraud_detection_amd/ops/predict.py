"""K5 batch predict and K6 fused predict + linear SHAP."""
from __future__ import annotations

import numpy as np
import torch

from . import reference as ref
from .layout import BIAS_COL, DEFAULT_FP8_SCALE, NCOLS, check_rows, storage_kind
from .native import native, ptr, stream_of


def _w32(w: torch.Tensor, device) -> torch.Tensor:
    """[32] fp32 weights on ``device``.  The predict kernels ignore w[LABEL_COL] (predict.hip:
    the label column's weight is taken as 0), so resident fp32 device weights are used as they
    are: no copy, no read-back, no host synchronisation per call."""
    if tuple(w.shape) != (NCOLS,):
        raise ValueError("weights must be [32] (padded layout; w[30] = intercept)")
    return w.to(device=device, dtype=torch.float32).contiguous()


def fp8_weights(w: torch.Tensor, d: int = 30, fp8_scale: float = DEFAULT_FP8_SCALE) -> torch.Tensor:
    """Weights for fp8 rows, which store features * fp8_scale (bias/label unscaled)."""
    w2 = w.clone()
    w2[:d] = w2[:d] / fp8_scale
    return w2


def predict_rows(rows: torch.Tensor, w: torch.Tensor, want_logit: bool = False,
                 fp8_scale: float = DEFAULT_FP8_SCALE, d: int = 30):
    """P(fraud) for standardized padded rows (bf16 or fp8).  Returns prob (and logit)."""
    check_rows(rows)
    n = rows.shape[0]
    kind = storage_kind(rows)
    if not rows.is_cuda:
        R = ref.rows_to_f32(rows, fp8_scale, d).numpy()
        p, z = ref.predict_rows(R, w.cpu().double().numpy())
        p = torch.from_numpy(p.astype(np.float32))
        z = torch.from_numpy(z.astype(np.float32))
        return (p, z) if want_logit else p
    m = native()
    wv = _w32(w, rows.device)
    prob = torch.empty(n, device=rows.device, dtype=torch.float32)
    logit = torch.empty(n, device=rows.device, dtype=torch.float32) if want_logit else None
    s = stream_of(rows)
    if kind == "bf16":
        m.predict_bf16(ptr(rows), n, ptr(wv), ptr(prob), ptr(logit), s)
    elif kind == "fp8":
        m.predict_fp8(ptr(rows), n, ptr(fp8_weights(wv, d, fp8_scale)), ptr(prob), ptr(logit), s)
    else:
        raise ValueError("predict_rows supports bf16 / fp8 row storage")
    return (prob, logit) if want_logit else prob


def fold_scaler(w: np.ndarray, mean: np.ndarray, scale: np.ndarray, bg_std: np.ndarray | None = None):
    """Fold StandardScaler into the linear model so raw features are read once.

    z = sum_j w_j (x_j - mu_j)/sigma_j + b = sum_j a_j x_j + b',  a_j = w_j / sigma_j,
    b' = b - sum_j a_j mu_j.   LinearSHAP in standardized space with background mean bg:
    phi_j = w_j ((x_j - mu_j)/sigma_j - bg_j) = a_j (x_j - c_j),  c_j = mu_j + sigma_j bg_j.
    """
    d = len(mean)
    w = np.asarray(w, dtype=np.float64)
    a = np.zeros(NCOLS)
    c = np.zeros(NCOLS)
    a[:d] = w[:d] / np.asarray(scale, dtype=np.float64)
    bg = np.zeros(d) if bg_std is None else np.asarray(bg_std, dtype=np.float64)[:d]
    c[:d] = np.asarray(mean, dtype=np.float64) + np.asarray(scale, dtype=np.float64) * bg
    bias = float(w[BIAS_COL] - np.dot(a[:d], mean))
    return a, c, bias


def predict_shap_raw(X: torch.Tensor, a: torch.Tensor, c: torch.Tensor, bias: float, dphi: int | None = None,
                     want_logit: bool = False):
    """Fused scaler-folded predict + LinearSHAP on raw fp32 features [n, d] (online serving / XAI
    worker path).  Returns (prob, phi[n, dphi]) (+ logit)."""
    if X.dim() != 2 or X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("X must be row-major float32 [n, d]")
    n, d = X.shape
    dphi = d if dphi is None else dphi
    if not X.is_cuda:
        p, z, phi = ref.predict_shap(X.numpy(), a.cpu().numpy(), c.cpu().numpy(), bias, d, dphi)
        out = (torch.from_numpy(p.astype(np.float32)), torch.from_numpy(phi.astype(np.float32)))
        return out + (torch.from_numpy(z.astype(np.float32)),) if want_logit else out
    m = native()
    av = a.to(X.device, torch.float32).contiguous()
    cv = c.to(X.device, torch.float32).contiguous()
    prob = torch.empty(n, device=X.device, dtype=torch.float32)
    phi = torch.empty((n, dphi), device=X.device, dtype=torch.float32)
    phi_ptr = ptr(phi) if dphi > 0 else 0
    logit = torch.empty(n, device=X.device, dtype=torch.float32) if want_logit else None
    m.predict_shap(ptr(X), 1, n, X.stride(0), d, dphi, ptr(av), ptr(cv), float(bias), ptr(prob), ptr(logit),
                   phi_ptr, dphi, stream_of(X))
    return (prob, phi, logit) if want_logit else (prob, phi)


def predict_shap_rows(rows: torch.Tensor, w: torch.Tensor, bg: torch.Tensor, dphi: int = 30,
                      want_logit: bool = False):
    """Fused predict + LinearSHAP on standardized bf16 rows: phi_j = w_j (x_j - bg_j)."""
    check_rows(rows)
    if storage_kind(rows) != "bf16":
        raise ValueError("predict_shap_rows expects bf16 rows")
    n = rows.shape[0]
    w = w.to(torch.float64)
    bgv = bg.to(torch.float64).clone()
    bgv[BIAS_COL] = 1.0
    if not rows.is_cuda:
        p, z, phi = ref.predict_shap(rows.float().numpy(), w.cpu().numpy(), bgv.cpu().numpy(), 0.0, 31, dphi)
        out = (torch.from_numpy(p.astype(np.float32)), torch.from_numpy(phi.astype(np.float32)))
        return out + (torch.from_numpy(z.astype(np.float32)),) if want_logit else out
    m = native()
    av = w.to(rows.device, torch.float32).contiguous()
    cv = bgv.to(rows.device, torch.float32).contiguous()
    prob = torch.empty(n, device=rows.device, dtype=torch.float32)
    phi = torch.empty((n, dphi), device=rows.device, dtype=torch.float32)
    logit = torch.empty(n, device=rows.device, dtype=torch.float32) if want_logit else None
    m.predict_shap(ptr(rows), 0, n, NCOLS, 31, dphi, ptr(av), ptr(cv), 0.0, ptr(prob), ptr(logit), ptr(phi), dphi,
                   stream_of(rows))
    return (prob, phi, logit) if want_logit else (prob, phi)
