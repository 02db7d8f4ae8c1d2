"""K7 KernelSHAP coalition GEMM (csrc/kernels/kernelshap.hip) -- device wrapper."""
from __future__ import annotations

import numpy as np
import torch

from .native import native, ptr, stream_of

_LINKS = {"identity": 0, "logit": 1, "logit_model": 2}


def _device_design(expl, dev):
    """Upload the explainer's design once: Z as bf16 [S_pad, 32] (col 31 = 1 folds the
    background intercepts into the GEMM), A [d-1, S_pad] (zero-padded), A z_M, the weighted
    background rows W and the background logits."""
    key = (str(dev),)
    if expl._dev_cache is not None and expl._dev_cache[0] == key:
        return expl._dev_cache[1]
    d = expl.d
    S = expl.Z.shape[0]
    S_pad = (S + 31) // 32 * 32
    if S_pad > 4096:
        raise ValueError("at most 4096 coalitions per design on device")
    Zp = np.zeros((S_pad, 32), np.float32)
    Zp[:S, :d] = expl.Z
    Zp[:, 31] = 1.0
    a32 = np.zeros(32, np.float32)
    a32[:d] = expl.a[:d]
    cb = (expl.B.astype(np.float64) @ expl.a[:d] + expl.bias).astype(np.float32)
    # W = [a o B_b, 0.., -c_b]: u_b = a o x - W_b, with u_b[31] = c_b folding the intercepts
    W = np.zeros((expl.B.shape[0], 32), np.float32)
    W[:, :d] = (expl.B.astype(np.float32) * a32[:d][None, :]).astype(np.float32)
    W[:, 31] = -cb
    Ap = np.zeros((d - 1, S_pad), np.float32)
    Ap[:, :S] = expl.A
    t = {
        "Z": torch.from_numpy(Zp).to(dev).to(torch.bfloat16).contiguous(),
        "A": torch.from_numpy(Ap).to(dev).contiguous(),
        "Az": torch.from_numpy((expl.A @ expl.zM).astype(np.float32)).to(dev),
        "a": torch.from_numpy(a32).to(dev),
        "bg": torch.from_numpy(W).to(dev),
        "cb": torch.from_numpy(cb).to(dev),
        "S": S, "S_pad": S_pad,
    }
    expl._dev_cache = (key, t)
    return t


def kernelshap(X: torch.Tensor, expl, sync: bool = True, stamps: torch.Tensor | None = None):
    """X [E, d] raw fp32 on device -> (phi [E, d], fx [E], f0) (numpy if sync else tensors).
    ``stamps`` (int64 [E, 8], tools/kernelshap_stamps.py): per-explanation phase timestamps."""
    if X.dim() != 2 or X.dtype != torch.float32 or X.shape[1] != expl.d or not X.is_contiguous():
        raise ValueError(f"X must be contiguous float32 [E, {expl.d}]")
    m = native()
    dev = X.device
    t = _device_design(expl, dev)
    E = X.shape[0]
    phi = torch.empty((E, expl.d), device=dev, dtype=torch.float32)
    fx = torch.empty(E, device=dev, dtype=torch.float32)
    f0 = torch.empty(E, device=dev, dtype=torch.float32)
    m.kernelshap(ptr(X), E, expl.d, ptr(t["a"]), float(expl.bias), ptr(t["bg"]), ptr(t["cb"]), expl.B.shape[0],
                 ptr(t["Z"]), t["S"], t["S_pad"], ptr(t["A"]), ptr(t["Az"]), _LINKS[expl.link], ptr(phi), ptr(fx),
                 ptr(f0), stream_of(X), ptr(stamps))
    if not sync:
        return phi, fx, f0
    return phi.cpu().numpy().astype(np.float64), fx.cpu().numpy().astype(np.float64), float(f0[0].item()) if E else 0.0
