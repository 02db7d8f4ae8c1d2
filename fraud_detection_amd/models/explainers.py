"""Explainers: LinearSHAP (K6) and KernelSHAP with the coalition-masked MFMA GEMM (K7).

Reference: shap.LinearExplainer in explain_model.py:24-27 / api/worker.py:53-75 and the
``coef_ * x`` attribution of xai_tasks.py:103-110 (BASELINE.json
config 4).  shap is not installed here; the algorithms are implemented directly:

LinearSHAP (interventional, independent features): phi_i = w_i (x_i - E_bg[x_i]) in the model's
standardized input space; logit(x) = E[logit] + sum(phi).

KernelSHAP (Lundberg & Lee 2017, shap.KernelExplainer semantics without L1 feature selection):
  * coalition design Z (S x M, S = 2M + 2048 by default): subset sizes enumerated completely from
    the outside in (size 1 and M-1, then 2 and M-2, ...) while the remaining sample budget covers
    them, the rest drawn in complement pairs with Shapley-kernel weights; duplicates merge weights;
  * f(z) = mean_b link(model(z * x + (1 - z) * B_b)) over the background rows B;
  * efficiency-constrained weighted least squares: eliminating the last feature,
        phi_{<M} = A (y - z_M * delta),  phi_M = delta - sum(phi_{<M}),
        A = (X^T W X)^-1 X^T W,  X = Z[:, :M-1] - Z[:, M-1],  y = f(z) - f0,  delta = f(x) - f0,
    so A is solved ONCE per design (fp64, host) and every explanation is two GEMMs.
For the logistic model the coalition logits are linear in z:
    logit(z, b) = sum_i z_i u_bi + c_b,   u_b = a * (x - B_b),   c_b = a . B_b + bias,
i.e. one (n_bg x M) x (M x S) GEMM per explanation: on MI355X bf16 MFMA with Z exact in bf16
and u split into hi + lo bf16 (fp32-grade products), sigmoid/mean epilogue fused, then A y.
Identity link on logits (``link="logit_model"``) makes KernelSHAP exactly equal LinearSHAP, which
is the exact oracle the tests use.
"""
from __future__ import annotations

import itertools
import math
import time

import numpy as np
import torch

from ..ops import predict as P


# ------------------------------------------------------------------------------------------
# coalition design + WLS operator
# ------------------------------------------------------------------------------------------
def coalition_design(M: int, nsamples: int | None = None, seed: int = 0):
    """Return (Z [S, M] uint8, w [S] float64) following shap's KernelExplainer sampling scheme."""
    nsamples = nsamples or 2 * M + 2048
    max_samples = 2 ** 30 if M > 30 else 2 ** M - 2
    nsamples = min(nsamples, max_samples)
    rng = np.random.default_rng(seed)
    num_sizes = int(math.ceil((M - 1) / 2.0))
    num_paired = int(math.floor((M - 1) / 2.0))
    wv = np.array([(M - 1.0) / (i * (M - i)) for i in range(1, num_sizes + 1)])
    wv[:num_paired] *= 2
    wv /= wv.sum()
    rows, weights = [], []
    left = nsamples
    full_sizes = 0
    rem = wv.copy()
    for size in range(1, num_sizes + 1):
        nsub = math.comb(M, size) * (2 if size <= num_paired else 1)
        if left * rem[size - 1] / nsub >= 1.0 - 1e-8:
            full_sizes += 1
            left -= nsub
            if rem[size - 1] < 1.0:
                rem /= 1.0 - rem[size - 1]
            w = wv[size - 1] / math.comb(M, size)
            if size <= num_paired:
                w /= 2.0
            for inds in itertools.combinations(range(M), size):
                z = np.zeros(M, np.uint8)
                z[list(inds)] = 1
                rows.append(z)
                weights.append(w)
                if size <= num_paired:
                    rows.append(1 - z)
                    weights.append(w)
        else:
            break
    nfixed = len(rows)
    if full_sizes != num_sizes and left > 0:
        rem_w = wv[full_sizes:].copy()
        rem_w /= rem_w.sum()
        seen = {}
        drawn = 0
        budget = left
        while drawn < budget:
            size = rng.choice(len(rem_w), p=rem_w) + full_sizes + 1
            z = np.zeros(M, np.uint8)
            z[rng.permutation(M)[:size]] = 1
            key = z.tobytes()
            if key in seen:
                weights[seen[key]] += 1.0
            else:
                seen[key] = len(rows)
                rows.append(z)
                weights.append(1.0)
            drawn += 1
            if drawn < budget and size <= num_paired:
                zc = 1 - z
                kc = zc.tobytes()
                if kc in seen:
                    weights[seen[kc]] += 1.0
                else:
                    seen[kc] = len(rows)
                    rows.append(zc)
                    weights.append(1.0)
                drawn += 1
        # the sampled part shares the remaining weight mass
        wsum = sum(weights[nfixed:])
        if wsum > 0:
            scale = float(wv[full_sizes:].sum()) / wsum
            for i in range(nfixed, len(weights)):
                weights[i] *= scale
    return np.asarray(rows, np.uint8), np.asarray(weights, np.float64)


def wls_operator(Z: np.ndarray, w: np.ndarray):
    """(A [M-1, S], zlast [S]) of the efficiency-constrained WLS (last feature eliminated)."""
    Zf = Z.astype(np.float64)
    zM = Zf[:, -1]
    Xm = Zf[:, :-1] - zM[:, None]
    XtW = Xm.T * w[None, :]
    G = XtW @ Xm
    A = np.linalg.solve(G + 1e-12 * np.eye(G.shape[0]), XtW)
    return A, zM


def _link(v, link):
    if link == "logit":
        v = np.clip(v, 1e-12, 1 - 1e-12)
        return np.log(v / (1 - v))
    return v


def kernelshap_reference(X: np.ndarray, a: np.ndarray, bias: float, B: np.ndarray, Z: np.ndarray, A: np.ndarray,
                         zM: np.ndarray, link: str = "identity") -> tuple:
    """Vectorized fp64 oracle.  X [E, d] raw, B [n_bg, d] raw background, a/bias folded weights.
    link: "identity" (probabilities, shap default), "logit" (shap's logit link on the mean
    probability) or "logit_model" (explain the model's log-odds: equals LinearSHAP exactly).
    Returns (phi [E, d], fx [E], f0)."""
    X = np.asarray(X, np.float64)
    B = np.asarray(B, np.float64)
    d = X.shape[1]
    a = np.asarray(a, np.float64)[:d]
    Zf = Z.astype(np.float64)
    c = B @ a + bias                                 # [n_bg]
    U = a[None, None, :] * (X[:, None, :] - B[None, :, :])  # [E, n_bg, d]
    L = np.einsum("ebd,sd->ebs", U, Zf) + c[None, :, None]  # [E, n_bg, S]
    if link == "logit_model":
        f = L.mean(1)
        f0 = float(c.mean())
        fx = X @ a + bias
    else:
        f = (1.0 / (1.0 + np.exp(-L))).mean(1)
        f0 = float((1.0 / (1.0 + np.exp(-c))).mean())
        fx = 1.0 / (1.0 + np.exp(-(X @ a + bias)))
        f, f0, fx = _link(f, link), float(_link(np.asarray(f0), link)), _link(fx, link)
    y = f - f0
    delta = fx - f0
    phi = np.empty((X.shape[0], d))
    phi[:, :-1] = y @ A.T - np.outer(delta, A @ zM)
    phi[:, -1] = delta - phi[:, :-1].sum(1)
    return phi, fx, f0


# ------------------------------------------------------------------------------------------
# explainers
# ------------------------------------------------------------------------------------------
class LinearExplainer:
    """phi_i = w_i ((x_i - mu_i)/sigma_i - E_bg[(x_i - mu_i)/sigma_i]) on raw inputs, computed by
    the fused predict + SHAP kernel with the scaler folded into (a, c)."""

    def __init__(self, coef, intercept: float, mean, scale, background: np.ndarray | None = None, device="auto"):
        d = len(mean)
        w = np.zeros(32)
        w[:d] = coef
        w[30] = intercept
        bg_std = None
        if background is not None:
            bg_std = ((np.asarray(background, np.float64) - mean) / scale).mean(0)
        self.a, self.c, self.bias = P.fold_scaler(w, np.asarray(mean), np.asarray(scale), bg_std)
        self.d = d
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)
        self.expected_value = float(self.a[:d] @ self.c[:d] + self.bias)

    def shap_values(self, X) -> np.ndarray:
        Xt = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float32)).to(self.device)
        _, phi = P.predict_shap_raw(Xt, torch.from_numpy(self.a).to(self.device),
                                    torch.from_numpy(self.c).to(self.device), self.bias)
        return phi.cpu().numpy()


class KernelExplainer:
    def __init__(self, a: np.ndarray, bias: float, background: np.ndarray, nsamples: int | None = None,
                 link: str = "identity", seed: int = 0, device="auto"):
        B = np.asarray(background, np.float32)
        if B.shape[0] > 128:
            raise ValueError("at most 128 background rows (summarize larger sets, e.g. k-means)")
        self.d = B.shape[1]
        self.a = np.asarray(a, np.float64)
        self.bias = float(bias)
        self.B = B
        self.link = link
        self.Z, self.w = coalition_design(self.d, nsamples, seed)
        self.A, self.zM = wls_operator(self.Z, self.w)
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)
        self._dev_cache = None

    @property
    def nsamples(self) -> int:
        return self.Z.shape[0]

    def shap_values(self, X) -> np.ndarray:
        return self.explain(X)[0]

    def explain(self, X):
        """-> (phi [E, d], fx [E], f0)."""
        X = np.ascontiguousarray(X, np.float32)
        if self.device.type == "cuda":
            from ..ops.kernelshap import kernelshap

            return kernelshap(torch.from_numpy(X).to(self.device), self)
        return kernelshap_reference(X, self.a, self.bias, self.B, self.Z, self.A, self.zM, self.link)


def kernelshap_throughput(res, dev, comm=None, n_expl: int = 1000, n_bg: int = 100, reps: int = 5) -> dict:
    """bench.py extra: KernelSHAP values/s for 1k explanations/batch (DP: per-rank shards)."""
    from ..data.synthetic import separable

    a, c, b = res.folded()
    Xb, _ = separable(n_bg, seed=91, device="cpu")
    Xe, _ = separable(n_expl, seed=92 + (comm.rank if comm else 0), device="cpu")
    ke = KernelExplainer(a, b, Xb.numpy(), device=str(dev) if dev.type == "cuda" else "cpu")
    Xd = Xe.to(dev)
    from ..ops.kernelshap import kernelshap

    for _ in range(2):
        kernelshap(Xd, ke)
    if comm:
        comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        kernelshap(Xd, ke, sync=False)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if comm:
        dt = comm.max_over_ranks(dt)
    world = comm.world_size if comm else 1
    return {"kernelshap_values_per_sec": round(n_expl * ke.d * reps * world / dt, 1),
            "kernelshap_config": {"explanations_per_batch": n_expl * world, "coalitions": ke.nsamples,
                                  "background": n_bg, "link": ke.link}}
