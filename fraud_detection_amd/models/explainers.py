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

Model-agnostic paths (shap.KernelExplainer takes any model; reference train_model.py:95-113 ships an
XGBoost model):
  * ``TreeKernelExplainer`` -- the GBDT family: every masked row z * x + (1 - z) * B_b is walked
    through the ensemble inside the kernel (kernelshap_tree_kernel), never materialised;
  * ``TreeExplainer`` -- interventional TreeSHAP of the GBDT margin: exact, no coalition sampling
    (treeshap.hip), orders of magnitude less work than KernelSHAP on trees;
  * ``FunctionKernelExplainer`` -- any callable on device tensors (e.g. a torch model): masked rows
    are built in chunks on the device, the model is called on them, and the shared WLS operator
    projects the coalition values.
All three share one cached coalition design per (M, nsamples, seed).
"""
from __future__ import annotations

import functools
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


@functools.lru_cache(maxsize=16)
def cached_design(M: int, nsamples: int | None = None, seed: int = 0):
    """(Z, w, A, zM) for a design, solved once per process (read-only arrays)."""
    Z, w = coalition_design(M, nsamples, seed)
    A, zM = wls_operator(Z, w)
    for v in (Z, w, A, zM):
        v.setflags(write=False)
    return Z, w, A, zM


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
        self.Z, self.w, self.A, self.zM = cached_design(self.d, nsamples or None, seed)
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


def _project(f, f0, fx, A, zM):
    """Efficiency-constrained WLS projection of coalition values f [E, S] (fp64 numpy)."""
    y = f - f0
    delta = fx - f0
    phi = np.empty((f.shape[0], A.shape[0] + 1))
    phi[:, :-1] = y @ A.T - np.outer(delta, A @ zM)
    phi[:, -1] = delta - phi[:, :-1].sum(1)
    return phi


def _standardize(X, mean, scale) -> np.ndarray:
    """The device scaler's arithmetic ((x - mean32) * inv32 in fp32, ops/reference.scale_cast)."""
    d = len(mean)
    m32 = np.asarray(mean, np.float64).astype(np.float32)
    i32 = (1.0 / np.asarray(scale, np.float64)).astype(np.float32)
    return ((np.asarray(X, np.float32)[:, :d] - m32[None, :]) * i32[None, :]).astype(np.float32)


def tree_direction_bits(Xs: np.ndarray, ens) -> np.ndarray:
    """uint32 [T, n]: bit n+1 set where row goes right at internal node n (1-based heap; the
    kernel's convention).  Pass-through nodes (feat -1) go left."""
    Xs = np.asarray(Xs, np.float32)
    T, ni = ens.feat.shape
    if ni > 31:
        raise ValueError("tree KernelSHAP supports depth <= 5")
    out = np.zeros((T, Xs.shape[0]), np.uint32)
    for n in range(ni):
        f = ens.feat[:, n]
        v = Xs[:, np.maximum(f, 0)].T                       # [T, n]
        right = (f[:, None] >= 0) & ~(v < ens.thr[:, n][:, None])
        out |= right.astype(np.uint32) << np.uint32(n + 1)
    return out


def _margins_from_bits(R1: np.ndarray, ens) -> np.ndarray:
    """float32 margins (tree order, as the kernel) from direction bits R1 [T, ...]."""
    D = ens.depth
    node = np.ones(R1.shape[1:], np.int64)
    m = np.full(R1.shape[1:], np.float32(ens.base_margin), np.float32)
    for t in range(R1.shape[0]):
        node[...] = 1
        for _ in range(D):
            node = (node << 1) | ((R1[t] >> node.astype(np.uint32)) & 1).astype(np.int64)
        m = (m + ens.leaf[t][node - (1 << D)]).astype(np.float32)
    return m


def kernelshap_tree_reference(Xs: np.ndarray, Bs: np.ndarray, ens, Z: np.ndarray, A: np.ndarray, zM: np.ndarray,
                              link: str = "identity") -> tuple:
    """fp64 oracle of the tree path on STANDARDIZED rows: f(z) = mean_b link(model(z x + (1-z) B_b))
    with float32 margins summed in tree order (the kernel's and the predict kernel's order)."""
    Xs = np.asarray(Xs, np.float32)
    Bs = np.asarray(Bs, np.float32)
    bw = tree_direction_bits(Bs, ens)                      # [T, nb]
    xw = tree_direction_bits(Xs, ens)                      # [T, E]
    T, ni = ens.feat.shape
    fidx = np.maximum(ens.feat, 0)
    zb = Z.astype(bool)
    # node z-bits per (tree, coalition): Zt[t, s] bit n+1 = z_s[feat[t, n]]
    Zt = np.zeros((T, Z.shape[0]), np.uint32)
    for n in range(ni):
        Zt |= zb[:, fidx[:, n]].T.astype(np.uint32) << np.uint32(n + 1)
    sig = (lambda v: v.astype(np.float64)) if link == "logit_model" else (lambda v: 1.0 / (1.0 + np.exp(-v.astype(np.float64))))
    f0 = float(np.mean(sig(_margins_from_bits(bw, ens))))
    mx = _margins_from_bits(xw, ens).astype(np.float64)
    fx = mx if link == "logit_model" else 1.0 / (1.0 + np.exp(-mx))
    f = np.empty((Xs.shape[0], Z.shape[0]))
    for e in range(Xs.shape[0]):
        R1 = (Zt[:, :, None] & xw[:, e][:, None, None]) | (~Zt[:, :, None] & bw[:, None, :])  # [T, S, nb]
        f[e] = sig(_margins_from_bits(R1, ens)).mean(1)
    if link == "logit":
        f, f0, fx = _link(f, link), float(_link(np.asarray(f0), link)), _link(fx, link)
    return _project(f, f0, fx, A, zM), fx, f0


class TreeKernelExplainer:
    """KernelSHAP of a tree ensemble (ops/gbdt.TreeEnsemble trained on standardized rows) over RAW
    inputs: the model is standardize -> ensemble, as served.  Background: <= 128 raw rows."""

    def __init__(self, ens, mean, scale, background: np.ndarray, nsamples: int | None = None,
                 link: str = "identity", seed: int = 0, device="auto"):
        B = np.asarray(background, np.float32)
        if B.shape[0] > 128:
            raise ValueError("at most 128 background rows (summarize larger sets)")
        if ens.depth > 5:
            raise ValueError("tree KernelSHAP supports depth <= 5 (the reference trains max_depth=5)")
        self.ens = ens
        self.d = B.shape[1]
        self.mean = np.asarray(mean, np.float64)
        self.scale = np.asarray(scale, np.float64)
        self.B = B
        self.Bs = _standardize(B, self.mean, self.scale)
        self.bw = tree_direction_bits(self.Bs, ens)         # [T, n_bg]
        self.link = link
        self.Z, self.w, self.A, self.zM = cached_design(self.d, nsamples or None, seed)
        self.zmasks = (self.Z.astype(np.uint64) << np.arange(self.d, dtype=np.uint64)[None, :]).sum(1).astype(np.uint32)
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)
        self._dev_cache = None

    @property
    def nsamples(self) -> int:
        return self.Z.shape[0]

    def shap_values(self, X) -> np.ndarray:
        return self.explain(X)[0]

    def explain(self, X):
        """-> (phi [E, d], fx [E], f0) in the link's space (identity: probabilities)."""
        X = np.ascontiguousarray(X, np.float32)
        if self.device.type == "cuda":
            from ..ops.kernelshap import kernelshap_tree

            return kernelshap_tree(torch.from_numpy(X).to(self.device), self)
        return kernelshap_tree_reference(_standardize(X, self.mean, self.scale), self.Bs, self.ens, self.Z, self.A,
                                         self.zM, self.link)


def _treeshap_weights(depth: int):
    """(Wpos, Wneg) [depth+1, depth+1]: (a-1)! b! / (a+b)! and a! (b-1)! / (a+b)!."""
    f = [math.factorial(i) for i in range(2 * depth + 2)]
    wp = np.zeros((depth + 1, depth + 1))
    wn = np.zeros((depth + 1, depth + 1))
    for a in range(depth + 1):
        for b in range(depth + 1 - a):
            if a:
                wp[a, b] = f[a - 1] * f[b] / f[a + b]
            if b:
                wn[a, b] = f[a] * f[b - 1] / f[a + b]
    return wp, wn


def treeshap_reference(Xs: np.ndarray, Bs: np.ndarray, ens) -> tuple:
    """fp64 oracle of interventional TreeSHAP on STANDARDIZED rows (treeshap.hip's algorithm):
    per (x, background z, tree) a depth-first walk over the leaves some hybrid x_S z_~S reaches,
    leaf value v with A (features taken from x where z goes the other way) and B (vice versa)
    contributes v (a-1)! b! / (a+b)! to every i in A and -v a! (b-1)! / (a+b)! to every i in B.
    Returns (phi [E, d] of the margin, margin(x) [E], f0 = mean background margin)."""
    Xs = np.asarray(Xs, np.float32)
    Bs = np.asarray(Bs, np.float32)
    xw = tree_direction_bits(Xs, ens)
    bw = tree_direction_bits(Bs, ens)
    D = ens.depth
    wp, wn = _treeshap_weights(D)
    E, d = Xs.shape
    nb = Bs.shape[0]
    phi = np.zeros((E, d))

    def walk(t, k, level, A, B, xb, zb, acc):
        if level == D:
            if A or B:
                v = float(ens.leaf[t, k - (1 << D)])
                a, b = bin(A).count("1"), bin(B).count("1")
                for i in range(d):
                    if A >> i & 1:
                        acc[i] += v * wp[a, b]
                    if B >> i & 1:
                        acc[i] -= v * wn[a, b]
            return
        f = int(ens.feat[t, k - 1])
        if f < 0:
            return walk(t, 2 * k, level + 1, A, B, xb, zb, acc)
        dx, dz = (xb >> k) & 1, (zb >> k) & 1
        bit = 1 << f
        if dx == dz or A & bit:
            return walk(t, 2 * k + dx, level + 1, A, B, xb, zb, acc)
        if B & bit:
            return walk(t, 2 * k + dz, level + 1, A, B, xb, zb, acc)
        walk(t, 2 * k + dx, level + 1, A | bit, B, xb, zb, acc)
        walk(t, 2 * k + dz, level + 1, A, B | bit, xb, zb, acc)

    for e in range(E):
        acc = np.zeros(d)
        for b in range(nb):
            for t in range(ens.n_trees):
                walk(t, 1, 0, 0, 0, int(xw[t, e]), int(bw[t, b]), acc)
        phi[e] = acc / nb
    fx = _margins_from_bits(xw, ens).astype(np.float64)
    f0 = float(np.mean(_margins_from_bits(bw, ens).astype(np.float64)))
    return phi, fx, f0


class TreeExplainer:
    """Interventional TreeSHAP of a tree ensemble (ops/gbdt.TreeEnsemble on standardized rows)
    over RAW inputs, in margin (log-odds) space -- shap.TreeExplainer(model, data=background,
    feature_perturbation="interventional") semantics, exact (no coalition sampling): the fast
    explainer of the GBDT family (csrc/kernels/treeshap.hip).  Background: <= 1024 raw rows."""

    link = "logit_model"

    def __init__(self, ens, mean, scale, background: np.ndarray, device="auto"):
        B = np.asarray(background, np.float32)
        if B.shape[0] < 1 or B.shape[0] > 1024:
            raise ValueError("1..1024 background rows")
        if ens.depth > 5:
            raise ValueError("TreeSHAP kernel supports depth <= 5 (the reference trains max_depth=5)")
        self.ens = ens
        self.d = B.shape[1]
        self.mean = np.asarray(mean, np.float64)
        self.scale = np.asarray(scale, np.float64)
        self.B = B
        self.Bs = _standardize(B, self.mean, self.scale)
        self.bw = tree_direction_bits(self.Bs, ens)
        # expected value: mean background margin (float32 tree-order sums, as the predict kernel)
        self.f0 = float(np.mean(_margins_from_bits(self.bw, ens).astype(np.float64)))
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)
        self._dev_cache = None

    @property
    def expected_value(self) -> float:
        return self.f0

    def shap_values(self, X) -> np.ndarray:
        return self.explain(X)[0]

    def explain(self, X):
        """-> (phi [E, d], margin(x) [E], f0) in log-odds space; sum(phi) = margin(x) - f0."""
        X = np.ascontiguousarray(X, np.float32)
        if self.device.type == "cuda":
            from ..ops.treeshap import treeshap

            return treeshap(torch.from_numpy(X).to(self.device), self)
        return treeshap_reference(_standardize(X, self.mean, self.scale), self.Bs, self.ens)


class FunctionKernelExplainer:
    """KernelSHAP of any model given as ``fn(rows: Tensor[N, d]) -> Tensor[N]`` (the model output
    in the link's input space: probabilities for identity / logit, log-odds for logit_model).
    Masked rows are formed on ``device`` in chunks of explanations and the coalition values are
    projected with the shared WLS operator (a plain GEMM: hipBLASLt through torch)."""

    def __init__(self, fn, background: np.ndarray, nsamples: int | None = None, link: str = "identity",
                 seed: int = 0, device="auto", max_rows_per_call: int = 1 << 24):
        self.fn = fn
        self.B = np.asarray(background, np.float32)
        self.d = self.B.shape[1]
        self.link = link
        self.Z, self.w, self.A, self.zM = cached_design(self.d, nsamples or None, seed)
        self.device = torch.device("cuda", 0) if (device == "auto" and torch.cuda.is_available()) else torch.device(
            "cpu" if device == "auto" else device)
        self.max_rows = max_rows_per_call

    @property
    def nsamples(self) -> int:
        return self.Z.shape[0]

    def shap_values(self, X) -> np.ndarray:
        return self.explain(X)[0]

    @torch.no_grad()
    def explain(self, X):
        dev = self.device
        X = torch.as_tensor(np.ascontiguousarray(X, np.float32), device=dev)
        B = torch.from_numpy(self.B).to(dev)
        Z = torch.from_numpy(self.Z.astype(np.float32)).to(dev)            # [S, d]
        E, S, nb = X.shape[0], Z.shape[0], B.shape[0]
        f0 = float(self.fn(B).double().mean())
        fx = self.fn(X).double()
        per = max(1, self.max_rows // (S * nb))
        f = torch.empty((E, S), dtype=torch.float64, device=dev)
        for e0 in range(0, E, per):
            xe = X[e0:e0 + per]                                             # [c, d]
            rows = Z[None, :, None, :] * xe[:, None, None, :] + (1 - Z)[None, :, None, :] * B[None, None, :, :]
            out = self.fn(rows.reshape(-1, self.d)).double().reshape(xe.shape[0], S, nb)
            f[e0:e0 + per] = out.mean(2)
        f, fx = f.cpu().numpy(), fx.cpu().numpy()
        if self.link == "logit":
            f, f0, fx = _link(f, "logit"), float(_link(np.asarray(f0), "logit")), _link(fx, "logit")
        return _project(f, f0, fx, self.A, self.zM), fx, f0


def kernelshap_throughput(res, dev, comm=None, n_expl: int = 1000, n_bg: int = 100, reps: int = 100) -> dict:
    """bench.py extra: KernelSHAP values/s for 1k explanations/batch (DP: per-rank shards), the
    steady state of a loaded XAI worker.  ~20 ms of back-to-back batches first: the GPU clock
    ramps over milliseconds, and after only 10 warm-up batches (0.6 ms) a 55 us batch measured
    61-63 us (profiles/r2_s5h)."""
    from ..data.synthetic import separable

    a, c, b = res.folded()
    Xb, _ = separable(n_bg, seed=91, device="cpu")
    Xe, _ = separable(n_expl, seed=92 + (comm.rank if comm else 0), device="cpu")
    ke = KernelExplainer(a, b, Xb.numpy(), device=str(dev) if dev.type == "cuda" else "cpu")
    Xd = Xe.to(dev)
    from ..ops.kernelshap import kernelshap

    kernelshap(Xd, ke)
    for _ in range(300):
        kernelshap(Xd, ke, sync=False)
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
