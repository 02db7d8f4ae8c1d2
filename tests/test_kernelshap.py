"""KernelSHAP for every model family (models/explainers.py; SURVEY.md §2.3 K7, BASELINE config 4).

CPU: the three explainers agree with each other (linear fast path vs the generic masked-row
path; tree-ensemble walk vs the generic path over the same ensemble) and satisfy efficiency.
GPU: the linear MFMA kernel and the tree kernel match their fp64 oracles and are deterministic for
a given coalition-part count (the last-arriver reduction sums partials in part order).
"""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models import explainers as EX
from fraud_detection_amd.ops import gbdt as gb
from fraud_detection_amd.ops import reference_gbdt as RG


def _linear_model(d=30, seed=0):
    """Standardized-space weights folded onto raw features (as a served model: ops/predict.fold_scaler)."""
    rng = np.random.default_rng(seed)
    Xr, _ = separable(4000, seed=99)
    Xr = Xr.numpy().astype(np.float64)
    mean, std = Xr.mean(0), Xr.std(0)
    a = np.zeros(32)
    a[:d] = rng.normal(0, 0.4, d) / std
    return a, float(-2.0 - a[:d] @ mean)


def _tree_model(n=6000, trees=12, depth=5, seed=1):
    X, y = separable(n, fraud_rate=0.1, seed=seed)
    X = X.numpy()
    mean, scale = X.mean(0), X.std(0) + 1e-3
    Xs = EX._standardize(X, mean, scale)
    ens = gb.fit(torch.from_numpy(Xs), y, gb.GBDTParams(n_estimators=trees, max_depth=depth, learning_rate=0.3))
    return ens, mean, scale, X


def test_linear_matches_generic_function_path():
    a, bias = _linear_model()
    X, _ = separable(40, seed=3)
    B, _ = separable(20, seed=4)
    X, B = X.numpy(), B.numpy()
    ke = EX.KernelExplainer(a, bias, B, nsamples=300, device="cpu")
    phi, fx, f0 = ke.explain(X)
    fn = lambda R: torch.sigmoid(R.double() @ torch.from_numpy(a[:30]) + bias)  # noqa: E731
    fe = EX.FunctionKernelExplainer(fn, B, nsamples=300, device="cpu")
    phi2, fx2, f02 = fe.explain(X)
    np.testing.assert_allclose(phi, phi2, atol=1e-10)
    np.testing.assert_allclose(fx, fx2, atol=1e-12)
    assert abs(f0 - f02) < 1e-12
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-10)   # efficiency


@pytest.mark.parametrize("link", ["identity", "logit_model", "logit"])
def test_tree_walk_matches_generic_function_path(link):
    ens, mean, scale, Xall = _tree_model()
    X, B = Xall[:25], Xall[3000:3060]
    te = EX.TreeKernelExplainer(ens, mean, scale, B, nsamples=400, link=link, device="cpu")
    phi, fx, f0 = te.explain(X)

    def fn(R):
        Rs = EX._standardize(R.numpy(), mean, scale)
        m = RG.predict_margin(Rs, ens.feat, ens.thr, ens.leaf, ens.depth, ens.base_margin).astype(np.float64)
        return torch.from_numpy(m if link == "logit_model" else 1.0 / (1.0 + np.exp(-m)))

    fe = EX.FunctionKernelExplainer(fn, B, nsamples=400, link=link, device="cpu")
    phi2, fx2, f02 = fe.explain(X)
    np.testing.assert_allclose(phi, phi2, atol=1e-9)
    np.testing.assert_allclose(fx, fx2, atol=1e-12)
    assert abs(f0 - f02) < 1e-12
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-9)
    assert np.abs(phi).max() > 1e-4                                 # a non-trivial explanation


def test_tree_direction_bits_follow_predict():
    ens, mean, scale, Xall = _tree_model(trees=5, depth=3)
    Xs = EX._standardize(Xall[:500], mean, scale)
    m = EX._margins_from_bits(EX.tree_direction_bits(Xs, ens), ens)
    ref = RG.predict_margin(Xs, ens.feat, ens.thr, ens.leaf, ens.depth, ens.base_margin)
    assert np.array_equal(m, ref)


def test_design_cache_shared():
    a, bias = _linear_model()
    B = np.zeros((4, 30), np.float32)
    k1 = EX.KernelExplainer(a, bias, B, device="cpu")
    k2 = EX.KernelExplainer(a, bias + 1, B, device="cpu")
    assert k1.A is k2.A and k1.nsamples == 2 * 30 + 2048 - 6 or k1.nsamples > 2000


# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("link", ["identity", "logit_model"])
def test_linear_kernel_parts_bit_identical(dev, link):
    a, bias = _linear_model()
    X, _ = separable(300, seed=5)
    B, _ = separable(100, seed=6)
    ke = EX.KernelExplainer(a, bias, B.numpy(), link=link, device=str(dev))
    from fraud_detection_amd.ops.kernelshap import kernelshap

    Xd = X.to(dev)
    outs = [kernelshap(Xd, ke, parts=P) for P in (1, 2, 3, 8)]
    for P, o in zip((1, 2, 3, 8), outs):
        assert np.array_equal(o[0], kernelshap(Xd, ke, parts=P)[0])    # deterministic per part count
        scale = np.abs(outs[0][0]).max()                                # only the sum order differs
        np.testing.assert_allclose(o[0], outs[0][0], rtol=1e-5, atol=1e-6 * scale)
        assert np.array_equal(o[1], outs[0][1])
    ref = EX.kernelshap_reference(X.numpy(), ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, link)
    np.testing.assert_allclose(outs[0][0], ref[0], atol=2e-5)
    np.testing.assert_allclose(outs[0][0].sum(1), outs[0][1] - outs[0][2], atol=2e-5)
    again = kernelshap(Xd, ke)
    assert np.array_equal(again[0], kernelshap(Xd, ke)[0])          # deterministic (auto parts)


@pytest.mark.gpu
def test_linear_kernel_extreme_logits(dev):
    """Coalition logits below -88 overflow exp2 in the paired-reciprocal epilogue: the per-element
    fallback keeps the result finite.  (At |logit| ~ 100s the hi/lo bf16 split of u -- ~16
    mantissa bits per product -- bounds the accuracy, hence the looser tolerance here.)"""
    a, bias = _linear_model()
    a[:30] *= 40.0
    X, _ = separable(64, seed=7)
    B, _ = separable(100, seed=8)
    ke = EX.KernelExplainer(a, bias, B.numpy(), device=str(dev))
    from fraud_detection_amd.ops.kernelshap import kernelshap

    phi, fx, f0 = kernelshap(X.to(dev), ke)
    assert np.all(np.isfinite(phi))
    ref = EX.kernelshap_reference(X.numpy(), ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, "identity")
    assert np.min(ke.B @ ke.a[:30] + ke.bias) < -88 or np.min(X.numpy() @ ke.a[:30] + ke.bias) < -88
    np.testing.assert_allclose(phi, ref[0], atol=2e-3)
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("depth,trees,nbg", [(5, 30, 100), (3, 7, 37), (5, 300, 16)])
def test_tree_kernel_matches_oracle(dev, depth, trees, nbg):
    ens, mean, scale, Xall = _tree_model(trees=trees, depth=depth)
    X, B = Xall[:40], Xall[3000:3000 + nbg]
    te = EX.TreeKernelExplainer(ens, mean, scale, B, nsamples=500, device=str(dev))
    from fraud_detection_amd.ops.kernelshap import kernelshap_tree

    Xd = torch.from_numpy(X).to(dev)
    outs = [kernelshap_tree(Xd, te, parts=P) for P in (1, 4)]
    assert np.array_equal(outs[1][0], kernelshap_tree(Xd, te, parts=4)[0])
    np.testing.assert_allclose(outs[0][0], outs[1][0], atol=1e-6)
    phi, fx, f0 = outs[0]
    ref = EX.kernelshap_tree_reference(EX._standardize(X, mean, scale), te.Bs, ens, te.Z, te.A, te.zM)
    np.testing.assert_allclose(fx, ref[1], atol=1e-6)
    assert abs(f0 - ref[2]) < 1e-6
    np.testing.assert_allclose(phi, ref[0], atol=2e-5)
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-5)


# ---------------------------------------------------------------------------------------------
def _paired_emulation(X, ke, link):
    """numpy (fp64) emulation of the complement-paired layout: base logits from one GEMM,
    complement logits T_b - L_b(z) (here through sigma(1 - z) = E / (E + K_b), the same identity the
    kernel evaluates with a shifted exponent), null background rows padded to a multiple of 8 and
    removed again as the exact 1/2 per row, paired A layout."""
    from fraud_detection_amd.ops.kernelshap import complement_pairs

    d = ke.d
    base, comp = complement_pairs(ke.Z)
    Ppad = (len(base) + 31) // 32 * 32
    Zb = np.zeros((Ppad, d))
    Zb[: len(base)] = ke.Z[base]
    Ap = np.zeros((d - 1, 2 * Ppad))
    Ap[:, : len(base)] = ke.A[:, base]
    has = comp >= 0
    Ap[:, Ppad + np.nonzero(has)[0]] = ke.A[:, comp[has]]
    a = ke.a[:d]
    B = ke.B.astype(np.float64)
    nb = B.shape[0]
    nb_pad = (nb + 7) // 8 * 8
    c = np.zeros(nb_pad)
    c[:nb] = B @ a + ke.bias
    phis = []
    for x in np.asarray(X, np.float64):
        lx = x @ a + ke.bias
        U = np.zeros((nb_pad, d))
        U[:nb] = a * (x - B)
        L = Zb @ U.T + np.where(np.arange(nb_pad) < nb, c, 0.0)[None, :]        # [Ppad, nb_pad]
        T = np.where(np.arange(nb_pad) < nb, lx + c, 0.0)
        if link == "logit_model":
            fb = L[:, :nb].sum(1)
            fc = T[:nb].sum() - fb
            f0, fx = c[:nb].mean(), lx
        else:
            E = np.exp(-L)
            K = np.exp(-T)
            nulls = 0.5 * (nb_pad - nb)
            fb = (1.0 / (1.0 + E)).sum(1) - nulls
            fc = (E / (E + K[None, :])).sum(1) - nulls
            f0, fx = (1.0 / (1.0 + np.exp(-c[:nb]))).mean(), 1.0 / (1.0 + np.exp(-lx))
        y = np.r_[fb, fc] / nb - f0
        delta = fx - f0
        ph = np.empty(d)
        ph[:-1] = Ap @ y - (ke.A @ ke.zM) * delta
        ph[-1] = delta - ph[:-1].sum()
        phis.append(ph)
    return np.asarray(phis)


def test_complement_pairs_cover_design():
    from fraud_detection_amd.ops.kernelshap import complement_pairs

    Z, _, _, _ = EX.cached_design(30)
    base, comp = complement_pairs(Z)
    idx = np.r_[base, comp[comp >= 0]]
    assert np.array_equal(np.sort(idx), np.arange(len(Z)))             # every row exactly once
    assert np.array_equal(Z[comp[comp >= 0]], 1 - Z[base[comp >= 0]])
    assert len(base) <= len(Z) // 2 + 32                                # shap samples in pairs


@pytest.mark.parametrize("link", ["identity", "logit_model"])
def test_paired_arithmetic_matches_oracle(link):
    a, bias = _linear_model()
    X, _ = separable(6, seed=5)
    B, _ = separable(37, seed=6)                                        # 37 rows: 3 null rows padded
    ke = EX.KernelExplainer(a, bias, B.numpy(), link=link, device="cpu")
    ref = EX.kernelshap_reference(X.numpy(), ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, link)
    np.testing.assert_allclose(_paired_emulation(X.numpy(), ke, link), ref[0], atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("link", ["identity", "logit", "logit_model"])
def test_paired_kernel_matches_unpaired(dev, link, monkeypatch):
    """The complement-paired kernel (default) and the one-coalition-per-column kernel explain
    the same design: equal to fp32 rounding, both within the oracle tolerance."""
    a, bias = _linear_model()
    X, _ = separable(200, seed=11)
    B, _ = separable(100, seed=12)
    ke = EX.KernelExplainer(a, bias, B.numpy(), link=link, device=str(dev))
    from fraud_detection_amd.ops.kernelshap import kernelshap

    Xd = X.to(dev)
    pp = kernelshap(Xd, ke, paired=True)
    pu = kernelshap(Xd, ke, paired=False)
    ref = EX.kernelshap_reference(X.numpy(), ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, link)
    tol = 2e-4 if link == "logit" else 2e-5
    np.testing.assert_allclose(pp[0], ref[0], atol=tol)
    np.testing.assert_allclose(pp[0], pu[0], atol=tol)
    np.testing.assert_allclose(pp[1], pu[1], rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("paired", [True, False])
def test_linear_kernel_wide_logit_range(dev, paired):
    """The shipped reference LR on Kaggle-like raw rows: explanation and background logits span
    -33..31, so pair products of the sigmoid epilogue overflow (a background logit T_b below -44,
    or one coalition logit below -44 next to a moderate one).  Such tiles must take the
    per-element path instead of losing the partner's sigma."""
    from _models import kaggle_like_rows
    from fraud_detection_amd.compat.safe_joblib import decode_logistic, decode_scaler
    from fraud_detection_amd.ops import predict as P
    from fraud_detection_amd.ops.kernelshap import kernelshap

    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    m = decode_logistic(os.path.join(root, "models", "logistic_model.joblib"))
    s = decode_scaler(os.path.join(root, "models", "scaler.joblib"))
    w = np.zeros(32)
    w[:30] = m["coef"].ravel()
    w[30] = float(m["intercept"].ravel()[0])
    a, _, bias = P.fold_scaler(w, s["mean_"], s["scale_"], None)
    B, X = kaggle_like_rows(100, seed=1), kaggle_like_rows(96, seed=5)
    ke = EX.KernelExplainer(a, bias, B, device=str(dev))
    phi, fx, f0 = kernelshap(torch.from_numpy(X).to(dev), ke, paired=paired)
    ref = EX.kernelshap_reference(X, ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, "identity")
    np.testing.assert_allclose(phi, ref[0], atol=5e-6)
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=2e-6)
