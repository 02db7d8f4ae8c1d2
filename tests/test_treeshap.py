"""Interventional TreeSHAP (GBDT family explainer): the numpy oracle of treeshap.hip's algorithm
against brute-force exact Shapley values, efficiency, and agreement with exact (fully
enumerated) KernelSHAP on the margin -- two independent algorithms, one answer."""
import itertools
import math

import numpy as np
import pytest

from fraud_detection_amd.models.explainers import (
    KernelExplainer, _margins_from_bits, cached_design, kernelshap_tree_reference, tree_direction_bits,
    treeshap_reference,
)
from fraud_detection_amd.ops.gbdt import TreeEnsemble


def random_ensemble(d, depth, T, seed, p_pass=0.15):
    rng = np.random.default_rng(seed)
    ni = (1 << depth) - 1
    feat = rng.integers(0, d, (T, ni)).astype(np.int32)
    feat[rng.random((T, ni)) < p_pass] = -1  # pass-through nodes
    thr = rng.normal(0, 0.7, (T, ni)).astype(np.float32)
    thr[feat < 0] = np.inf
    leaf = rng.normal(0, 0.3, (T, 1 << depth)).astype(np.float32)
    return TreeEnsemble(depth=depth, feat=feat, bin=np.zeros_like(feat), thr=thr, gain=np.zeros(feat.shape),
                        leaf=leaf, cuts=np.zeros((d, 256), np.float32), nbins=np.full(d, 256, np.int32),
                        base_score=0.3)


def exact_shapley(Xs, Bs, ens):
    """Brute force over all 2^d coalitions of v(S) = mean_b margin(x_S, z_~S)."""
    E, d = Xs.shape
    masks = np.array(list(itertools.product([0, 1], repeat=d)), bool)  # [2^d, d]
    phi = np.zeros((E, d))
    w = {s: math.factorial(s) * math.factorial(d - s - 1) / math.factorial(d) for s in range(d)}
    for e in range(E):
        hyb = np.where(masks[:, None, :], Xs[e][None, None, :], Bs[None, :, :])  # [2^d, nb, d]
        m = _margins_from_bits(tree_direction_bits(hyb.reshape(-1, d), ens), ens).astype(np.float64)
        v = m.reshape(len(masks), -1).mean(1)
        idx = {tuple(mk): i for i, mk in enumerate(masks)}
        for i in range(d):
            for k, mk in enumerate(masks):
                if mk[i]:
                    continue
                with_i = mk.copy()
                with_i[i] = True
                phi[e, i] += w[int(mk.sum())] * (v[idx[tuple(with_i)]] - v[k])
    return phi


@pytest.mark.parametrize("d,depth,T,seed", [(4, 3, 6, 0), (6, 5, 8, 1), (7, 4, 12, 2), (5, 5, 20, 3)])
def test_treeshap_equals_brute_force_shapley(d, depth, T, seed):
    ens = random_ensemble(d, depth, T, seed)
    rng = np.random.default_rng(seed + 10)
    Xs = rng.normal(size=(3, d)).astype(np.float32)
    Bs = rng.normal(size=(5, d)).astype(np.float32)
    phi, fx, f0 = treeshap_reference(Xs, Bs, ens)
    np.testing.assert_allclose(phi, exact_shapley(Xs, Bs, ens), atol=1e-6)  # brute force sums fp32 margins
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-6)  # efficiency (fx, f0: fp32 tree sums)


def test_treeshap_matches_exact_kernelshap_on_the_margin():
    """KernelSHAP with every coalition enumerated (d = 8: 254 <= nsamples) is exact Shapley too."""
    d = 8
    ens = random_ensemble(d, 5, 15, 7)
    rng = np.random.default_rng(8)
    Xs = rng.normal(size=(4, d)).astype(np.float32)
    Bs = rng.normal(size=(6, d)).astype(np.float32)
    Z, _, A, zM = cached_design(d, 4096, 0)
    assert Z.shape[0] == 2 ** d - 2
    phi_k, _, _ = kernelshap_tree_reference(Xs, Bs, ens, Z, A, zM, link="logit_model")
    phi_t, _, _ = treeshap_reference(Xs, Bs, ens)
    np.testing.assert_allclose(phi_t, phi_k, atol=1e-6)


def test_tree_explainer_cpu_path_on_raw_rows():
    from fraud_detection_amd.models.explainers import TreeExplainer, _standardize

    d = 6
    ens = random_ensemble(d, 4, 10, 4)
    rng = np.random.default_rng(5)
    mean, scale = rng.normal(size=d) * 10, rng.uniform(0.5, 3, d)
    B = (rng.normal(size=(7, d)) * scale + mean).astype(np.float32)
    X = (rng.normal(size=(3, d)) * scale + mean).astype(np.float32)
    te = TreeExplainer(ens, mean, scale, B, device="cpu")
    phi, fx, f0 = te.explain(X)
    ref = treeshap_reference(_standardize(X, mean, scale), _standardize(B, mean, scale), ens)
    np.testing.assert_allclose(phi, ref[0], atol=1e-12)
    assert f0 == pytest.approx(te.expected_value)
    np.testing.assert_allclose(phi.sum(1), fx - f0, atol=1e-6)
