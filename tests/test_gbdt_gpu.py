"""K11 GBDT kernels on the GPU vs the numpy oracle (ops/reference_gbdt.py).

Integer histograms make the comparison exact: bins, quantised gradients of the first round,
every split of the first tree and the training/inference margins must match bit for bit; later
rounds agree to fp64-libm rounding of the gradients."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.ops import gbdt as gb
from fraud_detection_amd.ops import reference_gbdt as R

pytestmark = pytest.mark.gpu


def _data(n, d, seed=0, dev="cuda"):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    X[:, 1] = np.round(X[:, 1] * 3) / 3  # a few-valued feature (few bins, many ties)
    logit = 1.2 * X[:, 0] - 1.5 * (X[:, 1] > 0.3) + X[:, 2] * X[:, 3] - 3.0
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.uint8)
    return torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev), X, y


def test_bin_kernel_exact(dev):
    Xd, _, X, _ = _data(100_003, 30)
    cuts, nb = R.quantile_cuts(X[::7], 256)
    got = gb.bin_rows(Xd, cuts, nb).cpu().numpy()
    assert np.array_equal(got, R.bin_rows(X, cuts, nb))


def test_bin_kernel_strided_rows(dev):
    Xd, _, X, _ = _data(20_000, 30)
    pad = torch.zeros((20_000, 32), device=dev)
    pad[:, :30] = Xd
    cuts, nb = R.quantile_cuts(X, 64)
    got = gb.bin_rows(pad[:, :30], cuts, nb).cpu().numpy()
    assert np.array_equal(got, R.bin_rows(X, cuts, nb))


@pytest.mark.parametrize("n,d,sample,max_bin", [(300_001, 30, 1 << 16, 256), (5_000, 3, 1 << 20, 256),
                                                 (70_000, 17, 9_999, 37), (1, 2, 1 << 20, 256)])
def test_quantile_select_matches_sort(dev, n, d, sample, max_bin):
    """quantile.hip radix select == np.sort of the same strided sample, bit for bit: ties, a constant
    feature, signed zeros, huge / tiny magnitudes, infinities."""
    rng = np.random.default_rng(n)
    X = rng.normal(size=(n, d)).astype(np.float32)
    X[:, 0] = np.round(X[:, 0] * 3) / 3
    if d > 2:
        X[:, 1] = 7.25                               # constant: every target in one bucket
        X[:, 2] = np.where(rng.random(n) < 0.5, -0.0, 0.0) * rng.integers(0, 2, n)
    if d > 5:
        X[:, 3] *= 1e30
        X[:, 4] *= 1e-30
        X[::97, 5] = np.inf
        X[::89, 5] = -np.inf
    Xd = torch.from_numpy(X).to(dev)
    got = gb.quantile_cuts(Xd, max_bin, sample_rows=sample)
    per = max(1, sample)
    stride = max(1, n // per)
    ref = R.quantile_cuts(X[::stride][:per], max_bin)
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0], ref[0])


def test_quantile_select_padded_rows(dev):
    """The pipeline's [n, 32] table: the select reads the 30 features through the row stride."""
    Xd, _, X, _ = _data(123_457, 30)
    pad = torch.zeros((123_457, 32), device=dev)
    pad[:, :30] = Xd
    got = gb.quantile_cuts(pad[:, :30], 256, sample_rows=50_000)
    stride = 123_457 // 50_000
    ref = R.quantile_cuts(X[::stride][:50_000], 256)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])


@pytest.mark.parametrize("spw", [1.0, 37.5])
def test_grad_kernel_matches_oracle(dev, spw):
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    n = 50_000
    rng = np.random.default_rng(1)
    margin = rng.normal(scale=3.0, size=n).astype(np.float32)
    y = (rng.random(n) < 0.3).astype(np.uint8)
    gs, hs = R.grad_scales(spw)
    md, yd = torch.from_numpy(margin).to(dev), torch.from_numpy(y).to(dev)
    gh = torch.empty((n, 2), dtype=torch.int16, device=dev)  # (g, h) packed per row
    native().gbdt_grad(ptr(md), ptr(yd), n, spw, gs, hs, ptr(gh), stream_of(md))
    ref = R.gradients(margin, y, spw, gs, hs)
    diff = np.abs(gh.cpu().numpy().astype(np.int64) - ref)
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3


@pytest.mark.parametrize("n,d,depth", [(60_000, 30, 5), (5_000, 7, 3), (777, 4, 6), (3_000, 5, 7)])
def test_first_tree_exact(dev, n, d, depth):
    """Round 1 (margin 0 -> exactly representable gradients): the device tree equals the oracle."""
    Xd, yd, X, y = _data(n, d, seed=n)
    p = gb.GBDTParams(n_estimators=1, max_depth=depth, scale_pos_weight=3.0)
    cuts = R.quantile_cuts(X, 256)
    ens, margin = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True)
    ref, rmargin = gb.fit(torch.from_numpy(X), torch.from_numpy(y), p, cuts=cuts, return_margin=True)
    assert np.array_equal(ens.feat, ref.feat) and np.array_equal(ens.bin, ref.bin)
    assert np.array_equal(ens.thr, ref.thr)
    assert np.array_equal(ens.gain, ref.gain)
    assert np.array_equal(ens.leaf, ref.leaf)
    assert np.array_equal(margin.cpu().numpy(), rmargin.numpy())


def test_boosting_matches_oracle(dev):
    Xd, yd, X, y = _data(80_000, 12, seed=5)
    p = gb.GBDTParams(n_estimators=12, max_depth=5, scale_pos_weight=5.0)
    cuts = R.quantile_cuts(X, 256)
    ens, margin = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True)
    ref, rmargin = gb.fit(torch.from_numpy(X), torch.from_numpy(y), p, cuts=cuts, return_margin=True)
    same = np.all(ens.feat == ref.feat, axis=1) & np.all(ens.bin == ref.bin, axis=1)
    assert same.mean() >= 0.9  # fp64 libm rounding may flip an isolated near-tie late on
    np.testing.assert_allclose(margin.cpu().numpy(), rmargin.numpy(), atol=2e-3)


def test_predict_kernel_exact_and_training_margins(dev):
    Xd, yd, X, y = _data(40_000, 30, seed=9)
    ens, margin = gb.fit(Xd, yd, gb.GBDTParams(n_estimators=20, max_depth=5), return_margin=True)
    got = gb.predict_margin(Xd, ens)
    assert torch.equal(got, margin)  # bins in training == float thresholds at inference
    ref = R.predict_margin(X, ens.feat, ens.thr, ens.leaf, ens.depth, ens.base_margin)
    assert np.array_equal(got.cpu().numpy(), ref)


def test_predict_many_trees_chunks_lds(dev):
    Xd, yd, X, y = _data(3_000, 8, seed=2)
    ens = gb.fit(Xd, yd, gb.GBDTParams(n_estimators=150, max_depth=6))  # > 1 LDS chunk of trees
    ref = R.predict_margin(X, ens.feat, ens.thr, ens.leaf, ens.depth, ens.base_margin)
    assert np.array_equal(gb.predict_margin(Xd, ens).cpu().numpy(), ref)


def test_gbdt_pipeline_gpu_quality(dev):
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.gbdt import GBDTPipeline
    from fraud_detection_amd.models.pipeline import TrainConfig

    X, y = separable(400_000, seed=21, device=dev)
    Xt, yt = separable(100_000, seed=22, device=dev)
    res = GBDTPipeline(TrainConfig(), gb.GBDTParams(n_estimators=100, max_depth=5)).fit(X, y)
    ev = res.evaluate(Xt, yt)
    assert ev["auc"] > 0.93, ev
    assert res.n_train_rows == 2 * (400_000 - int(y.sum()))


def test_gbdt_device_resume_bit_identical(dev, tmp_path):
    from fraud_detection_amd.utils.checkpoint import CheckpointManager

    Xd, yd, X, y = _data(30_000, 10, seed=13)
    p10 = gb.GBDTParams(n_estimators=10, max_depth=4)
    cuts = R.quantile_cuts(X, 256)
    full = gb.fit(Xd, yd, p10, cuts=cuts)
    mgr = CheckpointManager(str(tmp_path), prefix="g")
    gb.fit(Xd, yd, gb.GBDTParams(n_estimators=4, max_depth=4), cuts=cuts, checkpoint=mgr, checkpoint_every=2)
    res = gb.fit(Xd, yd, p10, cuts=cuts, checkpoint=mgr, checkpoint_every=2)
    for k in ("feat", "bin", "thr", "leaf"):
        assert np.array_equal(getattr(res, k), getattr(full, k)), k


def test_hist_multi_flush_bit_identical(dev, monkeypatch):
    """A histogram block flushes its packed LDS words to its slot every HIST_FLUSH_ROWS rows (the
    bound that keeps (h << 32) + g exact); flushing every 1000 rows -- many flushes per block,
    accumulated into the same slot -- gives the same trees bit for bit, and so does the oracle."""
    Xd, yd, X, y = _data(120_000, 30, seed=15)
    p = gb.GBDTParams(n_estimators=3, max_depth=5)
    cuts = R.quantile_cuts(X, 256)
    a, ma = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True)
    monkeypatch.setattr(gb, "HIST_FLUSH_ROWS", 1000)
    b, mb = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True)
    for k in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert torch.equal(ma, mb)
    ref = gb.fit(torch.from_numpy(X), torch.from_numpy(y), gb.GBDTParams(n_estimators=1, max_depth=5), cuts=cuts)
    assert np.array_equal(a.feat[0], ref.feat[0]) and np.array_equal(a.bin[0], ref.bin[0])


@pytest.mark.parametrize("var", [1, 2, 3])
def test_hist_variants_bit_identical(dev, var):
    """The histogram kernel's variants (rotated features; split int32 g/h adds; eight lanes per row,
    conflict-free bin-major slots -- the default) build the same integer histograms, so the trees and
    margins are bit-identical to the lockstep form."""
    from fraud_detection_amd.ops.native import native

    Xd, yd, X, y = _data(150_000, 30, seed=16)
    p = gb.GBDTParams(n_estimators=3, max_depth=5)
    cuts = R.quantile_cuts(X, 256)
    m = native()
    try:
        m.set_gbdt_hist_variant(0)
        a, ma = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True, use_graph=False)
        m.set_gbdt_hist_variant(var)
        b, mb = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True, use_graph=False)
    finally:
        m.set_gbdt_hist_variant(-1)
    for k in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert torch.equal(ma, mb)


def test_gbdt_deterministic_runs(dev):
    Xd, yd, X, y = _data(50_000, 30, seed=14)
    p = gb.GBDTParams(n_estimators=8, max_depth=5)
    a, ma = gb.fit(Xd, yd, p, return_margin=True)
    b, mb = gb.fit(Xd, yd, p, return_margin=True)
    assert np.array_equal(a.leaf, b.leaf) and torch.equal(ma, mb)


def test_gbdt_hipgraph_replay_bit_identical(dev):
    Xd, yd, X, y = _data(200_000, 30, seed=15)
    cuts = R.quantile_cuts(X, 256)
    p = gb.GBDTParams(n_estimators=12, max_depth=5)
    g_ens, g_m = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True, use_graph=True)
    e_ens, e_m = gb.fit(Xd, yd, p, cuts=cuts, return_margin=True, use_graph=False)
    for k in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(g_ens, k), getattr(e_ens, k)), k
    assert torch.equal(g_m, e_m)


@pytest.mark.parametrize("depth,n_bg", [(5, 32), (3, 7)])
def test_treeshap_kernel_matches_oracle(dev, depth, n_bg):
    """Interventional TreeSHAP on the device (treeshap.hip) vs the fp64 oracle of the same
    algorithm (exact vs brute-force Shapley in tests/test_treeshap.py): same attributions to fp32
    accumulation order, efficiency, bitwise run-to-run determinism."""
    from fraud_detection_amd.models.explainers import TreeExplainer

    Xd, yd, X, _ = _data(60_000, 30, seed=31)
    ens = gb.fit(Xd, yd, gb.GBDTParams(n_estimators=40, max_depth=depth))
    mean, scale = X.mean(0).astype(np.float64), X.std(0).astype(np.float64)
    raw = (X * scale + mean).astype(np.float32)  # the explainer standardizes raw rows
    te_g = TreeExplainer(ens, mean, scale, raw[:n_bg], device=str(dev))
    te_c = TreeExplainer(ens, mean, scale, raw[:n_bg], device="cpu")
    rows = raw[1000:1012]
    pg, fg, f0g = te_g.explain(rows)
    pc, fc, f0c = te_c.explain(rows)
    np.testing.assert_allclose(pg, pc, atol=2e-5)
    np.testing.assert_allclose(fg, fc, atol=1e-5)
    assert f0g == pytest.approx(f0c)
    np.testing.assert_allclose(pg.sum(1), fg - f0g, atol=1e-4)
    pg2, _, _ = te_g.explain(rows)
    assert np.array_equal(pg, pg2)
