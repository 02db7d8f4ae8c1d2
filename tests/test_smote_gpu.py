"""SMOTE generation from bf16 parents in the training rows' space (ops/knn.smote_parents): the
device parents equal the CPU ones bit for bit, and the generated rows match the numpy oracle
(ops/reference.py smote_generate on the same parents) up to the oracle's two-rounding
interpolation (one fma on the device)."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.ops import knn as K
from fraud_detection_amd.ops import reference as ref
from fraud_detection_amd.ops import scaler as S


def _minority(n=60_000, seed=8):
    X, y = separable(n, fraud_rate=0.05, seed=seed)
    rows = torch.empty((X.shape[0], 32), dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, rows)
    idx = torch.nonzero(y == 1).reshape(-1)
    xmin = S.scale_cast(X[idx].contiguous(), st, labels=y[idx].contiguous(), out_dtype="f32")
    return st, xmin


def test_smote_draws_pack_and_decode():
    nbr = np.random.default_rng(0).integers(0, 1000, size=(700, 5)).astype(np.int32)
    plan = ref.smote_plan(nbr, 50_000, 42, 3)
    i, j, lam = ref.smote_draws_decode(plan)
    assert i.min() >= 0 and i.max() < 700
    assert np.all(np.isin(j, nbr[i]))   # every neighbour index comes from its parent's k-NN row
    assert lam.min() >= 0.0 and lam.max() < 1.0
    assert abs(float(lam.mean()) - 0.5) < 0.01
    # a 2^-16 grid
    assert np.all((lam * 65536.0) == np.round(lam * 65536.0))


@pytest.mark.gpu
def test_smote_parents_match_cpu(dev):
    st, xmin = _minority()
    for aff in (None, st.aff):
        cpu = K.smote_parents(xmin, aff)
        gpu = K.smote_parents(xmin.to(dev), aff.to(dev) if aff is not None else None).cpu()
        assert torch.equal(cpu, gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("self_search", [True, False])
def test_knn_prep_writes_parents(dev, self_search):
    """knn_topk(parents=...) fills the parents from the operand-prep launch (role 2 when queries
    are the candidates, role 0 otherwise): == smote_parents bit for bit, same neighbour lists."""
    st, xmin = _minority(n=80_000, seed=12)
    C = xmin.to(dev)
    Q = C if self_search else C[: C.shape[0] // 2].clone()
    aff = st.aff.to(dev)
    base = K.knn_topk(Q, C, k=5, self_offset=0)
    for a in (None, aff):
        P = torch.empty((C.shape[0], 32), dtype=torch.bfloat16, device=dev)
        nbr = K.knn_topk(Q, C, k=5, self_offset=0, parents=P, parents_affine=a)
        assert torch.equal(nbr, base)
        assert torch.equal(P, K.smote_parents(C, a))
    with pytest.raises(ValueError):
        K.knn_topk(Q, C, k=5, self_offset=0, parents=torch.empty((3, 32), dtype=torch.bfloat16, device=dev))


def test_knn_topk_parents_cpu():
    st, xmin = _minority(n=20_000, seed=13)
    P = torch.empty((xmin.shape[0], 32), dtype=torch.bfloat16)
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0, parents=P, parents_affine=st.aff)
    assert torch.equal(nbr, K.knn_topk(xmin, xmin, k=5, self_offset=0))
    assert torch.equal(P, K.smote_parents(xmin, st.aff))
    with pytest.raises(ValueError):
        K.knn_topk(xmin, xmin, k=5, self_offset=0, parents_affine=st.aff)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bf16", "fp8", "f32"])
def test_smote_generate_bf16_parents(dev, kind):
    st, xmin = _minority(seed=9)
    P = K.smote_parents(xmin, st.aff if kind == "bf16" else None)
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0)
    n_new = 40_000
    dt = {"bf16": torch.bfloat16, "fp8": torch.uint8, "f32": torch.float32}[kind]
    out_gpu = torch.empty((n_new, 32), dtype=dt, device=dev)
    K.smote_generate(P.to(dev), nbr.to(dev), 0, n_new, out_gpu, seed=5, counter_base=1)
    exp = ref.smote_generate(P.float().numpy(), nbr.numpy(), 0, n_new, 5, 1)
    got = ref.rows_to_f32(out_gpu.cpu()).numpy() if kind == "fp8" else out_gpu.float().cpu().numpy()
    if kind == "fp8":
        e = exp.copy()
        e[:, :30] *= 4.0
        exp = ref.rows_to_f32(torch.from_numpy(ref.fp8_encode(e))).numpy()
        assert np.mean(got != exp) < 2e-3
    elif kind == "bf16":
        e = ref.bf16_round(exp)
        assert np.all(np.abs(got - e) <= 2.0 ** -7 * np.abs(e) + 1e-6)
        assert np.mean(got != e) < 1e-3
    else:
        np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-6)
    assert np.all(got[:, 31] == 1.0) and np.all(got[:, 30] == 1.0)


def test_smote_bf16_parents_need_no_affine():
    st, xmin = _minority(n=20_000)
    P = K.smote_parents(xmin, st.aff)
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0)
    out = torch.empty((10, 32), dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        K.smote_generate(P, nbr, 0, 10, out, affine=st.aff)
    K.smote_generate(P, nbr, 0, 10, out)
    assert torch.all(out[:, 31] == 1)


def test_fp32_reciprocal_pick_division_is_exact():
    """common.h smote_pack_draw: for pick < 2^22, floor((pick + 0.5f) * RN(1/k)) == pick / k for
    every k the kernel accepts (1..8) and beyond (to 64) -- exhaustive over the pick range."""
    p = np.arange(1 << 22, dtype=np.uint32)
    pf = p.astype(np.float32) + np.float32(0.5)
    for k in range(1, 65):
        inv = np.float32(1.0) / np.float32(k)
        got = np.floor(pf * inv).astype(np.uint32)   # fp32 multiply, round-to-nearest
        assert np.array_equal(got, p // np.uint32(k)), k


def test_smote_range_guard():
    """i/j are packed in 24 bits -- parent sets of 2^24 rows or more must be refused,
    never silently wrapped."""
    with pytest.raises(ValueError, match="2\\^24"):
        ref.smote_check_ranges(1 << 24, 1000, 5)
    with pytest.raises(ValueError, match="32 bits"):
        ref.smote_check_ranges(1000, 1 << 30, 5)
    ref.smote_check_ranges((1 << 24) - 1, (1 << 24) - 1, 5)
    # the op checks before touching data: a huge virtual parent set via an expanded view
    C = torch.zeros((1, 32), dtype=torch.float32).expand(1 << 24, 32)
    nbr = torch.zeros((4, 5), dtype=torch.int32)
    with pytest.raises(ValueError, match="2\\^24"):
        K.smote_generate(C, nbr, 0, 4, torch.empty((4, 32), dtype=torch.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("mq", [100_000, 1_000_000])   # mq*k below / above 2^22 (fp32-reciprocal vs div path)
def test_smote_device_draws_exact(dev, mq):
    """Device (i, j, lambda) == smote_plan bit for bit: integer-valued fp32 parents make the fused
    interpolation exact, so any wrong draw shows up as a differing output value."""
    k, n_new, M = 5, 300_000, mq + 4096
    rng = np.random.default_rng(mq)
    C = np.zeros((M, 32), np.float32)
    r = np.arange(M, dtype=np.float32)
    C[:, 0] = r                                # row id (exact in fp32 below 2^24)
    C[:, 1] = (r * 7) % 1021
    C[:, 2] = M - r
    nbr = rng.integers(0, M, size=(mq, k)).astype(np.int32)
    q_off = M - mq
    out = torch.empty((n_new, 32), dtype=torch.float32, device=dev)
    K.smote_generate(torch.from_numpy(C).to(dev), torch.from_numpy(nbr).to(dev), q_off, n_new, out,
                     seed=11, counter_base=7)
    i, j, lam = ref.smote_draws_decode(ref.smote_plan(nbr, n_new, 11, 7))
    assert (mq * k < (1 << 22)) == (mq == 100_000)
    xi, xj = C[q_off + i, :3].astype(np.float64), C[j, :3].astype(np.float64)
    exp = (xi + lam.astype(np.float64)[:, None] * (xj - xi)).astype(np.float32)  # exact, then one rounding
    got = out[:, :3].cpu().numpy()
    assert np.array_equal(got, exp)


@pytest.mark.gpu
def test_smote_sample_offset_slices_equal_one_launch(dev):
    """DP global scope: 128-aligned slices of one draw sequence == one launch (device and oracle)."""
    st, xmin = _minority(seed=10)
    P = K.smote_parents(xmin, st.aff).to(dev)
    nbr = K.knn_topk(xmin, xmin, k=5, self_offset=0).to(dev)
    n = 10_000
    whole = torch.empty((n, 32), dtype=torch.bfloat16, device=dev)
    K.smote_generate(P, nbr, 0, n, whole, seed=3)
    parts = torch.empty_like(whole)
    for a, b in ((0, 1280), (1280, 1280), (1280, 7296), (7296, n)):
        K.smote_generate(P, nbr, 0, b - a, parts[a:b], seed=3, sample_offset=a)
    assert torch.equal(whole, parts)
    cpu = torch.empty((n - 1280, 32), dtype=torch.bfloat16)
    K.smote_generate(P.cpu(), nbr.cpu(), 0, n - 1280, cpu, seed=3, sample_offset=1280)
    e = cpu.float()
    g = whole[1280:].float().cpu()
    assert torch.mean((g != e).float()) < 1e-3 and torch.allclose(g, e, rtol=2 ** -7, atol=1e-6)
