"""HBM planner and the host-streaming fit (runtime/hbm.py, DevicePipeline.fit_host; VERDICT r1 #2,
SURVEY.md §5.7): a shard whose raw rows exceed the (budgeted) device memory trains by streaming
the raw rows twice through pinned staging, and gives the same model as the resident path."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.data.synthetic import separable
from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate
from fraud_detection_amd.runtime import hbm


def test_plan_regimes():
    p = hbm.plan_fit(10_000_000, 30, "bf16", budget=200 << 30)
    assert p.mode == "resident" and p.device_bytes < 200 << 30
    p = hbm.plan_fit(10_000_000, 30, "bf16", budget=int(2.2 * 2**30))
    assert p.mode == "stream_raw" and p.chunk_rows >= 4096 and p.device_bytes <= int(2.2 * 2**30)
    assert hbm.plan_fit(10_000_000, 30, "fp8", budget=int(1.1 * 2**30)).mode == "stream_raw"
    with pytest.raises(MemoryError, match="fp8 rows would need"):
        hbm.plan_fit(10_000_000, 30, "bf16", budget=1 << 30)
    # 100M rows x fp8 on one 288 GB MI355X: resident
    assert hbm.plan_fit(100_000_000, 30, "fp8", budget=260 << 30).mode == "resident"


def test_streaming_fit_equals_resident_cpu():
    X, y = separable(60_000, fraud_rate=0.03, seed=2)
    Xt, yt = separable(20_000, fraud_rate=0.03, seed=3)
    cfg = TrainConfig(tol=1e-8, init_std=0.0)
    ref = DevicePipeline(cfg).fit(X, y)
    pipe = DevicePipeline(cfg)
    st = pipe.fit_host(X, y, device="cpu", budget=30_000_000)
    assert pipe.last_plan.mode == "stream_raw" and pipe.last_plan.chunk_rows < 60_000
    np.testing.assert_allclose(st.scaler.mean64.numpy(), ref.scaler.mean64.numpy(), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(st.w, ref.w, atol=1e-9)
    assert st.n_train_rows == ref.n_train_rows
    assert evaluate(st, Xt, yt)["auc"] == pytest.approx(evaluate(ref, Xt, yt)["auc"], abs=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("storage", ["bf16", "fp8"])
def test_streaming_fit_larger_than_budget_gpu(dev, storage):
    """4M raw rows (480 MB fp32) against a budget below raw + training rows: the raw shard cannot
    be resident, the streamed fit equals the resident unfused fit (same kernels, chunked sums)."""
    X, y = separable(4_000_000, seed=11)
    Xt, yt = separable(500_000, seed=12, device=dev)
    Xp, yp = X.pin_memory(), y.pin_memory()
    cfg = TrainConfig(storage=storage, fold_scaler=False, seed=42)
    pipe = DevicePipeline(cfg)
    budget = (800 if storage == "bf16" else 600) << 20
    st = pipe.fit_host(Xp, yp, device=dev, budget=budget)
    assert pipe.last_plan.mode == "stream_raw"
    assert pipe.last_plan.raw_bytes + pipe.last_plan.rows_bytes > budget
    ref = DevicePipeline(cfg).fit(X.to(dev), y.to(dev))
    np.testing.assert_allclose(st.scaler.mean64.cpu().numpy(), ref.scaler.mean64.cpu().numpy(), rtol=1e-10)
    np.testing.assert_allclose(st.w[:31], ref.w[:31], atol=1e-5)
    a1, a2 = evaluate(st, Xt, yt)["auc"], evaluate(ref, Xt, yt)["auc"]
    assert a1 > 0.95 and abs(a1 - a2) < 1e-5
    # unpinned host rows go through the staging buffers
    st2 = DevicePipeline(cfg).fit_host(X, y, device=dev, budget=budget)
    np.testing.assert_allclose(st2.w[:31], st.w[:31], atol=1e-7)
