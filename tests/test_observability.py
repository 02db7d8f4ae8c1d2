"""Observability that is declared is also observed (the reference defined worker
metrics it never observed, xai_tasks.py:48-56): after a training run and a worker batch, /metrics
carries samples of the training, collective, HBM and span metrics; the worker span continues the
API request's trace; roctx ranges load from rocprofiler-sdk when present."""
import os
import uuid

from fastapi.testclient import TestClient

from fraud_detection_amd.config import Settings
from fraud_detection_amd.data.synthetic import separable_frame
from fraud_detection_amd.obs import tracing
from fraud_detection_amd.serve.app import create_app
from fraud_detection_amd.store.db import make_engine
from fraud_detection_amd.taskqueue.queue import DurableQueue
from fraud_detection_amd.taskqueue.worker import Worker


def _sample(text: str, name: str) -> float:
    vals = [float(ln.split()[-1]) for ln in text.splitlines() if ln.startswith(name) and not ln.startswith("#")]
    return max(vals) if vals else 0.0


def test_metrics_after_fit_and_worker_batch(tmp_path, monkeypatch):
    from fraud_detection_amd import train

    csv = str(tmp_path / "cc.csv")
    separable_frame(20_000, fraud_rate=0.02, seed=5).to_csv(csv, index=False)
    monkeypatch.setenv("DATA_CSV", csv)
    out = train.run(Settings.load(mlflow_tracking_uri=f"file:{tmp_path}/mlruns", device="cpu"), cv_folds=0,
                    model_dir=str(tmp_path / "models"), verbose=False)
    assert os.path.exists(out["paths"]["background"])
    import xai_tasks

    url = f"sqlite:///{tmp_path}/o.db"
    xai_tasks.celery_app.use_queue(DurableQueue(url=url))
    s = Settings.load(database_url=url, device="cpu", mlflow_tracking_uri=f"file:{tmp_path}/none")
    svc = xai_tasks.service
    svc.db_url, svc._db, svc._engine, svc._injected, svc.settings = url, None, None, False, s
    try:
        app = create_app(s, task_app=xai_tasks.celery_app, db_engine=make_engine(url))
        with TestClient(app) as c:
            tx = str(uuid.uuid4())
            c.post("/predict", json={"features": [0.2] * 30, "transaction_id": tx})
            Worker(xai_tasks.celery_app).run_once()
            m = c.get("/metrics").text
    finally:
        svc.settings, svc._engine = None, None
    assert _sample(m, "fdx_train_rows_per_second") > 0
    assert _sample(m, "fdx_span_seconds_count") > 0
    assert 'fdx_span_seconds_count{name="train.final_fit"}' in m
    assert 'fdx_span_seconds_count{name="xai.compute_shap"}' in m
    assert _sample(m, "xai_task_success_total") > 0
    assert "fdx_hbm_used_bytes" in m and "fdx_allreduce_seconds" in m and "fdx_gpu_kernel_seconds" in m


def test_worker_span_continues_the_request_trace():
    tp = tracing.new_traceparent()
    trace_id, parent = tracing.parse_traceparent(tp)
    with tracing.span("xai.compute_shap", parent=tp, batch=3) as rec:
        pass
    got = tracing.recent_spans("xai.compute_shap")[-1]
    assert got["trace_id"] == trace_id and got["parent_span_id"] == parent
    assert tracing.traceparent_of(rec).split("-")[1] == trace_id
    with tracing.span("root") as r2:
        pass
    assert r2["parent_span_id"] is None and len(r2["trace_id"]) == 32


def test_roctx_prefers_rocprofiler_sdk():
    tracing._roctx_tried = False
    tracing._roctx = None
    lib = tracing._load_roctx()
    if lib is not None and os.path.exists("/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
        assert "rocprofiler-sdk-roctx" in lib._name
    with tracing.roctx_range("test.range"):
        pass
