"""The GPU serving path under test: the FastAPI app on device="cuda" with the
micro-batcher live, the XAI worker's batched KernelSHAP on the device, and a registered GBDT
served and explained on the GPU.  Goldens of the shipped model: 0.000544 / 0.011905
(SURVEY.md App. C); phi against the fp64 oracles (2e-5) and efficiency."""
import concurrent.futures as cf
import os
import uuid

import numpy as np
import pytest
from fastapi.testclient import TestClient

from _models import gbdt_registered, kaggle_like_rows, linear_dir_with_background
from fraud_detection_amd.config import Settings
from fraud_detection_amd.serve.app import create_app
from fraud_detection_amd.store.db import make_engine
from fraud_detection_amd.taskqueue.queue import DurableQueue
from fraud_detection_amd.taskqueue.worker import Worker
from test_api_contract import GOLDEN_SAMPLE

pytestmark = pytest.mark.gpu


def _cuda_service(tmp_path, **kw):
    import xai_tasks

    url = f"sqlite:///{tmp_path}/g.db"
    q = DurableQueue(url=url)
    xai_tasks.celery_app.use_queue(q)
    s = Settings.load(database_url=url, device="cuda", microbatch_us=3000, **kw)
    svc = xai_tasks.service
    svc.db_url, svc._db, svc._engine, svc._injected, svc.settings, svc.device = url, None, None, False, s, "cuda"
    return create_app(s, task_app=xai_tasks.celery_app, db_engine=make_engine(url)), xai_tasks


@pytest.fixture()
def restore_service():
    import xai_tasks

    yield
    svc = xai_tasks.service
    svc.settings, svc._engine, svc._injected, svc.device = None, None, False, os.getenv("FDX_DEVICE", "auto")


def test_gpu_predict_goldens_through_microbatcher(dev, tmp_path, restore_service):
    app, _ = _cuda_service(tmp_path, mlflow_tracking_uri=f"file:{tmp_path}/none")
    with TestClient(app) as c:
        eng = app.state.fdx["engine"]
        assert eng.device.type == "cuda" and app.state.fdx["batcher"].enabled

        def one(i):
            x = GOLDEN_SAMPLE if i % 2 else [0.1] * 30
            return i, c.post("/predict", json={"features": x}).json()["score"]

        with cf.ThreadPoolExecutor(16) as ex:
            res = list(ex.map(one, range(64)))
        for i, s in res:
            assert s == pytest.approx(0.011905 if i % 2 else 0.000544, abs=5e-7)
        m = c.get("/metrics").text
        n_req = [ln for ln in m.splitlines() if ln.startswith("fdx_microbatch_size_count")]
        n_rows = [ln for ln in m.splitlines() if ln.startswith("fdx_microbatch_size_sum")]
        assert float(n_rows[0].split()[-1]) == 64.0 and float(n_req[0].split()[-1]) <= 64.0
        assert 'fdx_gpu_kernel_seconds_count{kernel="predict"}' in m


def test_gpu_worker_kernelshap_roundtrip(dev, tmp_path, restore_service):
    """POST /predict -> queue -> worker (CUDA, one batched KernelSHAP launch) -> GET /explain."""
    from fraud_detection_amd.models.explainers import kernelshap_reference

    mdir = linear_dir_with_background(tmp_path)
    app, xt = _cuda_service(tmp_path, model_path=os.path.join(mdir, "logistic_model.joblib"),
                            mlflow_tracking_uri=f"file:{tmp_path}/none")
    rows = kaggle_like_rows(48, seed=5)
    with TestClient(app) as c:
        txs = []
        for r in rows:
            tx = str(uuid.uuid4())
            assert c.post("/predict", json={"features": r.tolist(), "transaction_id": tx}).status_code == 200
            txs.append(tx)
        assert Worker(xt.celery_app, batch=256).run_once() == len(rows)
        ke = xt.service.engine().kernel_explainer()
        assert xt.service.engine().device.type == "cuda"
        phi_ref, fx_ref, f0_ref = kernelshap_reference(rows, ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, "identity")
        for j, tx in enumerate(txs):
            e = c.get(f"/explain/{tx}").json()
            assert e["explainer"] == "kernel"
            phi = np.array([e["shap_values"][n] for n in e["feature_names"]])
            np.testing.assert_allclose(phi, phi_ref[j], atol=2e-5)
            assert phi.sum() == pytest.approx(fx_ref[j] - f0_ref, abs=2e-5)
            assert e["base_value"] == pytest.approx(f0_ref, abs=1e-6)


def test_gpu_gbdt_alias_served_and_explained(dev, tmp_path, restore_service):
    from fraud_detection_amd.models.explainers import TreeKernelExplainer

    kw, res, X = gbdt_registered(tmp_path)
    app, xt = _cuda_service(tmp_path, **kw)
    rows = X[:32].numpy()
    with TestClient(app) as c:
        eng = app.state.fdx["engine"]
        assert eng.kind == "gbdt" and eng.device.type == "cuda"
        txs = []
        for r in rows:
            tx = str(uuid.uuid4())
            txs.append((tx, c.post("/predict", json={"features": r.tolist(), "transaction_id": tx}).json()["score"]))
        margin = res.predict_margin(X[:32]).numpy().astype(np.float64)
        np.testing.assert_allclose([s for _, s in txs], 1 / (1 + np.exp(-margin)), atol=1e-6)
        assert Worker(xt.celery_app, batch=64).run_once() == 32
        te = TreeKernelExplainer(res.ensemble, *res.scaler.numpy()[::2], eng.background, device="cpu")
        phi_ref, fx_ref, f0_ref = te.explain(rows)
        for j, (tx, score) in enumerate(txs):
            e = c.get(f"/explain/{tx}").json()
            phi = np.array([e["shap_values"][n] for n in e["feature_names"]])
            np.testing.assert_allclose(phi, phi_ref[j], atol=2e-5)
            assert phi.sum() == pytest.approx(score - e["base_value"], abs=1e-4)


def test_engine_staging_reuses_pinned_buffers(dev):
    """Pinned staging is allocated once; small batches run zero-copy (kernel on the pinned
    buffers' device mapping), large ones through the memcpy path -- same results."""
    from fraud_detection_amd.serve import engine as E
    from fraud_detection_amd.serve.engine import InferenceEngine

    eng = InferenceEngine.from_paths(device="cuda")
    p1, _ = eng.predict_proba(np.asarray([GOLDEN_SAMPLE], np.float32))
    assert eng._stage.zero_copy(1), "pinned host buffers must be device-mapped on MI355X"
    buf = eng._stage.hin.data_ptr()
    for n in (1, 7, 200, E.ZERO_COPY_ROWS + 1):
        p, z, phi = eng.predict_explain(np.asarray([GOLDEN_SAMPLE] * n, np.float32))
        assert p.shape == (n,) and phi.shape == (n, 30)
        assert p[0] == pytest.approx(0.011905, abs=5e-7)
    assert eng._stage.hin.data_ptr() != 0
    X2 = kaggle_like_rows(E.ZERO_COPY_ROWS + 40, seed=3)
    a = eng.predict_explain(X2[:E.ZERO_COPY_ROWS])          # zero-copy
    b = eng.predict_explain(X2)                              # memcpy path (grows the buffers once)
    np.testing.assert_allclose(a[0], b[0][:E.ZERO_COPY_ROWS], rtol=0, atol=0)
    np.testing.assert_allclose(a[2], b[2][:E.ZERO_COPY_ROWS], rtol=0, atol=0)
    buf = eng._stage.hin.data_ptr()
    eng.predict_proba(X2[:5])
    assert eng._stage.hin.data_ptr() == buf            # no per-request pinned allocation
    assert p1[0] == pytest.approx(0.011905, abs=5e-7)
    cpu = InferenceEngine.from_paths(device="cpu")
    X = kaggle_like_rows(300, seed=2)
    pg, zg, phig = eng.predict_explain(X)
    pc, zc, phic = cpu.predict_explain(X)
    np.testing.assert_allclose(pg, pc, atol=2e-6)
    np.testing.assert_allclose(phig, phic, rtol=1e-4, atol=1e-4)
