"""FastAPI application (reference: api/app.py, contract in SURVEY.md App. A).

Endpoints (same paths, bodies, status codes and header as the reference):
  POST /predict            200 PredictionOut{transaction_id, prediction, score, correlation_id,
                           explanation_status}; 422 on wrong feature count; header X-Correlation-ID.
                           Scoring: batches up to the calibrated host threshold run on the exact
                           fp64 host path, larger ones go to the GPU owner (serve/gpu_owner.py:
                           one process owns the GPU and batches every front-end's rows into one
                           fused launch); the SHAP explanation is queued as xai_tasks.compute_shap.
  GET  /explain/{id}       200 {transaction_id, created_at, shap_values, feature_names} | 404
  GET  /health             200 {status: OK, dependencies{postgres, redis_broker, mlflow, model}} | 503
  GET  /status             {"status": "UP"}
  GET  /metrics            Prometheus text (reference metric names, see obs/metrics.py)
Additions:
  POST /predict/async      202 {transaction_id, status: PENDING} (the intended A3 contract of
                           api/schemas.py / newgoal.md); the worker computes score + SHAP.
  GET  /result/{id}        PredictResponse{transaction_id, status, prediction_score, detail}
  POST /predict/batch      many rows in one device launch.
Differences from the reference, all deliberate: the model output is read
numerically (no regex over str(ndarray)), the worker receives the same feature keys it maps,
/explain reads the table the worker writes, the broker health is actually checked.
"""
from __future__ import annotations

import logging
import os
import time
import uuid
from contextlib import asynccontextmanager

import numpy as np
from fastapi import FastAPI, HTTPException, Request, Response, status
from fastapi.responses import HTMLResponse, JSONResponse
from sqlalchemy import select, text
from sqlalchemy.exc import SQLAlchemyError

from ..config import Settings
from ..obs import logging as fdx_logging
from ..obs import tracing
from ..obs.metrics import CONTENT_TYPE_LATEST, api_metrics
from ..store import db as store_db
from ..store.migrations import upgrade
from ..store.models import ShapExplanation, StatusEnum, TransactionResult
from . import gpu_owner
from .engine import InferenceEngine, load_engine_dir
from .schemas import BatchIn, BatchOut, PredictAccepted, PredictionOut, PredictResponse, TransactionIn

logger = logging.getLogger("api.app")

TASK_NAME = "xai_tasks.compute_shap"


def load_production_engine(settings: Settings, device: str) -> tuple[InferenceEngine, str]:
    """models:/<name>@<alias> from the registry (either model family: the sklearn-flavour linear
    model or the fdx-gbdt tree ensemble), falling back to the local artifacts (api/app.py:34-44)."""
    from ..compat import mlflow_compat

    uri = f"models:/{settings.mlflow_model_name}@{settings.mlflow_model_stage}"
    kw = {"kernel_nsamples": settings.kernelshap_nsamples, "kernel_link": settings.kernelshap_link}
    try:
        mdir = mlflow_compat.resolve_model_dir(uri, settings.mlflow_tracking_uri)
        eng = load_engine_dir(mdir, device=device, source="mlflow", **kw)
        logger.info("Loaded %s model %s using alias '%s'", eng.kind, settings.mlflow_model_name,
                    settings.mlflow_model_stage)
        return eng, "mlflow"
    except Exception as e:  # noqa: BLE001
        logger.warning("Failed to load model from registry alias '%s' (%s); falling back to local model file",
                       settings.mlflow_model_stage, e)
    eng = InferenceEngine.from_paths(settings.model_path, settings.scaler_path, settings.feature_names_path,
                                     device=device, **kw)
    return eng, "local"


def create_app(settings: Settings | None = None, engine: InferenceEngine | None = None, task_app=None,
               db_engine=None) -> FastAPI:
    settings = settings or Settings.load()
    fdx_logging.configure()
    metrics = api_metrics()
    state = {"engine": engine, "model_source": "injected" if engine else None, "task_app": task_app,
             "db": db_engine, "batcher": None}

    def _db():
        if state["db"] is None:
            state["db"] = store_db.make_engine(settings.database_url)
        return state["db"]

    def _tasks():
        if state["task_app"] is None:
            import xai_tasks  # the reference's module path for the task app

            state["task_app"] = xai_tasks.celery_app
        return state["task_app"]

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        try:
            with metrics.db_latency.time():
                upgrade(_db())
        except Exception as e:  # noqa: BLE001 - same policy as the reference: log, keep serving
            logger.error("Failed to connect or create tables: %s", e)
        state["batcher"] = _make_dispatcher()
        tracing.configure(settings.otel_service_name)
        yield
        state["batcher"].close()

    app = FastAPI(title="Fraud Detection API", version="1.0.0", lifespan=lifespan)
    app.state.fdx = state
    app.state.metrics = metrics
    app.state.settings = settings

    def engine_() -> InferenceEngine:
        if state["engine"] is None:  # used without lifespan (reference tests build TestClient(app) bare)
            eng, src = load_production_engine(settings, settings.device)
            state["engine"], state["model_source"] = eng, src
        return state["engine"]

    def _make_dispatcher() -> gpu_owner.Dispatcher:
        """Multi-worker front-end (FDX_GPU_OWNER_RING): a CPU copy of the model for the host path
        plus the ring to the GPU-owner process.  Single worker: the owner thread in-process."""
        if settings.gpu_owner_ring:
            if state["engine"] is None:
                eng, src = load_production_engine(settings, "cpu")
                state["engine"], state["model_source"] = eng, src
            deadline = time.time() + 120
            while not os.path.exists(settings.gpu_owner_ring):  # the owner is still loading
                if time.time() > deadline:
                    raise RuntimeError(f"GPU owner ring {settings.gpu_owner_ring} never appeared")
                time.sleep(0.05)
            return gpu_owner.Dispatcher(state["engine"], gpu_owner.RingClient(settings.gpu_owner_ring),
                                        metrics=metrics)
        return gpu_owner.in_process(engine_(), settings.microbatch_us, settings.microbatch_max, metrics)

    def batcher_() -> gpu_owner.Dispatcher:
        if state["batcher"] is None:  # used without lifespan: no owner thread, direct engine calls
            state["batcher"] = gpu_owner.Dispatcher(engine_(), metrics=metrics)
        return state["batcher"]

    @app.middleware("http")
    async def correlation_and_metrics(request: Request, call_next):
        cid = request.headers.get("X-Correlation-ID") or str(uuid.uuid4())
        request.state.correlation_id = cid
        tok = fdx_logging.correlation_id.set(cid)
        t0 = time.perf_counter()
        logger.info("[%s] Request received: %s", cid, request.url)
        try:
            response = await call_next(request)
        finally:
            fdx_logging.correlation_id.reset(tok)
        route = request.scope.get("route")
        handler = getattr(route, "path", None) or "none"
        dt = time.perf_counter() - t0
        metrics.http_requests.labels(request.method, f"{response.status_code // 100}xx", handler).inc()
        metrics.http_duration.labels(request.method, handler).observe(dt)
        metrics.http_req_size.labels(handler).observe(int(request.headers.get("content-length") or 0))
        metrics.http_resp_size.labels(handler).observe(int(response.headers.get("content-length") or 0))
        response.headers["X-Correlation-ID"] = cid
        return response

    @app.get("/status", tags=["Health"])
    def get_status():
        """Liveness check."""
        return {"status": "UP"}

    @app.get("/health", tags=["Health"])
    def get_health():
        """Readiness: database, queue broker, model registry and model."""
        deps, degraded = {}, False
        try:
            with _db().connect() as c:
                c.execute(text("SELECT 1"))
            deps["postgres"] = "UP"
        except Exception as e:  # noqa: BLE001
            deps["postgres"] = f"DOWN ({e})"
            degraded = True
        try:
            deps["redis_broker"] = "UP" if _tasks().queue.ping() else "DOWN"
        except Exception as e:  # noqa: BLE001
            deps["redis_broker"] = f"DOWN ({e})"
        try:
            from ..compat import mlflow_compat

            mlflow_compat.resolve_model_dir(f"models:/{settings.mlflow_model_name}@{settings.mlflow_model_stage}",
                                            settings.mlflow_tracking_uri)
            deps["mlflow"] = "UP"
        except Exception as e:  # noqa: BLE001
            deps["mlflow"] = f"DOWN ({e})"
        try:
            eng = engine_()
            ok = eng.health()
        except Exception:  # noqa: BLE001
            ok = False
        if not ok:
            deps["model"] = "DOWN"
            degraded = True
        else:
            deps["model"] = "UP" if state["model_source"] in ("mlflow", "injected") else "DEGRADED (using fallback)"
        body = {"status": "DEGRADED" if degraded else "OK", "dependencies": deps}
        if degraded:
            raise HTTPException(status_code=status.HTTP_503_SERVICE_UNAVAILABLE, detail=body)
        return body

    def _validate(features) -> np.ndarray:
        eng = engine_()
        if len(features) != eng.d:
            raise HTTPException(status_code=422, detail=(
                f"Input data must have {eng.d} features, but got {len(features)}. "
                "This is the raw input size, *before* encoding/scaling."))
        try:
            x = np.asarray([float(v) for v in features], dtype=np.float32)
        except (TypeError, ValueError):
            raise HTTPException(status_code=422, detail="All features must be numeric.")
        if not np.all(np.isfinite(x)):
            raise HTTPException(status_code=422, detail="Features must be finite numbers.")
        return x

    def _persist_pending(tx_id: str, features_dict: dict, score: float | None):
        try:
            with store_db.session_factory(_db())() as s:
                rid = uuid.UUID(tx_id)
                if s.get(TransactionResult, rid) is None:
                    s.add(TransactionResult(id=rid, input_data=features_dict, prediction_score=score,
                                            status=StatusEnum.PENDING.value))
                    s.commit()
        except (ValueError, SQLAlchemyError) as e:  # non-UUID ids skip the row; DB outage is non-fatal
            logger.warning("could not persist pending row for %s: %s", tx_id, e)

    def _enqueue(tx_id: str, features_dict: dict, cid: str, conn=None) -> str:
        try:
            kw = {"conn": conn} if conn is not None else {}
            _tasks().send_task(TASK_NAME, args=[tx_id, features_dict, cid],
                               headers={"correlation_id": cid, "traceparent": tracing.new_traceparent()}, **kw)
            return "Calculation queued"
        except Exception as e:  # noqa: BLE001
            if conn is not None:
                raise  # the one-transaction path falls back to the two separate writes
            logger.error("[%s] Failed to queue SHAP task: %s", cid, e)
            return "Queue failed"

    def _shared_queue_engine() -> bool:
        """The durable broker lives in the store's database (the default: FDX_QUEUE_URL unset)."""
        try:
            q = _tasks().queue
        except Exception:  # noqa: BLE001
            return False
        return getattr(q, "engine", None) is _db()

    def _persist_and_enqueue(tx_id: str, features_dict: dict, score: float | None, cid: str) -> str:
        """Pending row + SHAP task.  When the broker shares the store's database both inserts go
        in ONE transaction (one commit per request instead of two: the commit, not the model, is
        what a deployed /predict waits on); otherwise, or if that transaction fails, the two
        separate writes with their own failure semantics."""
        if _shared_queue_engine():
            try:
                with _db().begin() as c:
                    try:
                        rid = uuid.UUID(tx_id)
                    except ValueError:
                        rid = None  # non-UUID ids skip the row, as in _persist_pending
                    t = TransactionResult.__table__
                    if rid is not None and c.execute(select(t.c.id).where(t.c.id == rid)).first() is None:
                        c.execute(t.insert().values(id=rid, input_data=features_dict, prediction_score=score,
                                                    status=StatusEnum.PENDING.value))
                    return _enqueue(tx_id, features_dict, cid, conn=c)
            except Exception as e:  # noqa: BLE001
                logger.warning("[%s] single-transaction enqueue failed (%s); separate writes", cid, e)
        _persist_pending(tx_id, features_dict, score)
        return _enqueue(tx_id, features_dict, cid)

    @app.post("/predict", response_model=PredictionOut, tags=["Prediction"])
    def predict(transaction: TransactionIn, request: Request):
        """Synchronous scoring and asynchronous SHAP calculation.  A plain (threadpool) handler:
        the ring wait and the DB insert block this request's thread, never the event loop."""
        cid = request.state.correlation_id
        metrics.predictions_submitted.inc()
        x = _validate(transaction.features)
        with metrics.inference_time.time():
            prob, _ = batcher_().predict_one(x)
        prediction = int(prob > 0.5)
        features_dict = {f"feature_{i}": float(v) for i, v in enumerate(x.tolist())}
        explanation_status = _persist_and_enqueue(transaction.transaction_id, features_dict, prob, cid)
        logger.info("[%s] Prediction done: %s, SHAP status: %s", cid, prediction, explanation_status)
        return PredictionOut(transaction_id=transaction.transaction_id, prediction=prediction, score=prob,
                             correlation_id=cid, explanation_status=explanation_status)

    @app.post("/predict/async", response_model=PredictAccepted, status_code=202, tags=["Prediction"])
    def predict_async(transaction: TransactionIn, request: Request):
        cid = request.state.correlation_id
        metrics.predictions_submitted.inc()
        x = _validate(transaction.features)
        features_dict = {f"feature_{i}": float(v) for i, v in enumerate(x.tolist())}
        if _persist_and_enqueue(transaction.transaction_id, features_dict, None, cid) != "Calculation queued":
            raise HTTPException(status_code=503, detail="Queue unavailable")
        return PredictAccepted(transaction_id=transaction.transaction_id, status="PENDING")

    @app.post("/predict/batch", response_model=BatchOut, tags=["Prediction"])
    def predict_batch(batch: BatchIn):
        eng = engine_()
        X = np.asarray(batch.rows, dtype=np.float32)
        if X.ndim != 2 or X.shape[1] != eng.d:
            raise HTTPException(status_code=422, detail=f"rows must be [n, {eng.d}]")
        metrics.predictions_submitted.inc(X.shape[0])
        disp = batcher_()
        with metrics.inference_time.time():
            if batch.explain:  # the GPU owner explains (split to ring-sized requests), else this engine
                p, phi = disp.explain(X, settings.xai_method)
            else:
                p, _ = disp.predict_proba(X)
                phi = None
        return BatchOut(predictions=(p > 0.5).astype(int).tolist(), scores=p.tolist(),
                        shap_values=phi.tolist() if phi is not None else None)

    @app.get("/result/{transaction_id}", response_model=PredictResponse, tags=["Prediction"])
    def get_result(transaction_id: str):
        try:
            rid = uuid.UUID(transaction_id)
        except ValueError:
            raise HTTPException(status_code=404, detail="Unknown transaction id")
        with store_db.session_factory(_db())() as s:
            r = s.get(TransactionResult, rid)
        if r is None:
            raise HTTPException(status_code=404, detail="Unknown transaction id")
        return PredictResponse(transaction_id=transaction_id, status=r.status, prediction_score=r.prediction_score,
                               detail=None if r.status != StatusEnum.FAILED.value else "explanation failed")

    @app.get("/explain/{transaction_id}", tags=["Explanation"])
    def get_shap_explanation(transaction_id: str):
        """Stored SHAP results for a transaction."""
        with store_db.session_factory(_db())() as s:
            r = s.execute(select(ShapExplanation).where(ShapExplanation.transaction_id == transaction_id)).scalar()
        if r is None:
            raise HTTPException(status_code=404, detail="SHAP explanation not found. Calculation may still be pending.")
        return {"transaction_id": transaction_id, "created_at": r.created_at, "shap_values": r.shap_values,
                "feature_names": r.feature_names, "explainer": r.explainer, "base_value": r.base_value}

    @app.get("/ui", include_in_schema=False)
    def console():
        """Minimal browser console (fraud-frontend/index.html): /predict then /explain polling."""
        path = os.environ.get("FDX_UI_HTML") or os.path.join(os.path.dirname(__file__), "..", "..", "fraud-frontend",
                                                             "index.html")
        if not os.path.exists(path):
            raise HTTPException(status_code=404, detail="console not installed")
        with open(path, encoding="utf-8") as f:
            return HTMLResponse(f.read())

    @app.get("/metrics", include_in_schema=False)
    def prometheus_metrics():
        disp = state["batcher"]
        if disp is not None and disp.client is not None:
            metrics.owner_rows.set(disp.client.stats()["rows"])
        return Response(metrics.render(), media_type=CONTENT_TYPE_LATEST)

    @app.exception_handler(SQLAlchemyError)
    async def db_error(_request: Request, exc: SQLAlchemyError):
        logger.error("database error: %s", exc)
        return JSONResponse(status_code=503, content={"detail": "database unavailable"})

    return app
