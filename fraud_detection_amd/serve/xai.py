"""Async explainability service behind task ``xai_tasks.compute_shap`` (reference: xai_tasks.py:63-167,
dead duplicate api/worker.py:65-102).

One worker lease = one batched device explanation: every leased task's features are stacked into
one [B, 30] matrix, scored, and explained -- by default with the model family's explainer
(LinearSHAP for the linear model: log-odds attributions, the reference worker's semantics,
xai_tasks.py:103-115 / api/worker.py:53; KernelSHAP for GBDT), and with KernelSHAP when
``FDX_XAI_METHOD=kernel`` (BASELINE config 4: the MFMA coalition GEMM, probability space,
background = the training rows saved with the model; the stored ``explainer`` field says which)
or interventional TreeSHAP when ``FDX_XAI_METHOD=tree`` -- then all rows are upserted in one DB
transaction into BOTH
``transaction_results`` (status COMPLETED, prediction_score, shap_values) and
``shap_explanations`` (what /explain reads, with the explainer and its base value).  The model is
the one the API serves: the registry alias, else the local artifacts (either family).  Scaling
out: one worker process per GPU (``worker --gpus N``) leasing disjoint batches.

Fixes relative to the reference: the feature keys the API sends
(``feature_i``) are mapped positionally; features are standardized (the scaler is folded into
the kernel weights) instead of feeding raw values to a model trained on scaled ones; the model
is cached (reloaded when the file changes) instead of re-read per task; updates go through the
ORM so they are persisted; worker metrics are observed.
Retry policy kept: DB errors -> retry in 5 s, other errors -> row FAILED + retry in 10 s,
max_retries = 5 -> {"status": "FAILED"}.
Fault injection (tests, chaos drills): FDX_FAULT=db_error_rate=<p> raises a DB error with
probability p per batch.
"""
from __future__ import annotations

import logging
import os
import random
import re
import threading
import time
import uuid

import numpy as np
from sqlalchemy.exc import OperationalError, SQLAlchemyError

from ..store import db as store_db
from ..store.migrations import upgrade
from ..store.models import ShapExplanation, StatusEnum, TransactionResult
from ..taskqueue.app import BoundTask, MaxRetriesExceededError
from ..config import Settings
from ..obs import tracing
from .engine import InferenceEngine

logger = logging.getLogger("xai")

_FEATURE_KEY = re.compile(r"^feature_(\d+)$")


class XaiService:
    def __init__(self, engine: InferenceEngine | None = None, db_url: str | None = None, device: str = "auto",
                 metrics=None, method: str | None = None, settings: Settings | None = None):
        self._engine = engine
        self._engine_mtime = None
        self._injected = engine is not None
        self.device = device
        self.db_url = db_url
        self.metrics = metrics
        self.settings = settings
        self._method = method
        self._lock = threading.Lock()
        self._db = None

    @property
    def method(self) -> str:
        return self._method or os.getenv("FDX_XAI_METHOD", "auto")

    # ---- resources ---------------------------------------------------------------------
    def db(self):
        if self._db is None:
            self._db = store_db.make_engine(self.db_url)
            upgrade(self._db)
        return self._db

    def engine(self) -> InferenceEngine:
        """The API's model (registry alias -> local artifacts), reloaded when a local model file
        changes on disk."""
        with self._lock:
            if self._injected:
                return self._engine
            st = self.settings or Settings.load()
            path = st.model_path
            mtime = os.path.getmtime(path) if os.path.exists(path) else None
            if self._engine is None or (self._engine.source == "local" and mtime != self._engine_mtime):
                from .app import load_production_engine

                self._engine, _ = load_production_engine(st, self.device)
                self._engine_mtime = mtime
            return self._engine

    # ---- feature mapping ---------------------------------------------------------------
    @staticmethod
    def features_to_row(input_data, names: list[str]) -> np.ndarray:
        d = len(names)
        if isinstance(input_data, (list, tuple)):
            if len(input_data) != d:
                raise ValueError(f"expected {d} features, got {len(input_data)}")
            return np.asarray(input_data, dtype=np.float32)
        row = np.zeros(d, dtype=np.float32)
        keys = list(input_data.keys())
        if keys and all(_FEATURE_KEY.match(k) for k in keys):
            for k, v in input_data.items():
                i = int(_FEATURE_KEY.match(k).group(1))
                if i >= d:
                    raise ValueError(f"feature index {i} out of range")
                row[i] = float(v)
            return row
        index = {n: i for i, n in enumerate(names)}
        missing = [n for n in names if n not in input_data]
        if missing:
            raise ValueError(f"missing features: {missing[:5]}")
        for n, i in index.items():
            row[i] = float(input_data[n])
        return row

    # ---- batch -------------------------------------------------------------------------
    def explain_batch(self, calls, task=None) -> list:
        """calls: objects with .args = [transaction_id, input_data, correlation_id?] and .request.
        Returns per call: result dict | Retry | MaxRetriesExceededError."""
        t0 = time.perf_counter()
        eng = self.engine()
        names = eng.feature_names
        results: list = [None] * len(calls)
        rows, good = [], []
        for i, c in enumerate(calls):
            try:
                rows.append(XaiService.features_to_row(c.args[1], names))
                good.append(i)
            except Exception as e:  # noqa: BLE001 - bad payload: this call fails, others proceed
                results[i] = self._fail_or_retry(task, c, e, countdown=10.0, mark_failed=True)
        method = ""
        if good:
            X = np.stack(rows)
            parent = next((calls[i].request.headers.get("traceparent") for i in good
                           if getattr(calls[i], "request", None) is not None and calls[i].request.headers), None)
            with tracing.span("xai.compute_shap", parent=parent, batch=len(good)) as sp, \
                    tracing.roctx_range("xai.explain_batch"):
                ex = eng.explain(X, self.method)
                method = ex.method
                sp["attrs"]["method"] = method
            try:
                self._maybe_inject_db_fault()
                self._store(calls, good, ex, names)
                for j, i in enumerate(good):
                    results[i] = {"transaction_id": str(calls[i].args[0]), "status": "COMPLETED",
                                  "prediction_score": float(ex.prob[j]), "explainer": method}
            except SQLAlchemyError as e:
                logger.error("Database error for %d explanations: %s", len(good), e)
                for i in good:
                    results[i] = self._fail_or_retry(task, calls[i], e, countdown=5.0, mark_failed=False)
        dt = time.perf_counter() - t0
        if self.metrics is not None and good:
            self.metrics.batch_size.observe(len(good))
            self.metrics.shap_values_per_second.set(len(good) * len(names) / max(dt, 1e-9))
        return results

    def _fail_or_retry(self, task, call, exc, countdown: float, mark_failed: bool):
        if mark_failed:
            self._mark_failed(call.args[0])
        if task is None:
            return exc
        try:
            return BoundTask(task, call.request).retry(exc=exc, countdown=countdown)
        except MaxRetriesExceededError as e:
            logger.error("Max retries exceeded for %s. Final status: FAILED.", call.args[0])
            self._mark_failed(call.args[0])
            return e

    def _maybe_inject_db_fault(self):
        f = os.getenv("FDX_FAULT", "")
        if f.startswith("db_error_rate="):
            if random.random() < float(f.split("=", 1)[1]):
                raise OperationalError("injected fault", None, Exception("FDX_FAULT"))

    def _store(self, calls, good, ex, names):
        p, phi = ex.prob, ex.phi
        Session = store_db.session_factory(self.db())
        with Session() as s:
            for j, i in enumerate(good):
                c = calls[i]
                tx = str(c.args[0])
                cid = c.args[2] if len(c.args) > 2 else None
                sv = {n: float(v) for n, v in zip(names, phi[j])}
                try:
                    rid = uuid.UUID(tx)
                except ValueError:
                    rid = None
                if rid is not None:
                    rec = s.get(TransactionResult, rid)
                    if rec is None:
                        rec = TransactionResult(id=rid, input_data=c.args[1], status=StatusEnum.COMPLETED.value)
                        s.add(rec)
                    rec.shap_values = sv
                    rec.prediction_score = float(p[j])
                    rec.status = StatusEnum.COMPLETED.value
                row = s.get(ShapExplanation, tx)
                if row is None:
                    s.add(ShapExplanation(transaction_id=tx, correlation_id=cid, shap_values=sv, feature_names=names,
                                          explainer=ex.method, base_value=float(ex.base_value)))
                else:
                    row.shap_values, row.correlation_id, row.feature_names = sv, cid, names
                    row.explainer, row.base_value = ex.method, float(ex.base_value)
            s.commit()

    def _mark_failed(self, tx):
        try:
            rid = uuid.UUID(str(tx))
        except ValueError:
            return
        try:
            with store_db.session_factory(self.db())() as s:
                rec = s.get(TransactionResult, rid)
                if rec is not None:
                    rec.status = StatusEnum.FAILED.value
                    s.commit()
        except SQLAlchemyError:
            pass
