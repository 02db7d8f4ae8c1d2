"""Async XAI task module (reference path: xai_tasks.py; Celery app ``celery_app``, task
``xai_tasks.compute_shap(transaction_id, input_data, correlation_id)``, bind=True, max_retries=5,
acks_late=True).

Run the worker:  python -m fraud_detection_amd.taskqueue.worker --app xai_tasks:celery_app
(the equivalent of ``celery -A xai_tasks.celery_app worker``).  The broker is the durable SQL
queue (fraud_detection_amd/taskqueue); leased tasks are explained in one batched GPU launch.
"""
import logging
import os

from fraud_detection_amd.obs.metrics import worker_metrics
from fraud_detection_amd.serve.xai import XaiService
from fraud_detection_amd.taskqueue.app import TaskApp

logger = logging.getLogger(__name__)

CELERY_BROKER_URL = os.getenv("CELERY_BROKER_URL", "redis://redis:6379/0")
celery_app = TaskApp("xai_tasks", broker=CELERY_BROKER_URL)

metrics = worker_metrics()
service = XaiService(device=os.getenv("FDX_DEVICE", "auto"), metrics=metrics)


@celery_app.task(bind=True, max_retries=5, acks_late=True)
def compute_shap(self, transaction_id: str, input_data: dict, correlation_id: str | None = None):
    """Prediction + SHAP attributions for one transaction, persisted to the store."""
    from fraud_detection_amd.taskqueue.app import Retry, TaskCall

    call = TaskCall(self.request.id, [transaction_id, input_data, correlation_id], {}, self.request)
    res = service.explain_batch([call], task=self.task)[0]
    if isinstance(res, Retry):
        raise res  # worker re-queues with the countdown
    if isinstance(res, BaseException):  # max retries exhausted / eager call without a task
        return {"transaction_id": transaction_id, "status": "FAILED"}
    return res


@compute_shap.batch
def compute_shap_batch(calls):
    """Worker fast path: all leased compute_shap calls in one device launch."""
    return service.explain_batch(calls, task=compute_shap)
