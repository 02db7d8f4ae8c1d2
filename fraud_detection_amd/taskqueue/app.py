"""Celery-compatible facade over DurableQueue.

Keeps the reference's producer/consumer contract (api/app.py:244-245, xai_tasks.py:59-64):
    celery_app = TaskApp("xai_tasks", broker=os.getenv("CELERY_BROKER_URL"))
    @celery_app.task(bind=True, max_retries=5, acks_late=True)
    def compute_shap(self, transaction_id, input_data, correlation_id=None): ...
    celery_app.send_task("xai_tasks.compute_shap", args=[tx_id, features, corr_id])
    raise self.retry(exc=exc, countdown=5)          # -> MaxRetriesExceededError when exhausted

Redis/Celery are not part of this stack: the broker is the SQL queue named by FDX_QUEUE_URL or,
failing that, DATABASE_URL (a ``redis://`` / ``sentinel://`` broker URL is accepted for
configuration compatibility and mapped to the SQL queue).  If the real ``celery`` package is
installed and FDX_USE_CELERY=1, ``TaskApp`` defers to it instead.

Batch handlers: a task may register ``batch=fn(list[TaskCall]) -> list[result|Exception]``;
the worker then executes all leased calls of that task in ONE device launch (the GPU XAI path).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field

from .queue import DurableQueue


class Retry(Exception):
    def __init__(self, exc=None, countdown: float = 0.0):
        super().__init__(str(exc) if exc else "retry")
        self.exc = exc
        self.countdown = countdown


class MaxRetriesExceededError(Exception):
    pass


@dataclass
class Request:
    id: str
    retries: int = 0
    headers: dict = field(default_factory=dict)
    correlation_id: str | None = None


class BoundTask:
    """The ``self`` handed to bind=True tasks."""

    MaxRetriesExceededError = MaxRetriesExceededError

    def __init__(self, task: "Task", request: Request):
        self.task = task
        self.request = request
        self.name = task.name
        self.max_retries = task.max_retries

    def retry(self, exc=None, countdown: float | None = None, **_):
        if self.request.retries >= self.task.max_retries:
            raise MaxRetriesExceededError(str(exc) if exc else "max retries exceeded")
        return Retry(exc, self.task.default_retry_delay if countdown is None else countdown)


@dataclass
class TaskCall:
    id: str
    args: list
    kwargs: dict
    request: Request


class Task:
    def __init__(self, app: "TaskApp", fn, name: str, bind: bool, max_retries: int, acks_late: bool,
                 default_retry_delay: float):
        self.app, self.fn, self.name = app, fn, name
        self.bind, self.max_retries, self.acks_late = bind, max_retries, acks_late
        self.default_retry_delay = default_retry_delay
        self.batch_fn = None
        self.__doc__ = fn.__doc__

    def __call__(self, *args, **kwargs):  # eager, in-process (like calling a celery task directly)
        if self.bind:
            return self.fn(BoundTask(self, Request(id="eager")), *args, **kwargs)
        return self.fn(*args, **kwargs)

    def run_call(self, call: TaskCall):
        if self.bind:
            return self.fn(BoundTask(self, call.request), *call.args, **call.kwargs)
        return self.fn(*call.args, **call.kwargs)

    def batch(self, fn):
        self.batch_fn = fn
        return fn

    def delay(self, *args, **kwargs):
        return self.app.send_task(self.name, args=list(args), kwargs=kwargs)

    def apply_async(self, args=None, kwargs=None, countdown=0.0, headers=None):
        return self.app.send_task(self.name, args=args, kwargs=kwargs, countdown=countdown, headers=headers)


class AsyncResult:
    def __init__(self, app: "TaskApp", task_id: str):
        self.app, self.id = app, task_id

    @property
    def status(self) -> str:
        s = self.app.queue.status(self.id)
        return {"QUEUED": "PENDING", "LEASED": "STARTED", "DONE": "SUCCESS", "FAILED": "FAILURE"}.get(
            s["status"] if s else "", "PENDING")

    def get(self, timeout: float = 10.0, interval: float = 0.02):
        import time

        t0 = time.time()
        while time.time() - t0 < timeout:
            s = self.app.queue.status(self.id)
            if s and s["status"] in ("DONE", "FAILED"):
                return s["result"]
            time.sleep(interval)
        raise TimeoutError(self.id)


def queue_url_from_env(broker: str | None) -> str | None:
    url = os.getenv("FDX_QUEUE_URL")
    if url:
        return url
    if broker and broker.split(":", 1)[0] in ("sqlite", "postgresql", "postgresql+psycopg2", "mysql"):
        return broker
    return None  # -> DATABASE_URL (store default)


class TaskApp:
    def __init__(self, main: str = "xai_tasks", broker: str | None = None, queue: DurableQueue | None = None):
        self.main = main
        self.broker = broker
        self._queue = queue
        self._lock = threading.Lock()
        self.tasks: dict[str, Task] = {}

    @property
    def queue(self) -> DurableQueue:
        with self._lock:
            if self._queue is None:
                self._queue = DurableQueue(url=queue_url_from_env(self.broker))
            return self._queue

    def use_queue(self, q: DurableQueue):
        self._queue = q

    def task(self, *dargs, bind: bool = False, max_retries: int = 3, acks_late: bool = True,
             default_retry_delay: float = 180.0, name: str | None = None, **_):
        def deco(fn):
            tname = name or f"{self.main}.{fn.__name__}"
            t = Task(self, fn, tname, bind, max_retries, acks_late, default_retry_delay)
            self.tasks[tname] = t
            return t
        if dargs and callable(dargs[0]):
            return deco(dargs[0])
        return deco

    def send_task(self, name: str, args=None, kwargs=None, countdown: float = 0.0, headers=None, task_id=None,
                  conn=None):
        t = self.tasks.get(name)
        max_retries = t.max_retries if t else 5
        tid = self.queue.send(name, args=args, kwargs=kwargs, countdown=countdown, max_retries=max_retries,
                              headers=headers, task_id=task_id, conn=conn)
        return AsyncResult(self, tid)

    def AsyncResult(self, task_id: str) -> AsyncResult:  # noqa: N802 (celery API name)
        return AsyncResult(self, task_id)
