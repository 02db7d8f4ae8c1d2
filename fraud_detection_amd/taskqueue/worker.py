"""Queue worker: leases batches, runs handlers (batched on the GPU when the task has one), acks late.

    python -m fraud_detection_amd.taskqueue.worker --app xai_tasks:celery_app [--batch 256]

Equivalent of ``celery -A xai_tasks.celery_app worker --concurrency=1`` (docker-compose.yml:98).
A crash between compute and ack (e.g. the pod is killed) leaves the lease to expire and the
task is redelivered (acks_late; docs/WorkerRecoveryTestPlan.md:52-56).  Fault injection for
tests: FDX_FAULT=worker_crash_after_compute makes the process exit hard before acking.
"""
from __future__ import annotations

import argparse
import importlib
import logging
import os
import signal
import socket
import threading
import time
import traceback

from .app import MaxRetriesExceededError, Request, Retry, TaskApp, TaskCall
from .queue import DurableQueue

logger = logging.getLogger("fdx.worker")


class _LeaseHeartbeat:
    """Extends the leases of an in-flight batch every visibility_timeout/3 seconds, so a batch
    that runs longer than the visibility timeout is not redelivered while it is still running."""

    def __init__(self, queue: DurableQueue, ids: list[str], visibility_timeout: float, worker: str):
        self.queue, self.ids, self.vt, self.worker = queue, ids, visibility_timeout, worker
        self._done = threading.Event()
        self._th = threading.Thread(target=self._beat, name="fdx-lease-heartbeat", daemon=True)

    def _beat(self):
        while not self._done.wait(max(self.vt / 3.0, 0.01)):
            try:
                self.queue.extend(self.ids, self.vt, self.worker)
            except Exception as e:  # noqa: BLE001 - a missed beat only risks a redelivery
                logger.warning("lease heartbeat failed: %s", e)

    def __enter__(self):
        self._th.start()
        return self

    def __exit__(self, *exc):
        self._done.set()
        self._th.join()
        return False


class Worker:
    def __init__(self, app: TaskApp, batch: int = 256, visibility_timeout: float = 60.0, poll_interval: float = 0.05,
                 name: str | None = None, metrics=None):
        self.app = app
        self.queue: DurableQueue = app.queue
        self.batch = batch
        self.visibility_timeout = visibility_timeout
        self.poll_interval = poll_interval
        self.name = name or f"{socket.gethostname()}:{os.getpid()}:{id(self) & 0xffff:x}"
        if metrics is None:  # the process-global worker metrics (what :8001 and /metrics expose)
            from ..obs.metrics import worker_metrics

            metrics = worker_metrics()
        self.metrics = metrics
        self._stop = threading.Event()

    def stop(self, *_):
        self._stop.set()

    def run_once(self) -> int:
        """Lease and process one batch.  Returns the number of tasks handled."""
        leased = self.queue.lease(self.name, self.batch, self.visibility_timeout, names=list(self.app.tasks) or None)
        if not leased:
            return 0
        with _LeaseHeartbeat(self.queue, [lt.id for lt in leased], self.visibility_timeout, self.name):
            self._process(leased)
        if self.metrics is not None:
            self.metrics.queue_depth.set(self.queue.depth())
        return len(leased)

    def _process(self, leased):
        by_name: dict[str, list] = {}
        for lt in leased:
            by_name.setdefault(lt.name, []).append(lt)
        for name, items in by_name.items():
            task = self.app.tasks.get(name)
            if task is None:
                for lt in items:
                    self.queue.fail(lt.id, f"unregistered task {name}", worker=self.name)
                continue
            calls = [TaskCall(lt.id, lt.args, lt.kwargs,
                              Request(id=lt.id, retries=lt.attempts, headers=lt.headers,
                                      correlation_id=lt.headers.get("correlation_id"))) for lt in items]
            t0 = time.perf_counter()
            if task.batch_fn is not None:
                try:
                    results = task.batch_fn(calls)
                except Exception as e:  # whole-batch failure: fall back to per-call so one bad row can't poison it
                    logger.warning("batch handler for %s failed (%s); retrying calls individually", name, e)
                    results = [self._run_single(task, c) for c in calls]
            else:
                results = [self._run_single(task, c) for c in calls]
            dt = time.perf_counter() - t0
            if os.getenv("FDX_FAULT") == "worker_crash_after_compute":
                os._exit(17)  # simulate SIGKILL between compute and ack
            for call, res in zip(calls, results):
                self._settle(task, call, res, dt / max(len(calls), 1))

    def _run_single(self, task, call):
        try:
            return task.run_call(call)
        except Exception as e:  # noqa: BLE001 - settled below
            return e

    def _settle(self, task, call: TaskCall, res, dt: float):
        m = self.metrics
        if isinstance(res, Retry):
            st = self.queue.retry(call.id, res.countdown, repr(res.exc), worker=self.name)
            if m is not None:
                m.task_failure.inc()
            logger.info("task %s retry in %.1fs -> %s", call.id, res.countdown, st)
        elif isinstance(res, MaxRetriesExceededError):
            self.queue.fail(call.id, str(res), result={"status": "FAILED"}, worker=self.name)
            if m is not None:
                m.task_failure.inc()
        elif isinstance(res, BaseException):
            self.queue.fail(call.id, "".join(traceback.format_exception_only(type(res), res)), worker=self.name)
            if m is not None:
                m.task_failure.inc()
        else:
            failed = isinstance(res, dict) and res.get("status") == "FAILED"
            self.queue.ack(call.id, res, worker=self.name)
            if m is not None:
                (m.task_failure if failed else m.task_success).inc()
                m.task_duration.observe(dt)

    def run(self, max_idle: float | None = None):
        idle_since = time.time()
        while not self._stop.is_set():
            n = self.run_once()
            if n:
                idle_since = time.time()
            else:
                if max_idle is not None and time.time() - idle_since > max_idle:
                    break
                time.sleep(self.poll_interval)


def load_app(spec: str) -> TaskApp:
    """``module:attr`` or ``module.attr`` (celery -A style)."""
    if ":" in spec:
        mod, attr = spec.split(":", 1)
    else:
        mod, _, attr = spec.rpartition(".")
    return getattr(importlib.import_module(mod), attr or "celery_app")


def _spawn_per_gpu(n: int, argv: list[str]) -> int:
    """One worker process per GPU (the service-level data parallelism of the XAI path, BASELINE
    config 4): child i sees only GPU i (HIP_VISIBLE_DEVICES, set before it touches HIP) and leases
    its own disjoint batches from the shared queue.  The parent never initialises the GPU; it
    forwards SIGTERM/SIGINT, and as soon as ANY child exits non-zero it stops the others and exits
    with that status.  Children get ``--gpus 0`` (and FDX_WORKER_GPUS=0) so none of them spawns
    again, and ``--metrics-port base+g`` each (base = the parent's --metrics-port, or
    FDX_WORKER_METRICS_PORT, or 8001) so N workers never contend for one port."""
    import subprocess
    import sys

    rest = []
    skip = False
    base = int(os.environ.get("FDX_WORKER_METRICS_PORT", "8001"))
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a in ("--gpus", "--metrics-port"):
            if a == "--metrics-port" and i + 1 < len(argv):
                base = int(argv[i + 1])
            skip = True
            continue
        if a.startswith("--gpus="):
            continue
        if a.startswith("--metrics-port="):
            base = int(a.split("=", 1)[1])
            continue
        rest.append(a)
    procs = []
    for g in range(n):
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(g), FDX_DEVICE="cuda:0", FDX_WORKER_RANK=str(g),
                   FDX_WORKER_GPUS="0", FDX_WORKER_METRICS_PORT=str(base + g if base else 0))
        port = ["--metrics-port", str(base + g if base else 0)]
        procs.append(subprocess.Popen([sys.executable, "-m", "fraud_detection_amd.taskqueue.worker", *rest,
                                       "--gpus", "0", *port], env=env))

    def _fwd(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    signal.signal(signal.SIGTERM, _fwd)
    signal.signal(signal.SIGINT, _fwd)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                logger.error("worker child pid %d exited with %d: stopping the others", p.pid, r)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.2)
    return rc


def main(argv=None):
    import sys

    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.getenv("FDX_WORKER_GPUS", "0")),
                    help="spawn one worker process per GPU (0 = this process only)")
    ap.add_argument("--app", default="xai_tasks:celery_app")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--visibility-timeout", type=float, default=60.0)
    ap.add_argument("--metrics-port", type=int, default=int(os.getenv("FDX_WORKER_METRICS_PORT", "8001")))
    ap.add_argument("--max-idle", type=float, default=None)
    a = ap.parse_args(argv)
    if a.gpus and a.gpus > 1:
        return _spawn_per_gpu(a.gpus, argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    app = load_app(a.app)
    from ..obs.metrics import worker_metrics, start_metrics_server

    metrics = worker_metrics()
    if a.metrics_port:
        start_metrics_server(a.metrics_port)
    w = Worker(app, a.batch, a.visibility_timeout, metrics=metrics)
    signal.signal(signal.SIGTERM, w.stop)
    signal.signal(signal.SIGINT, w.stop)
    logger.info("worker %s started (tasks: %s)", w.name, ", ".join(app.tasks))
    w.run(max_idle=a.max_idle)


if __name__ == "__main__":
    raise SystemExit(main() or 0)
