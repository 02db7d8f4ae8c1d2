"""Durable queue semantics (docs/WorkerRecoveryTestPlan.md of the reference):
acks_late redelivery, retry countdown, max_retries -> FAILED, crash recovery by fault injection."""
import os
import subprocess
import sys
import time
import uuid

import pytest

from fraud_detection_amd.taskqueue.app import MaxRetriesExceededError, TaskApp
from fraud_detection_amd.taskqueue.queue import DurableQueue
from fraud_detection_amd.taskqueue.worker import Worker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def q(tmp_path):
    return DurableQueue(url=f"sqlite:///{tmp_path}/q.db")


def test_send_lease_ack(q):
    tid = q.send("t.x", args=[1, 2])
    assert q.depth() == 1
    leased = q.lease("w1", 10, 30)
    assert [t.id for t in leased] == [tid]
    assert q.lease("w2", 10, 30) == []           # leased tasks are invisible to others
    assert q.ack(tid, {"ok": 1}, worker="w1")
    assert q.status(tid)["status"] == "DONE" and q.depth() == 0


def test_lease_expiry_redelivers(q):
    tid = q.send("t.x")
    assert q.lease("w1", 10, visibility_timeout=0.05)
    time.sleep(0.1)
    again = q.lease("w2", 10, 30)
    assert [t.id for t in again] == [tid]         # acks_late: a dead worker's task comes back
    assert not q.ack(tid, worker="w1")            # stale worker cannot ack
    assert q.ack(tid, worker="w2")


def test_stale_worker_cannot_retry_or_fail(q):
    """after A's lease expires and B re-leases, A's retry()/fail() must be no-ops."""
    tid = q.send("t.x")
    assert q.lease("A", 10, visibility_timeout=0.05)
    time.sleep(0.1)
    assert [t.id for t in q.lease("B", 10, 30)] == [tid]
    assert q.retry(tid, 0, "late A", worker="A") is None
    assert not q.fail(tid, "late A", worker="A")
    st = q.status(tid)
    assert st["status"] == "LEASED" and st["worker"] == "B"
    assert q.ack(tid, {"ok": 1}, worker="B")
    assert not q.fail(tid, "after done", worker="B")       # a DONE row is never overwritten
    assert q.retry(tid, 0, worker="B") is None
    assert q.status(tid)["status"] == "DONE"


def test_lease_expiry_counts_as_attempt(q):
    """A task that kills its worker every time ends FAILED after max_retries redeliveries."""
    tid = q.send("t.x", max_retries=2)
    seen = []
    for _ in range(5):
        got = q.lease("w", 10, visibility_timeout=0.02)
        seen.append(len(got))
        time.sleep(0.04)
    assert seen[:3] == [1, 1, 1] and seen[3:] == [0, 0]
    st = q.status(tid)
    assert st["status"] == "FAILED" and "lease expired" in st["error"]


def test_heartbeat_extends_long_batch(tmp_path):
    """A batch running past the visibility timeout keeps its lease (worker heartbeat)."""
    app = TaskApp("t", queue=DurableQueue(url=f"sqlite:///{tmp_path}/hb.db"))
    steals = []

    @app.task()
    def slow(x):
        time.sleep(0.5)
        steals.extend(app.queue.lease("thief", 10, 30))
        return x

    tid = slow.delay(3).id
    w = Worker(app, batch=4, visibility_timeout=0.15, poll_interval=0.01, name="w1")
    assert w.run_once() == 1
    assert steals == []
    assert app.queue.status(tid)["status"] == "DONE"


def test_retry_countdown_and_max_retries(q):
    tid = q.send("t.x", max_retries=2)
    q.lease("w", 1, 30)
    assert q.retry(tid, countdown=1.5) == "QUEUED"
    assert q.lease("w", 1, 30) == []              # not before eta
    time.sleep(1.6)
    assert len(q.lease("w", 1, 30)) == 1
    assert q.retry(tid, 0) == "QUEUED"
    q.lease("w", 1, 30)
    assert q.retry(tid, 0) == "FAILED"            # attempts 3 > max_retries 2
    assert q.status(tid)["status"] == "FAILED"


def test_bound_task_retry_semantics(tmp_path):
    app = TaskApp("t", queue=DurableQueue(url=f"sqlite:///{tmp_path}/b.db"))
    calls = []

    @app.task(bind=True, max_retries=2, acks_late=True)
    def flaky(self, x):
        calls.append(self.request.retries)
        if self.request.retries < 5:
            raise self.retry(exc=RuntimeError("boom"), countdown=0)
        return x

    r = app.send_task("t.flaky", args=[7])
    w = Worker(app, batch=4, visibility_timeout=30, poll_interval=0.0)
    for _ in range(5):
        w.run_once()
    assert calls == [0, 1, 2]
    st = app.queue.status(r.id)
    assert st["status"] == "FAILED" and st["result"] == {"status": "FAILED"}
    with pytest.raises(MaxRetriesExceededError):
        from fraud_detection_amd.taskqueue.app import BoundTask, Request

        BoundTask(app.tasks["t.flaky"], Request(id="x", retries=2)).retry(exc=None)


def test_worker_crash_then_recovery(tmp_path):
    """Kill the worker between compute and ack (FDX_FAULT); the lease expires and a healthy
    worker completes the task exactly once in the store."""
    url = f"sqlite:///{tmp_path}/crash.db"
    env = dict(os.environ, DATABASE_URL=url, FDX_QUEUE_URL=url, FDX_DEVICE="cpu")
    tx = str(uuid.uuid4())
    q = DurableQueue(url=url)
    q.send("xai_tasks.compute_shap", args=[tx, {f"feature_{i}": 0.1 for i in range(30)}, "cid"], max_retries=5)
    code = ("import sys; sys.path.insert(0, %r); from fraud_detection_amd.taskqueue.worker import Worker;"
            "import xai_tasks; Worker(xai_tasks.celery_app, visibility_timeout=0.5).run_once()") % ROOT
    p = subprocess.run([sys.executable, "-c", code], env=dict(env, FDX_FAULT="worker_crash_after_compute"),
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert p.returncode == 17, p.stderr[-2000:]
    st = q.counts()
    assert st.get("LEASED") == 1                   # crashed mid-task: still leased, not acked
    time.sleep(0.6)
    p2 = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                        timeout=120)
    assert p2.returncode == 0, p2.stderr[-2000:]
    assert q.counts().get("DONE") == 1
    from sqlalchemy import text

    from fraud_detection_amd.store.db import make_engine

    with make_engine(url).connect() as c:
        n = c.execute(text("select count(*) from shap_explanations where transaction_id=:t"), {"t": tx}).scalar()
        status = c.execute(text("select status from transaction_results")).scalar()
    assert n == 1 and status == "COMPLETED"


def test_db_fault_injection_retries(tmp_path, monkeypatch):
    import xai_tasks

    url = f"sqlite:///{tmp_path}/f.db"
    q = DurableQueue(url=url)
    xai_tasks.celery_app.use_queue(q)
    xai_tasks.service.db_url = url
    xai_tasks.service._db = None
    monkeypatch.setenv("FDX_FAULT", "db_error_rate=1.0")
    r = xai_tasks.celery_app.send_task("xai_tasks.compute_shap", args=[str(uuid.uuid4()), [0.0] * 30, None])
    Worker(xai_tasks.celery_app).run_once()
    st = q.status(r.id)
    assert st["status"] == "QUEUED" and st["attempts"] == 1 and st["eta"] > time.time() + 3  # DB error: 5 s countdown
    monkeypatch.setenv("FDX_FAULT", "")
