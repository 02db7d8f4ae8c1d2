"""Durable task queue on the SQL store (replaces the Redis broker).

Semantics kept from the reference's Celery configuration (xai_tasks.py:63; docs/WorkerRecoveryTestPlan.md):
  * acks_late: a task is LEASED to a worker for ``visibility_timeout`` seconds and only removed
    (DONE) after the handler returns; a worker that dies mid-task lets the lease expire and the
    task is redelivered to another worker;
  * retry with countdown: ``retry(countdown=s)`` re-queues with eta = now + s, attempts += 1;
  * max_retries: once attempts exceed it the task is FAILED (terminal).  A lease that expires
    (the worker died or hung mid-task) counts as an attempt too, so a task that kills its worker
    every time is not redelivered forever;
  * ownership: ack / retry / fail / extend only act on a row that is still LEASED by the calling
    worker, so a slow worker whose lease expired cannot settle the task a second worker now owns
    (or overwrite a DONE row).
  * queue depth is observable (the KEDA trigger of k8s/keda-scaledobject.yaml used the Redis list
    length; here ``depth()`` / the ``fdx_queue_depth`` gauge).
Claiming is a conditional UPDATE per row (status/lease predicate in the WHERE clause), which is
atomic on SQLite and PostgreSQL without table locks, so any number of workers can poll.
"""
from __future__ import annotations

import time
import uuid
from dataclasses import dataclass

from sqlalchemy import and_, case, func, or_, select, update
from sqlalchemy.engine import Engine

from ..store.db import make_engine
from ..store.migrations import upgrade
from ..store.models import TaskRecord

QUEUED, LEASED, DONE, FAILED = "QUEUED", "LEASED", "DONE", "FAILED"


@dataclass
class LeasedTask:
    id: str
    name: str
    args: list
    kwargs: dict
    headers: dict
    attempts: int
    max_retries: int


class DurableQueue:
    def __init__(self, engine: Engine | None = None, url: str | None = None, auto_migrate: bool = True):
        self.engine = engine or make_engine(url)
        if auto_migrate:
            upgrade(self.engine)

    # ---- producer ------------------------------------------------------------------------
    def send(self, name: str, args=None, kwargs=None, countdown: float = 0.0, max_retries: int = 5,
             headers: dict | None = None, task_id: str | None = None, conn=None) -> str:
        """Insert one QUEUED task.  ``conn``: an open transaction on this queue's engine to insert
        in (the API's /predict commits its pending row and the task together: one commit)."""
        now = time.time()
        tid = task_id or str(uuid.uuid4())
        ins = TaskRecord.__table__.insert().values(
            id=tid, name=name, args=list(args or []), kwargs=dict(kwargs or {}), headers=dict(headers or {}),
            status=QUEUED, attempts=0, max_retries=max_retries, eta=now + float(countdown), lease_until=0.0,
            worker=None, result=None, error=None, created_at=now, updated_at=now)
        if conn is not None:
            conn.execute(ins)
            return tid
        with self.engine.begin() as c:
            c.execute(ins)
        return tid

    # ---- consumer ------------------------------------------------------------------------
    def lease(self, worker: str, batch: int = 64, visibility_timeout: float = 60.0,
              names: list[str] | None = None) -> list[LeasedTask]:
        now = time.time()
        t = TaskRecord.__table__
        ready = or_(and_(t.c.status == QUEUED, t.c.eta <= now), and_(t.c.status == LEASED, t.c.lease_until < now))
        q = select(t.c.id).where(ready)
        if names:
            q = q.where(t.c.name.in_(names))
        q = q.order_by(t.c.eta).limit(batch * 2)
        out = []
        expired = and_(t.c.status == LEASED, t.c.lease_until < now)
        with self.engine.begin() as c:
            cand = [r[0] for r in c.execute(q)]
            for tid in cand:
                if len(out) >= batch:
                    break
                res = c.execute(update(t).where(and_(t.c.id == tid, ready)).values(
                    status=LEASED, worker=worker, lease_until=now + visibility_timeout, updated_at=now,
                    attempts=case((expired, t.c.attempts + 1), else_=t.c.attempts)))
                if res.rowcount != 1:
                    continue
                row = c.execute(select(t).where(t.c.id == tid)).mappings().one()
                if row["attempts"] > row["max_retries"]:
                    c.execute(update(t).where(t.c.id == tid).values(
                        status=FAILED, worker=None, lease_until=0.0, updated_at=now,
                        error=f"lease expired after {row['attempts']} attempts (max_retries={row['max_retries']})"))
                    continue
                out.append(LeasedTask(row["id"], row["name"], list(row["args"]), dict(row["kwargs"]),
                                      dict(row["headers"]), row["attempts"], row["max_retries"]))
        return out

    @staticmethod
    def _owned(t, task_id: str, worker: str | None):
        cond = [t.c.id == task_id, t.c.status == LEASED]
        if worker is not None:
            cond.append(t.c.worker == worker)
        return and_(*cond)

    def ack(self, task_id: str, result=None, worker: str | None = None) -> bool:
        t = TaskRecord.__table__
        with self.engine.begin() as c:
            r = c.execute(update(t).where(self._owned(t, task_id, worker)).values(
                status=DONE, result=result, updated_at=time.time()))
        return r.rowcount == 1

    def retry(self, task_id: str, countdown: float, error: str = "", worker: str | None = None) -> str | None:
        """Re-queue after a failure; returns the new status (QUEUED or FAILED), or None when the
        task is no longer leased by ``worker`` (nothing changed)."""
        t = TaskRecord.__table__
        now = time.time()
        with self.engine.begin() as c:
            row = c.execute(select(t.c.attempts, t.c.max_retries).where(self._owned(t, task_id, worker))).first()
            if row is None:
                return None
            attempts = row[0] + 1
            status = FAILED if attempts > row[1] else QUEUED
            r = c.execute(update(t).where(self._owned(t, task_id, worker)).values(
                status=status, attempts=attempts, eta=now + float(countdown), lease_until=0.0, error=error[:4000],
                worker=None, updated_at=now))
        return status if r.rowcount == 1 else None

    def fail(self, task_id: str, error: str = "", result=None, worker: str | None = None) -> bool:
        """Terminal failure of a task still leased by ``worker``; returns whether a row changed."""
        t = TaskRecord.__table__
        with self.engine.begin() as c:
            r = c.execute(update(t).where(self._owned(t, task_id, worker)).values(
                status=FAILED, error=error[:4000], result=result, updated_at=time.time()))
        return r.rowcount == 1

    def extend(self, task_ids: list[str], visibility_timeout: float, worker: str) -> int:
        """Heartbeat: push the lease of every task still held by ``worker``; returns rows extended."""
        if not task_ids:
            return 0
        t = TaskRecord.__table__
        with self.engine.begin() as c:
            r = c.execute(update(t).where(and_(t.c.id.in_(task_ids), t.c.worker == worker, t.c.status == LEASED)).values(
                lease_until=time.time() + visibility_timeout))
        return r.rowcount

    # ---- introspection -------------------------------------------------------------------
    def status(self, task_id: str) -> dict | None:
        t = TaskRecord.__table__
        with self.engine.connect() as c:
            r = c.execute(select(t).where(t.c.id == task_id)).mappings().first()
        return dict(r) if r else None

    def depth(self) -> int:
        """Tasks waiting or in flight (the analogue of LLEN celery)."""
        t = TaskRecord.__table__
        with self.engine.connect() as c:
            return int(c.execute(select(func.count()).select_from(t).where(t.c.status.in_([QUEUED, LEASED]))).scalar())

    def counts(self) -> dict:
        t = TaskRecord.__table__
        with self.engine.connect() as c:
            return {s: int(n) for s, n in c.execute(select(t.c.status, func.count()).group_by(t.c.status))}

    def purge(self):
        with self.engine.begin() as c:
            c.execute(TaskRecord.__table__.delete())

    def ping(self) -> bool:
        try:
            self.depth()
            return True
        except Exception:
            return False
