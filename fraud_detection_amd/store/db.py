"""Engine / session factory (reference: db/db.py:6-20).

``DATABASE_URL`` keeps the reference's meaning; when it is unset the default is a local SQLite
file (the reference's Postgres default needs psycopg2, which this image does not ship).  SQLite
runs in WAL mode with a busy timeout so the API, the worker and the queue can share it.
"""
from __future__ import annotations

import logging
import os
import threading

from sqlalchemy import create_engine, event
from sqlalchemy.engine import Engine
from sqlalchemy.orm import sessionmaker

logger = logging.getLogger(__name__)

DEFAULT_URL = "sqlite:///./fraud.db"
_lock = threading.Lock()
_engines: dict[str, Engine] = {}


def database_url() -> str:
    return os.getenv("DATABASE_URL", DEFAULT_URL)


def make_engine(url: str | None = None) -> Engine:
    url = url or database_url()
    with _lock:
        eng = _engines.get(url)
        if eng is not None:
            return eng
        kw = {"pool_pre_ping": True}
        if url.startswith("sqlite"):
            kw["connect_args"] = {"check_same_thread": False, "timeout": 30}
        eng = create_engine(url, **kw)
        if url.startswith("sqlite"):
            @event.listens_for(eng, "connect")
            def _sqlite_pragmas(dbapi_conn, _rec):  # pragma: no cover - trivial
                cur = dbapi_conn.cursor()
                if ":memory:" not in url:
                    cur.execute("PRAGMA journal_mode=WAL")
                cur.execute("PRAGMA busy_timeout=30000")
                cur.execute("PRAGMA synchronous=NORMAL")
                cur.close()
        _engines[url] = eng
        return eng


def session_factory(engine: Engine | None = None):
    return sessionmaker(bind=engine or make_engine(), autocommit=False, autoflush=False, expire_on_commit=False)


def init_db_tables(Base=None, engine: Engine | None = None):
    """Create tables (reference: db/db.py:18-20).  Prefer store.migrations.upgrade()."""
    from .models import Base as _Base

    logger.info("Creating database tables (if not exist)")
    (Base or _Base).metadata.create_all(bind=engine or make_engine())


def reset_engines():
    with _lock:
        for e in _engines.values():
            e.dispose()
        _engines.clear()
