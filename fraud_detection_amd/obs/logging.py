"""Logging with correlation / trace ids.

The reference formats plain text (api/app.py:24) but its README promises structured JSON logs
(README.md:117).  ``configure()`` installs either the reference text format or JSON lines
(FDX_LOG_FORMAT=json), and every record carries the current correlation id and trace id from
context variables set by the API middleware / worker.
"""
from __future__ import annotations

import contextvars
import json
import logging
import os
import time

correlation_id: contextvars.ContextVar[str | None] = contextvars.ContextVar("correlation_id", default=None)
trace_id: contextvars.ContextVar[str | None] = contextvars.ContextVar("trace_id", default=None)

TEXT_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


class _ContextFilter(logging.Filter):
    def filter(self, record):
        record.correlation_id = correlation_id.get()
        record.trace_id = trace_id.get()
        return True


class JsonFormatter(logging.Formatter):
    def format(self, record):
        d = {"ts": round(time.time(), 6), "level": record.levelname, "logger": record.name, "msg": record.getMessage()}
        for k in ("correlation_id", "trace_id", "transaction_id"):
            v = getattr(record, k, None)
            if v:
                d[k] = v
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


_configured = False


def configure(level: int = logging.INFO, fmt: str | None = None):
    global _configured
    if _configured:
        return
    fmt = fmt or os.getenv("FDX_LOG_FORMAT", "text")
    env_level = os.getenv("FDX_LOG_LEVEL")
    if env_level:  # e.g. WARNING in a latency benchmark (per-request INFO lines cost ~50 us each)
        level = getattr(logging, env_level.upper(), level)
    h = logging.StreamHandler()
    h.addFilter(_ContextFilter())
    h.setFormatter(JsonFormatter() if fmt == "json" else logging.Formatter(TEXT_FORMAT))
    root = logging.getLogger()
    root.addHandler(h)
    root.setLevel(level)
    _configured = True
