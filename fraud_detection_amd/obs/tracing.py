"""Tracing: OpenTelemetry when installed, otherwise a no-op shim; roctx ranges on the device side.

Reference: OTLP/HTTP exporter configured from OTEL_EXPORTER_OTLP_ENDPOINT and
OTEL_SERVICE_NAME in the API lifespan (api/app.py:88-104) and the worker (xai_tasks.py:33-45);
API -> worker propagation was only a correlation-id argument.  Here a W3C ``traceparent`` is
generated per request and carried in the task headers, so worker spans can join the request
trace whenever a real OTel SDK is present.

Without the OTel SDK, ``span`` still records each finished span (trace id, span id, parent span
id, name, duration, attributes) in a bounded in-process ring (``recent_spans``) and the
``fdx_span_seconds`` histogram, so the API -> worker trace continuation is observable and tested
(tests/test_observability.py).

Device ranges: ``roctx_range("name")`` pushes/pops a ROCTx range so rocprofv3 --marker-trace shows
pipeline phases (rocprofiler-sdk's librocprofiler-sdk-roctx first, the legacy libroctx64 after);
it is a no-op when neither library is available.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import logging
import os
import secrets
import threading
import time

logger = logging.getLogger(__name__)

try:  # pragma: no cover - opentelemetry is not installed in this image
    from opentelemetry import trace as _ot  # type: ignore

    HAVE_OTEL = True
except Exception:  # noqa: BLE001
    _ot = None
    HAVE_OTEL = False


def new_traceparent() -> str:
    return f"00-{secrets.token_hex(16)}-{secrets.token_hex(8)}-01"


def trace_id_of(traceparent: str | None) -> str | None:
    if not traceparent:
        return None
    parts = traceparent.split("-")
    return parts[1] if len(parts) == 4 else None


def configure(service_name: str | None = None) -> bool:
    """Configure an OTLP exporter if the SDK exists; returns whether tracing is live."""
    if not HAVE_OTEL:
        return False
    try:  # pragma: no cover
        from opentelemetry.exporter.otlp.proto.http.trace_exporter import OTLPSpanExporter
        from opentelemetry.sdk.resources import SERVICE_NAME, Resource
        from opentelemetry.sdk.trace import TracerProvider
        from opentelemetry.sdk.trace.export import BatchSpanProcessor

        endpoint = os.getenv("OTEL_EXPORTER_OTLP_ENDPOINT", "http://otel-collector:4318/v1/traces")
        name = service_name or os.getenv("OTEL_SERVICE_NAME", "fraud-api")
        provider = TracerProvider(resource=Resource.create({SERVICE_NAME: name}))
        provider.add_span_processor(BatchSpanProcessor(OTLPSpanExporter(endpoint=endpoint)))
        _ot.set_tracer_provider(provider)
        return True
    except Exception:  # noqa: BLE001
        logger.exception("Failed to configure OpenTelemetry")
        return False


_RECENT: collections.deque = collections.deque(maxlen=4096)
_RECENT_LOCK = threading.Lock()
_SPAN_HIST = None


def parse_traceparent(tp: str | None):
    """(trace_id, parent_span_id) of a W3C traceparent, or (None, None)."""
    if not tp:
        return None, None
    parts = tp.split("-")
    if len(parts) != 4 or len(parts[1]) != 32 or len(parts[2]) != 16:
        return None, None
    return parts[1], parts[2]


def traceparent_of(record: dict) -> str:
    return f"00-{record['trace_id']}-{record['span_id']}-01"


def recent_spans(name: str | None = None) -> list[dict]:
    with _RECENT_LOCK:
        return [dict(r) for r in _RECENT if name is None or r["name"] == name]


def _observe(name: str, dt: float):
    global _SPAN_HIST
    try:
        if _SPAN_HIST is None:
            from .metrics import span_histogram

            _SPAN_HIST = span_histogram()
        _SPAN_HIST.labels(name).observe(dt)
    except Exception:  # noqa: BLE001 - metrics are best effort
        pass


@contextlib.contextmanager
def span(name: str, parent: str | None = None, **attrs):
    """A span named ``name``; ``parent`` is a W3C traceparent to continue (e.g. the header the API
    put on a queued task).  Yields a dict record (``traceparent_of(rec)`` propagates it)."""
    trace_id, parent_id = parse_traceparent(parent)
    rec = {"name": name, "trace_id": trace_id or secrets.token_hex(16), "span_id": secrets.token_hex(8),
           "parent_span_id": parent_id, "attrs": dict(attrs), "start": time.time()}
    t0 = time.perf_counter()
    try:
        if HAVE_OTEL:  # pragma: no cover
            ctx = None
            if parent:
                from opentelemetry.propagate import extract

                ctx = extract({"traceparent": parent})
            with _ot.get_tracer("fraud_detection_amd").start_as_current_span(name, context=ctx) as s:
                for k, v in attrs.items():
                    s.set_attribute(k, v)
                yield rec
        else:
            yield rec
    finally:
        rec["seconds"] = time.perf_counter() - t0
        with _RECENT_LOCK:
            _RECENT.append(rec)
        _observe(name, rec["seconds"])


_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                 "librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            logger.debug("roctx ranges via %s", name)
            break
        except (OSError, AttributeError):
            continue
    return _roctx


def roctx_available() -> bool:
    return _load_roctx() is not None


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx() if os.getenv("FDX_ROCTX", "1") == "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def roctx_phases():
    """The roctx library when FDX_ROCTX_PHASES=1 (pipeline phase markers: off by default, the
    ctypes calls are host time on the fit's critical path), else None."""
    if os.getenv("FDX_ROCTX_PHASES", "0") != "1":
        return None
    return _load_roctx()


def roctx_mark(lib, name: str) -> None:
    if lib is not None:
        lib.roctxMarkA(name.encode())
