"""Tracing: OpenTelemetry when installed, otherwise a no-op shim; roctx ranges on the device side.

Reference: OTLP/HTTP exporter configured from OTEL_EXPORTER_OTLP_ENDPOINT and
OTEL_SERVICE_NAME in the API lifespan (api/app.py:88-104) and the worker (xai_tasks.py:33-45);
API -> worker propagation was only a correlation-id argument.  Here a W3C ``traceparent`` is
generated per request and carried in the task headers, so worker spans can join the request
trace whenever a real OTel SDK is present.

Device ranges: ``roctx_range("name")`` pushes/pops a ROCTx range (libroctx64) so rocprofv3
--marker-trace shows pipeline phases; it is a no-op when the library is unavailable.
"""
from __future__ import annotations

import contextlib
import ctypes
import logging
import os
import secrets

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


@contextlib.contextmanager
def span(name: str, **attrs):
    if HAVE_OTEL:  # pragma: no cover
        with _ot.get_tracer("fraud_detection_amd").start_as_current_span(name) as s:
            for k, v in attrs.items():
                s.set_attribute(k, v)
            yield s
    else:
        yield None


_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    for name in ("libroctx64.so.4", "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


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
