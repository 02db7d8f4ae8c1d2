"""Prometheus metrics.  Names of the reference are preserved exactly:

API  (api/app.py:66-68, 281):  predictions_submitted_total, api_inference_duration_seconds,
      api_db_latency_seconds, and the prometheus-fastapi-instrumentator default set
      http_requests_total{method,handler,status}, http_request_duration_seconds{method,handler},
      http_request_size_bytes{handler}, http_response_size_bytes{handler}.
Worker (xai_tasks.py:48-50): xai_task_duration_seconds, xai_task_success_total,
      xai_task_failures_total -- actually observed here (the reference never observed them).
New GPU/queue metrics: fdx_gpu_kernel_seconds{kernel}, fdx_train_rows_per_second,
      fdx_shap_values_per_second, fdx_queue_depth, fdx_allreduce_seconds{op},
      fdx_microbatch_size, fdx_hbm_used_bytes.
Metrics live in a per-process registry object so several apps can coexist in one test process.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest, start_http_server
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401  (re-export)

_LAT_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


@dataclass
class ApiMetrics:
    registry: CollectorRegistry
    predictions_submitted: Counter
    inference_time: Histogram
    db_latency: Histogram
    http_requests: Counter
    http_duration: Histogram
    http_req_size: Histogram
    http_resp_size: Histogram
    microbatch_size: Histogram
    host_rows: Counter          # rows scored on the exact host path (small batches, owner down)
    owner_rows: Gauge           # rows the GPU owner has scored (ring statistics, multi-worker)

    def render(self) -> bytes:
        """This app's metrics plus the process-global ones (worker / training / span / GPU
        metrics observed in the same process, e.g. an in-process worker or a fit)."""
        from prometheus_client import REGISTRY

        out = generate_latest(self.registry)
        return out if self.registry is REGISTRY else out + generate_latest(REGISTRY)


def api_metrics(registry: CollectorRegistry | None = None) -> ApiMetrics:
    gpu_kernel_histogram()  # declared with the app (observed by the device engines)
    span_histogram()
    r = registry or CollectorRegistry()
    size_buckets = (100, 1_000, 10_000, 100_000, 1_000_000)
    return ApiMetrics(
        registry=r,
        predictions_submitted=Counter("predictions_submitted_total", "Total number of prediction requests submitted",
                                      registry=r),
        inference_time=Histogram("api_inference_duration_seconds", "Synchronous model inference time (seconds)",
                                 buckets=_LAT_BUCKETS, registry=r),
        db_latency=Histogram("api_db_latency_seconds", "DB call latency for startup checks (seconds)",
                             buckets=_LAT_BUCKETS, registry=r),
        http_requests=Counter("http_requests_total", "Total number of requests by method, status and handler.",
                              ["method", "status", "handler"], registry=r),
        http_duration=Histogram("http_request_duration_seconds", "Latency with only few buckets by handler.",
                                ["method", "handler"], buckets=_LAT_BUCKETS, registry=r),
        http_req_size=Histogram("http_request_size_bytes", "Content length of incoming requests by handler.",
                                ["handler"], buckets=size_buckets, registry=r),
        http_resp_size=Histogram("http_response_size_bytes", "Content length of outgoing responses by handler.",
                                 ["handler"], buckets=size_buckets, registry=r),
        microbatch_size=Histogram("fdx_microbatch_size", "Rows per fused GPU predict launch",
                                  buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096), registry=r),
        host_rows=Counter("fdx_host_path_rows", "Rows scored on the exact host fp64 path", registry=r),
        owner_rows=Gauge("fdx_gpu_owner_rows", "Rows scored by the GPU-owner process (all front-ends)",
                         registry=r),
    )


@dataclass
class WorkerMetrics:
    registry: CollectorRegistry
    task_duration: Histogram
    task_success: Counter
    task_failure: Counter
    queue_depth: Gauge
    shap_values_per_second: Gauge
    batch_size: Histogram


_worker_lock = threading.Lock()


def worker_metrics(registry: CollectorRegistry | None = None) -> WorkerMetrics:
    from prometheus_client import REGISTRY

    r = registry or REGISTRY
    with _worker_lock:
        existing = getattr(r, "_fdx_worker_metrics", None)
        if existing is not None:
            return existing
        m = WorkerMetrics(
            registry=r,
            task_duration=Histogram("xai_task_duration_seconds", "XAI task duration seconds", buckets=_LAT_BUCKETS,
                                    registry=r),
            task_success=Counter("xai_task_success_total", "Number of successful XAI tasks", registry=r),
            task_failure=Counter("xai_task_failures_total", "Number of failed XAI tasks", registry=r),
            queue_depth=Gauge("fdx_queue_depth", "Tasks queued or leased (KEDA trigger)", registry=r),
            shap_values_per_second=Gauge("fdx_shap_values_per_second", "SHAP values per second of the last batch",
                                         registry=r),
            batch_size=Histogram("fdx_xai_batch_size", "Explanations per fused device launch",
                                 buckets=(1, 4, 16, 64, 256, 1024, 4096), registry=r),
        )
        r._fdx_worker_metrics = m
        return m


@dataclass
class TrainMetrics:
    registry: CollectorRegistry
    rows_per_second: Gauge
    allreduce_seconds: Histogram
    hbm_used_bytes: Gauge


_train_lock = threading.Lock()


def train_metrics(registry: CollectorRegistry | None = None) -> TrainMetrics:
    """Training metrics, one set per registry (default: the process-global one that /metrics and
    the worker's :8001 server expose)."""
    from prometheus_client import REGISTRY

    r = registry or REGISTRY
    with _train_lock:
        existing = getattr(r, "_fdx_train_metrics", None)
        if existing is not None:
            return existing
        m = TrainMetrics(
            registry=r,
            rows_per_second=Gauge("fdx_train_rows_per_second", "Post-SMOTE rows fitted per second", registry=r),
            allreduce_seconds=Histogram("fdx_allreduce_seconds", "Collective latency (host-observed, synchronised)",
                                        ["op"], buckets=_LAT_BUCKETS, registry=r),
            hbm_used_bytes=Gauge("fdx_hbm_used_bytes", "Device memory in use (torch allocator + native)", registry=r),
        )
        r._fdx_train_metrics = m
        return m


_span_lock = threading.Lock()


def span_histogram(registry: CollectorRegistry | None = None) -> Histogram:
    from prometheus_client import REGISTRY

    r = registry or REGISTRY
    with _span_lock:
        h = getattr(r, "_fdx_span_hist", None)
        if h is None:
            h = Histogram("fdx_span_seconds", "Duration of traced spans", ["name"], buckets=_LAT_BUCKETS, registry=r)
            r._fdx_span_hist = h
        return h


_gpu_lock = threading.Lock()


def gpu_kernel_histogram(registry: CollectorRegistry | None = None) -> Histogram:
    """fdx_gpu_kernel_seconds{kernel}: device time of serving / XAI launches (HIP events)."""
    from prometheus_client import REGISTRY

    r = registry or REGISTRY
    with _gpu_lock:
        h = getattr(r, "_fdx_gpu_hist", None)
        if h is None:
            h = Histogram("fdx_gpu_kernel_seconds", "Device time of serving / XAI launches (HIP events)", ["kernel"],
                          buckets=_LAT_BUCKETS, registry=r)
            r._fdx_gpu_hist = h
        return h


_servers: dict[int, object] = {}


def start_metrics_server(port: int, registry: CollectorRegistry | None = None) -> bool:
    """Start a /metrics HTTP server once per port (the reference's :8001 collided when several
    processes imported xai_tasks; here only the worker entry point starts it)."""
    if port in _servers:
        return True
    try:
        kw = {"registry": registry} if registry is not None else {}
        _servers[port] = start_http_server(port, **kw)
        return True
    except OSError:
        return False
