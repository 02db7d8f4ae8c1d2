"""The serving process model: ONE process owns the GPU, every front-end forwards to it.

The reference serves with ``gunicorn -k uvicorn.workers.UvicornWorker --workers 2``
(/root/reference/Dockerfile:21, docker-compose.yml:74): each worker process holds its own model
copy.  On MI355X a model copy per worker means a HIP context and a set of pinned buffers per
worker, and every single-row request a launch of its own.  Here:

* ``GpuOwner`` -- the only code that launches kernels.  A collector thread drains the
  shared-memory request ring (csrc/serve/shm_ring.cpp: lock-free slots, futex wake-ups, no
  pickling) straight into the engine's pinned input buffer and runs ONE fused launch per batch
  (continuous batching: whatever is queued when the previous launch returns forms the next
  batch; an optional window waits for more).  It runs inside a front-end (single-worker
  deployment: anonymous ring) or as its own process (``python -m
  fraud_detection_amd.serve.gpu_owner --ring /dev/shm/...``; serve/launch.py starts it first).
* ``RingClient`` -- a front-end's view: ``predict_proba`` / ``predict_explain`` of [n, d] rows
  through the ring (blocking, GIL released while waiting).
* ``Dispatcher`` -- what /predict calls: batches at or below the owner's calibrated
  ``host_max_rows`` run on the front-end's own exact fp64 host path (a GPU round trip costs more
  than scoring a few rows on the CPU), larger ones go through the ring to the GPU.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
import time

import numpy as np

logger = logging.getLogger("fdx.gpu_owner")

OP_PREDICT, OP_EXPLAIN = 0, 1
DEFAULT_SLOTS, DEFAULT_SLOT_ROWS = 1024, 64


def _ring_mod():
    from .. import _fdx_ring  # host-only C++ (no HIP): front-ends import it without a GPU context

    return _fdx_ring


class GpuOwner:
    """Collector thread: ring -> pinned batch -> one launch -> results back to the slots."""

    def __init__(self, engine, ring_path: str = "", max_batch: int = 8192, window_us: float = 0.0,
                 nslots: int = DEFAULT_SLOTS, slot_rows: int = DEFAULT_SLOT_ROWS, metrics=None,
                 persist_rows: int | None = None, persist_idle_ms: float | None = None):
        R = _ring_mod()
        self.engine = engine
        self.max_batch = int(max_batch)
        self.window_us = float(window_us)
        self.metrics = metrics
        self.ring = R.Ring(ring_path, nslots, engine.d, slot_rows, engine.d + 2)
        self.ring_path = ring_path
        env = os.environ.get("FDX_HOST_MAX_ROWS", "").strip()
        self.ring.host_max_rows = int(env) if env and int(env) >= 0 else int(min(engine.host_max_rows, 1 << 30))
        self._bufs = [engine.owner_input(self.max_batch, 0), engine.owner_input(self.max_batch, 1)]
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._loop, name="fdx-gpu-owner", daemon=True)
        self._native = None
        self.native = _native_capable(engine) and os.environ.get("FDX_OWNER_LOOP", "native") == "native"
        # native loop: small predict batches through the persistent mailbox kernel (None: engine default)
        self.persist_rows = persist_rows
        self.persist_idle_ms = persist_idle_ms

    def native_stats(self) -> dict:
        """Persistent-kernel counters of the native loop ({} for the Python loop)."""
        return self.engine.native_owner_stats(self._native) if self._native is not None else {}

    @property
    def batches(self) -> int:
        return int(self.ring.stats()["batches"])

    @property
    def rows(self) -> int:
        return int(self.ring.stats()["rows"])

    def start(self) -> "GpuOwner":
        if self.native:
            # the whole serving loop in C++ (csrc/bindings.cpp NativeOwner): ring -> mapped pinned
            # batch -> fused kernel -> mapped pinned results -> ring, no Python and no GIL per batch
            kw = {} if self.persist_rows is None else {"persist_rows": int(self.persist_rows)}
            if self.persist_idle_ms is not None:
                kw["idle_ms"] = float(self.persist_idle_ms)
            self._native = self.engine.start_native_owner(self.ring, self.max_batch, self.window_us, **kw)
        else:
            self._th.start()
        self.ring.owner_state = _ring_mod().OWNER_READY
        return self

    def stop(self):
        self._stop.set()
        if self._native is not None:
            errors = self.engine.stop_native_owner(self._native)
            self._native = None
            if errors:
                logger.error("native GPU owner loop failed %d batch(es)", errors)
        elif self._th.is_alive():
            self._th.join(timeout=5)
        self.ring.owner_state = _ring_mod().OWNER_STOPPED

    def _loop(self):
        """Pipelined: while batch i runs on the device from buffer set i % 2, whatever requests are
        queued are gathered into the other set and launched behind it; then batch i is waited for
        and its slots completed (one futex wake for all its producers)."""
        ring, eng = self.ring, self.engine
        try:
            from ..obs.metrics import gpu_kernel_histogram

            hist = gpu_kernel_histogram().labels("owner_batch")
        except Exception:  # noqa: BLE001 - metrics are best effort
            hist = None
        inflight = None  # (set, handle, rows, t_start)
        cur = 0
        while not self._stop.is_set() or inflight is not None:
            n = op = 0
            if not self._stop.is_set():
                # with a batch in flight only look (never wait): that batch must be completed promptly
                n, op = ring.collect(self._bufs[cur], self.max_batch, self.window_us,
                                     0.0 if inflight is not None else 50.0, cur)
            started = None
            if n:
                t0 = time.perf_counter()
                try:
                    started = (cur, eng.run_staged_async(n, op == OP_EXPLAIN, cur), n, t0)
                except Exception:  # noqa: BLE001 - fail the batch, keep serving
                    logger.exception("GPU owner batch of %d rows failed to launch", n)
                    ring.complete(0, 0, 0, 0, False, cur)
            if inflight is not None:
                s, h, rows, t0 = inflight
                try:
                    p, z, phi, dphi = eng.wait_staged(h)
                    if hist is not None:  # launch + device time + wait of one batch (host clock)
                        hist.observe(time.perf_counter() - t0)
                    ring.complete(p, z, phi, dphi, True, s)
                    if self.metrics is not None:
                        self.metrics.microbatch_size.observe(rows)
                except Exception:  # noqa: BLE001
                    logger.exception("GPU owner batch of %d rows failed", rows)
                    ring.complete(0, 0, 0, 0, False, s)
                inflight = None
            if started is not None:
                inflight = started
                cur ^= 1


def _native_capable(engine) -> bool:
    """The native loop serves the linear model's fused predict / LinearSHAP kernel on a GPU."""
    return (getattr(engine, "kind", "") == "linear" and engine.device.type == "cuda"
            and os.environ.get("FDX_XAI_METHOD", "auto") in ("auto", "linear")
            and hasattr(engine, "start_native_owner"))


class RingClient:
    """Front-end side of the ring (attach by path, or share an in-process GpuOwner's ring)."""

    def __init__(self, ring_or_path, timeout_ms: float = 10_000.0):
        self.ring = _ring_mod().Ring(ring_or_path) if isinstance(ring_or_path, str) else ring_or_path
        self.d = self.ring.d
        self.timeout_ms = timeout_ms

    @property
    def host_max_rows(self) -> int:
        return int(self.ring.host_max_rows)

    def owner_alive(self) -> bool:
        R = _ring_mod()
        if self.ring.owner_state != R.OWNER_READY:
            return False
        try:
            os.kill(self.ring.owner_pid, 0)
            return True
        except OSError:
            return False

    @property
    def max_request_rows(self) -> int:
        """Rows of one ring request: half the ring, so two such requests can be in flight."""
        return max(self.ring.slot_rows, (self.ring.nslots // 2) * self.ring.slot_rows)

    def _request(self, X: np.ndarray, op: int) -> np.ndarray:
        """One ring request per max_request_rows piece (a batch larger than the ring is split
        instead of refused)."""
        X = np.ascontiguousarray(X, np.float32)
        cap = self.max_request_rows
        if X.shape[0] <= cap:
            return self.ring.request(X, op, self.timeout_ms)
        return np.concatenate([self.ring.request(X[i:i + cap], op, self.timeout_ms)
                               for i in range(0, X.shape[0], cap)])

    def predict_proba(self, X: np.ndarray):
        o = self._request(X, OP_PREDICT)
        return o[:, 0].astype(np.float64), o[:, 1].astype(np.float64)

    def predict_explain(self, X: np.ndarray):
        o = self._request(X, OP_EXPLAIN)
        return o[:, 0].astype(np.float64), o[:, 1].astype(np.float64), o[:, 2:2 + self.d].astype(np.float64)

    def stats(self) -> dict:
        return dict(self.ring.stats())


class Dispatcher:
    """Routes one front-end's scoring: small batches on the host, the rest through the ring.

    ``engine`` is this process's engine (a CPU engine in a multi-worker front-end; the GPU engine
    itself when the owner runs in-process) -- its exact host path serves the small batches.
    ``client`` is None when there is no GPU owner (CPU deployment): everything runs on ``engine``.
    """

    def __init__(self, engine, client: RingClient | None = None, owner: GpuOwner | None = None,
                 host_max_rows: int | None = None, metrics=None):
        self.engine, self.client, self.owner, self.metrics = engine, client, owner, metrics
        self._host_max = host_max_rows

    @property
    def host_max_rows(self) -> int:
        if self._host_max is not None:
            return self._host_max
        if self.client is not None:
            v = self.client.host_max_rows
            return v if v >= 0 else 0
        return 1 << 62

    @property
    def enabled(self) -> bool:  # a GPU owner batches this process's device work
        return self.client is not None

    def _host(self, X):
        p, z = self.engine._predict_host(X)[:2]
        if self.metrics is not None:
            self.metrics.host_rows.inc(X.shape[0])
        return p, z

    def predict_proba(self, X: np.ndarray):
        X = np.ascontiguousarray(X, np.float32)
        if self.client is None:
            return self.engine.predict_proba(X)
        if X.shape[0] <= self.host_max_rows:
            return self._host(X)
        try:
            return self.client.predict_proba(X)
        except RuntimeError as e:  # owner gone or timed out: degrade to the host path, loudly
            logger.error("GPU owner unavailable (%s): scoring %d rows on the host", e, X.shape[0])
            return self._host(X)

    def explain(self, X: np.ndarray, method: str):
        """(prob, phi) of a batch: through the GPU owner when one serves this front-end (any size:
        the client splits it), else -- or when the owner is down or times out -- on this process's
        engine, loudly (this path used to raise HTTP 500 past 65,536 rows)."""
        X = np.ascontiguousarray(X, np.float32)
        if self.client is not None and self.owner is None and X.shape[0]:
            try:
                p, _, phi = self.client.predict_explain(X)
                return p, phi
            except RuntimeError as e:
                logger.error("GPU owner unavailable (%s): explaining %d rows on the host", e, X.shape[0])
        ex = self.engine.explain(X, method)
        return ex.prob, ex.phi

    def predict_one(self, x: np.ndarray):
        p, z = self.predict_proba(x.reshape(1, -1))
        return float(p[0]), float(z[0])

    def close(self):
        if self.owner is not None:
            self.owner.stop()
            self.owner = None


def in_process(engine, window_us: float, max_batch: int, metrics=None) -> Dispatcher:
    """Single-worker deployment: the owner thread lives in this process (anonymous ring)."""
    if engine.device.type != "cuda":
        return Dispatcher(engine, metrics=metrics)
    owner = GpuOwner(engine, "", max_batch=max_batch, window_us=window_us, metrics=metrics).start()
    return Dispatcher(engine, RingClient(owner.ring), owner, metrics=metrics)


def main(argv=None) -> int:
    """The GPU-owner process: load the production engine on the GPU, create the ring, serve."""
    ap = argparse.ArgumentParser(description="GPU-owner process for multi-worker serving")
    ap.add_argument("--ring", required=True, help="ring file (under /dev/shm)")
    ap.add_argument("--window-us", type=float, default=float(os.getenv("FDX_MICROBATCH_US", "0")))
    ap.add_argument("--max-batch", type=int, default=int(os.getenv("FDX_MICROBATCH_MAX", "8192")))
    ap.add_argument("--slots", type=int, default=DEFAULT_SLOTS)
    ap.add_argument("--slot-rows", type=int, default=DEFAULT_SLOT_ROWS)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    from ..config import Settings
    from ..obs.metrics import api_metrics
    from .app import load_production_engine

    s = Settings.load()
    eng, src = load_production_engine(s, s.device)
    tmp = a.ring + ".tmp"
    owner = GpuOwner(eng, tmp, max_batch=a.max_batch, window_us=a.window_us, nslots=a.slots,
                     slot_rows=a.slot_rows, metrics=api_metrics())
    os.replace(tmp, a.ring)  # front-ends never see a half-initialised ring
    owner.start()
    logger.info("GPU owner pid %d serving %s model (%s) on %s via %s; host path <= %d rows", os.getpid(), eng.kind,
                src, eng.device, a.ring, owner.ring.host_max_rows)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    signal.signal(signal.SIGINT, lambda *_: done.set())
    while not done.wait(0.5):
        pass
    owner.stop()
    try:
        os.unlink(a.ring)
    except OSError:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
