#!/usr/bin/env python3
"""Online serving latency / throughput on MI355X (CPU sklearn
transform + predict_proba p50 52 us / p99 65 us per row; config 2: batch /predict 1M x 30).

Measured (host wall clock, synchronised, after warm-up), each with the shipped model artifacts:
  * engine batch=1: InferenceEngine.predict_proba on one row -- pinned upload, fused scaler+GEMV+
    sigmoid kernel, download -- GPU and the exact fp64 CPU path side by side;
  * micro-batched: N concurrent single-row submissions through serve/batcher.MicroBatcher (what
    /predict uses on a GPU), per-request latency percentiles and rows/s;
  * HTTP: /predict through the FastAPI app in-process (TestClient), p50/p99 per request;
  * config 2: 1M rows in one call (host in, host out) and the device-only kernel rate.

    python tools/serve_latency.py [--json out.json] [--reps 2000]
"""
import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def pct(a):
    a = np.asarray(a) * 1e6
    return {"p50_us": round(float(np.percentile(a, 50)), 1), "p99_us": round(float(np.percentile(a, 99)), 1),
            "mean_us": round(float(a.mean()), 1)}


def engine_batch1(eng, x, reps):
    for _ in range(200):
        eng.predict_proba(x)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.predict_proba(x)
        t.append(time.perf_counter() - t0)
    return pct(t)


async def microbatched(eng, rows, concurrency, window_us):
    from fraud_detection_amd.serve.batcher import MicroBatcher

    b = MicroBatcher(eng, window_us, 4096)
    await b.start()
    lat = []

    async def one(r):
        t0 = time.perf_counter()
        await b.submit(r)
        lat.append(time.perf_counter() - t0)

    for i in range(0, 512, concurrency):  # warm-up
        await asyncio.gather(*[one(r) for r in rows[i:i + concurrency]])
    lat.clear()
    t0 = time.perf_counter()
    for i in range(0, len(rows), concurrency):
        await asyncio.gather(*[one(r) for r in rows[i:i + concurrency]])
    dt = time.perf_counter() - t0
    await b.stop()
    return {"requests": len(rows), "concurrency": concurrency, "window_us": window_us,
            "rows_per_sec": round(len(rows) / dt, 1), **pct(lat)}


def http(eng_device, reps):
    import tempfile

    from fastapi.testclient import TestClient

    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.serve.app import create_app
    from fraud_detection_amd.store.db import make_engine

    tmp = tempfile.mkdtemp()
    url = f"sqlite:///{tmp}/lat.db"

    class _NoQueue:  # measure the request path, not the queue insert
        class queue:  # noqa: N801
            @staticmethod
            def ping():
                return True

        @staticmethod
        def send_task(*a, **k):
            return None

    s = Settings.load(database_url=url, device=eng_device, mlflow_tracking_uri=f"file:{tmp}/none", microbatch_us=0)
    app = create_app(s, task_app=_NoQueue, db_engine=make_engine(url))
    t = []
    with TestClient(app) as c:
        for i in range(reps + 100):
            t0 = time.perf_counter()
            r = c.post("/predict", json={"features": [0.1] * 30, "transaction_id": f"lat-{i}"})
            dt = time.perf_counter() - t0
            assert r.status_code == 200
            if i >= 100:
                t.append(dt)
    return pct(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=2000)
    a = ap.parse_args()
    from fraud_detection_amd.serve.engine import InferenceEngine

    out = {"hardware": "MI355X" if torch.cuda.is_available() else "cpu"}
    rng = np.random.default_rng(0)
    x1 = rng.normal(0, 1, (1, 30)).astype(np.float32)
    x1[0, 0], x1[0, 29] = 50_000.0, 80.0
    cpu = InferenceEngine.from_paths(device="cpu")
    out["cpu_fp64_batch1"] = engine_batch1(cpu, x1, a.reps)
    if torch.cuda.is_available():
        gpu = InferenceEngine.from_paths(device="cuda")
        out["gpu_batch1"] = engine_batch1(gpu, x1, a.reps)
        rows = [r for r in rng.normal(0, 1, (20_000, 30)).astype(np.float32)]
        out["gpu_microbatched"] = [asyncio.run(microbatched(gpu, rows, c, w)) for c, w in ((64, 200), (512, 300))]
        X = rng.normal(0, 1, (1_000_000, 30)).astype(np.float32)
        for _ in range(3):
            gpu.predict_proba(X)
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            gpu.predict_proba(X)
        dt = (time.perf_counter() - t0) / reps
        from fraud_detection_amd.ops import predict as P

        Xd = torch.from_numpy(X).cuda()
        for _ in range(3):
            P.predict_shap_raw(Xd, gpu._a, gpu._c, gpu.bias, dphi=0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            P.predict_shap_raw(Xd, gpu._a, gpu._c, gpu.bias, dphi=0)
        torch.cuda.synchronize()
        dk = (time.perf_counter() - t0) / 20
        out["config2_batch_1M"] = {"host_to_host_ms": round(dt * 1e3, 3), "host_to_host_rows_per_sec": round(1e6 / dt, 1),
                                   "device_kernel_us": round(dk * 1e6, 1), "device_rows_per_sec": round(1e6 / dk, 1),
                                   "vs_cpu_sklearn_25.7M_rows_per_sec": round(1e6 / dt / 25.7e6, 2)}
        out["http_predict_gpu"] = http("cuda", min(a.reps, 1000))
    out["http_predict_cpu"] = http("cpu", min(a.reps, 1000))
    out["baseline_cpu_sklearn_row"] = {"p50_us": 52, "p99_us": 65, "source": "BASELINE.md §2 (transform + predict_proba)"}
    line = json.dumps(out)
    print(line)
    if a.json:
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
