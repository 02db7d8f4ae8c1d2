#!/usr/bin/env python3
"""A/B of SGD per-epoch minibatch counts in the bench pipeline (one GPU, bench shape): ms per fit
(event median), steps, convergence and AUC for each schedule.

    python tools/sgd_schedule_ab.py [--schedules 4,8,8:4,6,6] [--storage bf16] [--fits 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedules", default="4,8,8:4,6,6")
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--fits", type=int, default=20)
    ap.add_argument("--rows", type=int, default=10_000_000)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate

    dev = torch.device("cuda", 0)
    n_train = a.rows - a.rows // 5
    X, y = separable(n_train, seed=1000, device=dev)
    Xt, yt = separable(a.rows // 5, seed=2000, device=dev)
    for spec in a.schedules.split(":"):
        nbs = tuple(int(v) for v in spec.split(","))
        pipe = DevicePipeline(TrainConfig(seed=42, solver="sgd", storage=a.storage, sgd_epoch_batches=nbs))
        for _ in range(3):
            pipe.fit(X, y)
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.fits + 1)]
        ev[0].record()
        for i in range(a.fits):
            r = pipe.fit(X, y)
            ev[i + 1].record()
        torch.cuda.synchronize(dev)
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.fits)]
        f = r.fit
        print(json.dumps({"epoch_batches": list(nbs), "storage": a.storage, "ms_median": round(float(np.median(ms)), 4),
                          "ms_max": round(float(np.max(ms)), 4), "steps": int(f.n_iter), "converged": bool(f.converged),
                          "epoch_grad_max": float(f.grad_max), "auc": round(evaluate(r, Xt, yt)["auc"], 6)}), flush=True)


if __name__ == "__main__":
    main()
