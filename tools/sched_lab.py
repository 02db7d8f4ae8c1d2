#!/usr/bin/env python3
"""Newton warm-up schedules on the bench's own virtual-SMOTE fit (one MI355X).

    python tools/sched_lab.py [--rows-per-gpu 10000000] [--reps 10] [--json out.json]

For each candidate progressive schedule [(tile subsample, iterations), ...] the host-checked
newton_fit runs on the bench pipeline's stored rows + virtual SMOTE samples: device time (event
median), total / full-phase iterations, convergence, test AUC and max |w - w_default|.  A
schedule may replace the default only with the same full-phase iterations, AUC within 1e-5.
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
    ap.add_argument("--rows-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, PipelineResult, TrainConfig, evaluate
    from fraud_detection_amd.ops import logreg as L

    dev = torch.device("cuda", 0)
    n_test = a.rows_per_gpu // 5
    X, y = separable(a.rows_per_gpu - n_test, seed=1000, device=dev)
    Xt, yt = separable(n_test, seed=5000, device=dev)
    cfg = TrainConfig(seed=42, deferred_check=False)
    pipe = DevicePipeline(cfg, None)
    res = pipe.fit(X, y)
    torch.cuda.synchronize()
    v = pipe._virtual
    rows = pipe._buf[: res.n_rows]
    aff = res.scaler.aff
    ws = L.LRWorkspace(dev)
    w0 = np.zeros(32)
    w0[:30] = np.random.default_rng(cfg.seed).normal(0.0, cfg.init_std, 30)
    n = rows.shape[0] + v.n_new

    def run(sched, refresh="auto"):
        return L.newton_fit(rows, C=cfg.C, tol=cfg.tol, max_iter=cfg.max_iter, w0=w0, workspace=ws, affine=aff,
                            progressive=sched, virtual=v, hess_refresh=refresh).as_fit_info()

    def timed(fn):
        for _ in range(2):
            fn()
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f = fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)), f

    default = L.progressive_schedule(n)
    cases = [("default", default), ("16x2_4x2", [(16, 2), (4, 2)]), ("16x3_4x1", [(16, 3), (4, 1)]),
             ("16x2_4x1", [(16, 2), (4, 1)]), ("32x3_4x2", [(32, 3), (4, 2)]), ("32x2_8x2", [(32, 2), (8, 2)]),
             ("16x3_8x1_4x1", [(16, 3), (8, 1), (4, 1)]), ("8x3_2x1", [(8, 3), (2, 1)]), ("none", [])]
    out = {"rows": int(n), "default": default, "cases": {}}
    w_ref = None
    for name, sched in cases:
        ms, f = timed(lambda: run(sched))
        warm = sum(it for _, it in sched)
        r2 = PipelineResult(scaler=res.scaler, fit=f, n_rows=res.n_rows, n_train_rows=res.n_train_rows,
                            n_minority=res.n_minority, n_synthetic=res.n_synthetic, timings={})
        auc = float(evaluate(r2, Xt, yt, None)["auc"])
        w = np.asarray(f.w, dtype=np.float64)
        if w_ref is None:
            w_ref = w
        rec = {"ms": round(ms, 4), "iters": int(f.n_iter), "full_phase_iters": int(f.n_iter) - warm,
               "converged": bool(f.converged), "auc": round(auc, 7), "grad_max": float(f.grad_max),
               "max_abs_dw_vs_default": float(np.max(np.abs(w - w_ref))), "schedule": sched}
        out["cases"][name] = rec
        print(json.dumps({name: rec}), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
