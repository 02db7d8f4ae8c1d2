#!/usr/bin/env python3
"""Newton-fit schedule lab on the bench's own training rows (one MI355X).

    python tools/newton_lab.py [--rows-per-gpu 10000000] [--json out.json]

Runs the bench pipeline once (bench.py's data: separable(), seed 1000, 0.17% fraud, SMOTE to
balance) to get its post-SMOTE bf16 rows and affine map, then times ops.logreg.newton_fit on those
rows under several warm-up schedules / lookaheads (event-timed median of --reps fits, after
warm-up) and reports per case: ms, total and full-phase iterations, converged, max |w - w_ref|
against the default configuration, and the test AUC.  The verdict's constraint for any change to
the fit's tail: same full-phase iterations, AUC within 1e-5.
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, PipelineResult, TrainConfig, evaluate
    from fraud_detection_amd.ops import logreg as L

    dev = torch.device("cuda", 0)
    n_test = a.rows_per_gpu // 5
    X, y = separable(a.rows_per_gpu - n_test, seed=1000, device=dev)
    Xt, yt = separable(n_test, seed=5000, device=dev)
    cfg = TrainConfig(seed=42, smote_scope="global")
    pipe = DevicePipeline(cfg, None)
    res = pipe.fit(X, y)
    torch.cuda.synchronize()
    rows = pipe.training_rows(res)
    aff = res.scaler.aff
    ws = L.LRWorkspace(dev)
    n = rows.shape[0]
    w0 = np.zeros(32)
    if cfg.init_std > 0:
        w0[:30] = np.random.default_rng(cfg.seed).normal(0.0, cfg.init_std, 30)
    warm_iters = lambda sched: sum(it for _, it in sched)  # noqa: E731

    def run(sched, lookahead=None, hess_stride="auto", max_iter=None):
        # max_iter given: an "oracle" fit that enqueues exactly that many full-phase iterations
        # with no host convergence checks (the floor for the host-checked loop)
        f = L.newton_fit(rows, C=cfg.C, tol=cfg.tol, max_iter=max_iter or cfg.max_iter, w0=w0, workspace=ws,
                         progressive=sched, affine=aff, lookahead=lookahead, hess_stride=hess_stride,
                         check_every=cfg.check_every, sync=max_iter is None)
        return f

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f = fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)), float(np.min(ts)), f

    from fraud_detection_amd.ops.native import native, ptr, stream_of

    m = native()
    st = stream_of(rows)

    def burst(fn, k=20):
        """per-launch microseconds of k back-to-back launches (launch gaps included)"""
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            fn()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) * 1000.0 / k, 2)

    ws.reset(w0, (1.0, 1.0), ptr(aff))
    kern = {}
    for sub in (16, 4, 1):
        for h in (0, 1, 2, 8):
            kern[f"pass_sub{sub}_h{h}"] = burst(lambda: m.logreg_pass(ptr(rows), 0, n, ptr(ws.w32), ptr(ws.class_w), 0,
                                                                      h, sub, ptr(ws.partial), ws.nblocks, st))
    kern["reduce_full"] = burst(lambda: m.logreg_reduce(ptr(ws.partial), ws.nblocks, L.PART_STRIDE, ptr(ws.red), 0, st))
    kern["reduce_grad"] = burst(lambda: m.logreg_reduce(ptr(ws.partial), ws.nblocks, L.GRAD_SLOTS, ptr(ws.red), 0, st))
    kern["newton_update"] = burst(lambda: m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), 30,
                                                          1.0, 0.0, 1 << 30, 1, 0, ptr(aff), st))
    kern["init"] = burst(lambda: ws.reset(w0, (1.0, 1.0), ptr(aff)))
    for name, v in kern.items():
        print(f"{name:22s} {v:9.2f} us/launch", flush=True)

    default = L.progressive_schedule(n)
    cases = [("default", default, None, "auto"),
             ("oracle", default, None, "auto"),
             ("lookahead1", default, 1, "auto"),
             ("lookahead3", default, 3, "auto"),
             ("s16x2_4x2", [(16, 2), (4, 2)], None, "auto"),
             ("s16x3_4x1", [(16, 3), (4, 1)], None, "auto"),
             ("s16x3", [(16, 3)], None, "auto"),
             ("s32x3_8x2", [(32, 3), (8, 2)], None, "auto"),
             ("s64x3_16x2_4x1", [(64, 3), (16, 2), (4, 1)], None, "auto"),
             ("s8x3_2x1", [(8, 3), (2, 1)], None, "auto"),
             ("hs4", default, None, 4),
             ("hs16", default, None, 16),
             ("none", [], None, "auto")]
    out = {"rows": n, "default_schedule": default, "kernels_us": kern, "cases": {}}
    w_ref = None
    full_default = None
    for name, sched, la, hs in cases:
        mi = full_default if name == "oracle" else None
        med, mn, f = timed(lambda: run(sched, la, hs, mi))
        fi = f.as_fit_info() if hasattr(f, "as_fit_info") else f
        r2 = PipelineResult(scaler=res.scaler, fit=fi, n_rows=res.n_rows, n_train_rows=res.n_train_rows,
                            n_minority=res.n_minority, n_synthetic=res.n_synthetic, timings={})
        auc = float(evaluate(r2, Xt, yt, None)["auc"])
        w = np.asarray(fi.w, dtype=np.float64)
        if w_ref is None:
            w_ref = w
            full_default = int(fi.n_iter) - warm_iters(sched)
        rec = {"ms_median": round(med, 4), "ms_min": round(mn, 4), "iters": int(fi.n_iter),
               "full_phase_iters": int(fi.n_iter) - warm_iters(sched), "converged": bool(fi.converged),
               "auc": round(auc, 7), "max_abs_dw_vs_default": float(np.max(np.abs(w - w_ref))),
               "schedule": sched, "lookahead": la}
        out["cases"][name] = rec
        print(f"{name:18s} {med:8.4f} ms (min {mn:8.4f})  iters {rec['iters']:2d} (full {rec['full_phase_iters']})"
              f"  auc {auc:.7f}  dw {rec['max_abs_dw_vs_default']:.2e}", flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
