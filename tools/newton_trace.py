#!/usr/bin/env python3
"""Per-iteration Newton trace on the bench's post-SMOTE rows (GPU): objective, max|grad|,
backtracks and time per iteration for several (warm-up schedule, Hessian stride) variants.

Used to pick the default progressive schedule / Hessian sub-sampling (ops/logreg.py): the
winner is the variant that reaches max|grad| <= tol with the fewest full-data passes."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    dev = torch.device("cuda", 0)
    n_train = a.rows - a.rows // 5
    X, y = separable(n_train, seed=1000, device=dev)
    pipe = DevicePipeline(TrainConfig(seed=42))
    res = pipe.fit(X, y)
    rows = pipe.training_rows(res)
    n = rows.shape[0]
    m = native()
    s = stream_of(rows)
    ws = L.LRWorkspace(dev)
    w0 = np.zeros(32)
    w0[:30] = np.random.default_rng(42).normal(0.0, 0.01, 30)
    print(f"rows {n}  auto_hess_stride {L.auto_hess_stride(n)}  auto schedule {L.progressive_schedule(n)}")

    # name: (warm-up schedule, full-data Hessian stride, Hessian refresh period (0 = every iter))
    # name: (warm-up schedule, full-data Hessian stride, Hessian refresh period (0 = every iter),
    #        1 = the full phase starts from the warm-up's last Hessian)
    variants = {
        "auto": (L.progressive_schedule(n), L.auto_hess_stride(n), L.auto_hess_refresh(n), 0),
        "auto_lazy0": (L.progressive_schedule(n), L.auto_hess_stride(n), L.auto_hess_refresh(n), 1),
        "s16x3s4x2_h4_r4": ([(16, 3), (4, 2)], 4, 4, 0),
        "s16x3s4x1_h4_r4": ([(16, 3), (4, 1)], 4, 4, 0),
        "s16x2s4x2_h4_r4": ([(16, 2), (4, 2)], 4, 4, 0),
        "s16x3s4x2_h8_r4": ([(16, 3), (4, 2)], 8, 4, 0),
        "s32x3s8x2_h4_r4": ([(32, 3), (8, 2)], 4, 4, 0),
        "s32x3s8x1s2x1_h4_r4": ([(32, 3), (8, 1), (2, 1)], 4, 4, 0),
        "s16x3s4x2_h4_r0": ([(16, 3), (4, 2)], 4, 0, 0),
    }
    out = {}
    aff = res.scaler.aff  # the pipeline's rows are pivot-shifted (scaler folded into the solver)
    aptr = ptr(aff) if aff is not None else 0
    for name, (sched, hs, refresh, lazy0) in variants.items():
        ws.reset(w0, (1.0, 1.0))
        if aptr:
            m.logreg_fold(ptr(ws.state), aptr, ptr(ws.w32), s)
        trace = []
        j_full = 0
        for phase, (sub, iters) in enumerate(sched + [(1, 25)]):
            full = sub == 1
            hs_w = hs if full else L.auto_hess_stride(n // sub)
            for jj in range(iters):
                if full:
                    fresh = refresh <= 0 or (j_full + lazy0) % refresh == 0
                    j_full += 1
                    hs_w = hs if fresh else 0
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                L._pass(m, rows, ws, hs_w, 0, n, 4.0, s, sub=sub)
                m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), 30, 1.0,
                                a.tol if full else 0.0, 1 << 30, 1, int(jj == 0 and phase > 0), aptr, s)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e6
                st = ws.state.cpu().numpy()
                trace.append(dict(sub=sub, hs=hs_w, obj=float(st[L.S_OBJ]), gmax=float(st[L.S_GMAX]),
                                  bt=int(st[L.S_BACKTRACKS]), us=round(dt, 1)))
                if int(ws.done.item()):
                    break
        full_passes = sum(1 for t in trace if t["sub"] == 1)
        tot = sum(t["us"] for t in trace)
        print(f"== {name:14s} passes {len(trace):2d} (full {full_passes})  sum {tot:8.1f} us  final gmax {trace[-1]['gmax']:.2e} obj {trace[-1]['obj']:.9f}")
        for t in trace:
            print(f"     sub {t['sub']:2d} hs {t['hs']} obj {t['obj']:.9f} gmax {t['gmax']:.3e} bt {t['bt']} {t['us']:7.1f}us")
        out[name] = trace
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
