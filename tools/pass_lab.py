#!/usr/bin/env python3
"""Per-launch timings of the logistic solvers' building blocks at the bench shape (one MI355X):
every pass flavour the Newton and SGD fits launch over the bench's own training rows (8M stored
real rows + ~8M virtual SMOTE samples), the reduce / update kernels, and whole fits.

    python tools/pass_lab.py [--rows-per-gpu 10000000] [--reps 30] [--json out.json]

Event-timed medians of back-to-back launches (each launch is one timed unit).  Used to attribute
the SGD step and the Newton warm-up tails (latency-bound 1/16 passes, pick-tile chains).
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops import reference as ref
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    dev = torch.device("cuda", 0)
    n_test = a.rows_per_gpu // 5
    X, y = separable(a.rows_per_gpu - n_test, seed=1000, device=dev)
    pipe = DevicePipeline(TrainConfig(seed=42, solver="sgd", storage=a.storage), None)
    res = pipe.fit(X, y)
    torch.cuda.synchronize()
    v = pipe._virtual
    rows = pipe._buf[: res.n_rows]
    aff = res.scaler.aff
    m = native()
    ws = L.LRWorkspace(dev)
    ws.reset(np.zeros(32), (1.0, 1.0), ptr(aff))
    s = stream_of(rows)
    n = rows.shape[0] + v.n_new
    fp8 = a.storage != "bf16"
    out = {"stored_rows": int(rows.shape[0]), "virtual_samples": int(v.n_new), "picks": int(v.nbr.numel()),
           "pass_blocks": ws.nblocks_fp8 if fp8 else ws.nblocks}

    def timeit(fn, reps=a.reps):
        for _ in range(3):
            fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record()
        for i in range(reps):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize()
        return float(np.median([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(reps)]))

    def lp(h, sub):
        return lambda: L._pass(m, rows, ws, h, 0, n, 4.0, s, done=False, sub=sub, virtual=v)

    hs_full = L.auto_hess_stride(n)
    hs_warm = L.auto_warm_hess_stride(n // 16)
    passes = {
        "pass+reduce full H": lp(hs_full, 1),
        "pass+reduce full grad": lp(0, 1),
        "pass+reduce 1/16 H": lp(hs_warm, 16),
        "pass+reduce 1/4 H": lp(L.auto_warm_hess_stride(n // 4), 4),
    }
    n_st = rows.shape[0]
    passes.update({  # attribution: the same sub-samples without the virtual samples, and without H
        "pass+reduce 1/16 H stored-only": lambda: L._pass(m, rows, ws, hs_warm, 0, n_st, 4.0, s, done=False, sub=16),
        "pass+reduce 1/16 grad": lp(0, 16),
        "pass+reduce 1/16 grad stored-only": lambda: L._pass(m, rows, ws, 0, 0, n_st, 4.0, s, done=False, sub=16),
        "pass+reduce full grad stored-only": lambda: L._pass(m, rows, ws, 0, 0, n_st, 4.0, s, done=False, sub=1),
    })
    # (r4: the warm-up passes on 512 / 384 / 256-block grids measured equal or slower at every
    # sub-sample, profiles/r4_i/pass_lab.json)
    passes["pass+reduce 1/8 H"] = lp(L.auto_warm_hess_stride(n // 8), 8)
    us = {k: round(timeit(f), 2) for k, f in passes.items()}
    nb = pipe.cfg.sgd_batches
    blocks = ref.sgd_grid_blocks(rows.shape[0], nb, out["pass_blocks"])
    us["sgd pass 1/8"] = round(timeit(lambda: L._sgd_pass(m, rows, ws, n, 4.0, s, 0, nb, blocks, v)), 2)
    us["logreg_reduce 1088"] = round(timeit(lambda: m.logreg_reduce(ptr(ws.partial), ws.nblocks, 1088, ptr(ws.red), 0, s)), 2)
    us["logreg_reduce 34"] = round(timeit(lambda: m.logreg_reduce(ptr(ws.partial), ws.nblocks, 34, ptr(ws.red), 0, s)), 2)
    ws.red.zero_()
    ws.red[33] = float(n)
    ws.red[64::33] = 1.0  # a PD Hessian diagonal for the timing run
    us["newton_update"] = round(timeit(lambda: m.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done),
                                                                30, 1.0, 0.0, 1 << 30, 1, 0, ptr(aff), s)), 2)
    us["sgd_step (reduce+update)"] = round(timeit(lambda: m.sgd_step(ptr(ws.partial), blocks, ptr(ws.state), ptr(ws.w32),
                                                                      ptr(ws.done), ptr(aff), 30, 1.0, 0.0, 0.5, 1,
                                                                      nb, 0, 0, 0.0, s)), 2)
    mq, k = v.nbr.shape
    ws.done.zero_()
    us["sgd fused step (pass+update, 1 launch)"] = round(timeit(lambda: m.sgd_run(
        ptr(rows), int(fp8), 4.0, n, ptr(ws.w32), ptr(ws.class_w), ptr(ws.done), ptr(ws.partial), blocks, s,
        ptr(v.parents), ptr(v.nbr), ptr(v.lam), ptr(v.off), ptr(v.cnt), int(rows.shape[0]), int(v.q_offset), int(mq),
        int(k), 0, 0, ptr(ws.state), ptr(aff), 30, 1.0, 0.5, 1, 0.0, nb, 3, 1, [0.4, 0.6, 0.8], 0, 1,
        ptr(ws.sgd_acc), ptr(ws.sgd_acc[L.SGD_ACC_WORDS:]))), 2)
    out["launch_us"] = us
    w0 = np.zeros(32)
    w0[:30] = np.random.default_rng(42).normal(0.0, 0.01, 30)
    fits = {
        "sgd fit": lambda: L.sgd_fit(rows, w0=w0, affine=aff, virtual=v, workspace=ws),
        "newton fit (host-checked)": lambda: L.newton_fit(rows, tol=1e-4, w0=w0, affine=aff, virtual=v, workspace=ws),
    }
    out["fit_us"] = {k: round(timeit(f, reps=max(5, a.reps // 3)), 1) for k, f in fits.items()}
    # host enqueue time of one fit (no sync): a fit whose host side is slower than its device
    # side starves the GPU
    import time as _t
    host = {}
    for k2, f in fits.items():
        torch.cuda.synchronize()
        t0 = _t.perf_counter()
        r = f()
        host[k2] = round((_t.perf_counter() - t0) * 1e6, 1)
        r.w  # noqa: B018  (settle)
    out["fit_host_enqueue_us"] = host
    print(json.dumps(out), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
