#!/usr/bin/env python3
"""Per-kernel microbenchmarks on one MI355X: event-timed medians, effective HBM bandwidth.

    python tools/ubench.py [--rows 8000000] [--json out.json] [--only name,...]

Each case reports median/min microseconds over ``--reps`` launches (after warmup) and the
effective bandwidth = bytes the kernel must move / median time.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import knn as K
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops import metrics as M
    from fraud_detection_amd.ops import predict as P
    from fraud_detection_amd.ops import scaler as S
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    nat = native()
    dev = torch.device("cuda", 0)
    info = nat.device_info(0)
    n = a.rows
    X, y = separable(n, seed=1, device=dev)
    st = S.scaler_fit(X)
    rows2 = torch.empty((2 * n, 32), device=dev, dtype=torch.bfloat16)
    S.scale_cast(X, st, labels=y, out=rows2[:n])
    S.scale_cast(X, st, labels=y, out=rows2[n:])
    results = {}
    only = set(a.only.split(",")) if a.only else None

    def case(name, fn, nbytes):
        if only and name not in only:
            return
        med, mn = timeit(fn, a.reps)
        results[name] = {"median_us": round(med, 2), "min_us": round(mn, 2), "bytes": int(nbytes),
                         "GBps": round(nbytes / (med * 1e-6) / 1e9, 1)}
        print(f"{name:34s} {med:10.1f} us  (min {mn:9.1f})  {results[name]['GBps']:8.1f} GB/s", flush=True)

    pivot = X[0].clone()
    case("scaler_stats", lambda: S.scaler_partial_sums(X, pivot), n * 120)
    outb = torch.empty((n, 32), device=dev, dtype=torch.bfloat16)
    case("scaler_stats_cast_bf16", lambda: S.scaler_fit_cast(X, y, outb), n * (120 + 1 + 64))
    outf = torch.empty((n, 32), device=dev, dtype=torch.float32)
    out8 = torch.empty((n, 32), device=dev, dtype=torch.uint8)
    case("scale_cast_bf16", lambda: S.scale_cast(X, st, labels=y, out=outb), n * (120 + 1 + 64))
    case("scale_cast_f32", lambda: S.scale_cast(X, st, labels=y, out_dtype="f32", out=outf), n * (120 + 1 + 128))
    case("scale_cast_fp8", lambda: S.scale_cast(X, st, labels=y, out_dtype="fp8", out=out8), n * (120 + 1 + 32))
    w = torch.from_numpy(np.r_[np.random.default_rng(0).normal(0, 0.2, 30), -3.0, 0.0])
    case("predict_bf16_2n", lambda: P.predict_rows(rows2, w), 2 * n * (64 + 4))
    case("predict_fp8", lambda: P.predict_rows(out8, w), n * (32 + 4))
    a_, c_, b_ = P.fold_scaler(w.numpy(), *st.numpy()[::2])
    at, ct = torch.from_numpy(a_).to(dev), torch.from_numpy(c_).to(dev)
    X1 = X[:1_000_000]
    case("predict_shap_raw_1M", lambda: P.predict_shap_raw(X1, at, ct, b_), 1_000_000 * (120 + 4 + 120))
    ws = L.LRWorkspace(dev)
    ws.reset(w.numpy())
    s = stream_of(X)
    N2 = 2 * n

    def lr_pass(h):
        def f():
            nat.logreg_pass(ptr(rows2), 0, N2, ptr(ws.w32), ptr(ws.class_w), 0, h, 1, ptr(ws.partial), ws.nblocks, s)
        return f
    case("logreg_pass_hess_2n", lr_pass(1), N2 * 64)
    case("logreg_pass_hess_s3_2n", lr_pass(3), N2 * 64)
    case("logreg_pass_grad_2n", lr_pass(0), N2 * 64)
    out8_2 = torch.empty((N2, 32), device=dev, dtype=torch.uint8)  # same row count as the bf16 cases
    out8_2[:n].copy_(out8)
    out8_2[n:].copy_(out8)

    def lr_pass8(h):
        def f():
            nat.logreg_pass_fp8(ptr(out8_2), 0, N2, ptr(ws.w32), ptr(ws.class_w), 0, h, 1, 4.0, ptr(ws.partial),
                                ws.nblocks_fp8, s)
        return f
    case("logreg_pass_fp8_hess_2n", lr_pass8(1), N2 * 32)
    case("logreg_pass_fp8_hess_s8_2n", lr_pass8(8), N2 * 32)
    case("logreg_pass_fp8_grad_2n", lr_pass8(0), N2 * 32)
    case("logreg_reduce", lambda: nat.logreg_reduce(ptr(ws.partial), ws.nblocks, 1088, ptr(ws.red), 0, s),
         ws.nblocks * 1088 * 4)
    case("newton_update", lambda: nat.newton_update(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), 30, 1.0,
                                                    0.0, 1 << 30, 1, 0, 0, s), 0)
    case("newton_fit_2n_tol1e-4", lambda: L.newton_fit(rows2, tol=1e-4, workspace=ws), N2 * 64)
    case("newton_fit_2n_noprog", lambda: L.newton_fit(rows2, tol=1e-4, workspace=ws, progressive=[]), N2 * 64)
    from fraud_detection_amd.models.explainers import KernelExplainer
    from fraud_detection_amd.ops.kernelshap import kernelshap

    ke = KernelExplainer(a_, b_, X[:100].cpu().numpy(), device="cuda")
    Xe = X[:1000].contiguous()
    case("kernelshap_1k_expl", lambda: kernelshap(Xe, ke, sync=False), 1000 * 30 * 4)
    idx = S.compact_indices(y, 1)
    case("compact_indices", lambda: S.compact_indices(y, 1), n)
    xmin = S.scale_cast(X, st, labels=y, out_dtype="f32", idx=idx)
    m = xmin.shape[0]
    case(f"knn_topk_{m}", lambda: K.knn_topk(xmin, xmin, 5, 0), m * m * 64)
    nbr = K.knn_topk(xmin, xmin, 5, 0)
    case("smote_generate_n", lambda: K.smote_generate(xmin, nbr, 0, n, outb), n * 64)
    case("write_only_fill_n_rows", lambda: outb.zero_(), n * 64)   # store-bandwidth ceiling for SMOTE
    par = K.smote_parents(xmin)
    case("smote_generate_n_bf16_parents", lambda: K.smote_generate(par, nbr, 0, n, outb), n * 64)
    sc = torch.randn(2_000_000, device=dev)
    yl = (torch.rand(2_000_000, device=dev) < 0.002).to(torch.uint8)
    case("roc_auc_2M", lambda: M.roc_auc(sc, yl), 2_000_000 * 5)
    # exact AUC, large-P path (device radix sort): 20M scores at 50 % positives
    sc20 = torch.randn(20_000_000, device=dev)
    yl20 = (torch.rand(20_000_000, device=dev) < 0.5).to(torch.uint8)
    case("roc_auc_20M_50pct", lambda: M.roc_auc(sc20, yl20), 20_000_000 * 5)
    out = {"device": info, "rows": n, "results": results, "pass_blocks": ws.nblocks, "pass_blocks_fp8": ws.nblocks_fp8}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
