#!/usr/bin/env python3
"""KernelSHAP device throughput (BASELINE config 4 shape: 2042 coalitions x 100 background rows,
30 features) for the linear MFMA kernel and the tree-ensemble kernel, across batch sizes and
coalition-part counts.  Prints one JSON line per case.

    python tools/kernelshap_bench.py [--reps 10] [--trees 100] [--depth 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(max(3, reps // 2)):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--skip-tree", action="store_true")
    ap.add_argument("--quick", action="store_true", help="1000-explanation cases only")
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models import explainers as EX
    from fraud_detection_amd.ops import gbdt as gb
    from fraud_detection_amd.ops.kernelshap import kernelshap, kernelshap_tree

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    # a served model: standardized-space weights folded onto raw features (ops/predict.fold_scaler)
    Xr, _ = separable(20000, seed=90)
    Xr = Xr.numpy().astype(np.float64)
    w = np.zeros(32)
    w[:30] = rng.normal(0, 0.4, 30) / Xr.std(0)
    bias = float(-2.0 - w[:30] @ Xr.mean(0))
    B, _ = separable(100, seed=91)
    # clock / cache warm-up before the first timed case
    ke0 = EX.KernelExplainer(w, bias, B.numpy(), device="cuda")
    Xw, _ = separable(4096, seed=1)
    timeit(lambda: kernelshap(Xw.to(dev), ke0, sync=False), 50)
    for link in ("identity", "logit_model"):
        ke = EX.KernelExplainer(w, bias, B.numpy(), link=link, device="cuda")
        for E in ((1000,) if a.quick else (1000, 512, 4096, 64)):
            X, _ = separable(E, seed=92)
            Xd = X.to(dev)
            for P in ((None,) if a.quick else (None, 1, 2, 4)):
                dt = timeit(lambda: kernelshap(Xd, ke, sync=False, parts=P), a.reps)
                print(json.dumps({"kernel": "linear", "link": link, "explanations": E, "parts": P or "auto",
                                  "coalitions": ke.nsamples, "background": 100, "us_per_batch": round(dt * 1e6, 1),
                                  "values_per_sec": round(E * 30 / dt, 1)}), flush=True)
    if a.skip_tree:
        return
    Xtr, ytr = separable(200_000, fraud_rate=0.05, seed=3)
    mean, scale = Xtr.numpy().mean(0), Xtr.numpy().std(0)
    Xs = torch.from_numpy(EX._standardize(Xtr.numpy(), mean, scale)).to(dev)
    ens = gb.fit(Xs, ytr.to(dev), gb.GBDTParams(n_estimators=a.trees, max_depth=a.depth))
    te = EX.TreeKernelExplainer(ens, mean, scale, B.numpy(), device="cuda")
    for E in (1000, 128):
        X, _ = separable(E, seed=93)
        Xd = X.to(dev)
        for P in (None, 1):
            dt = timeit(lambda: kernelshap_tree(Xd, te, sync=False, parts=P), max(2, a.reps // 3))
            print(json.dumps({"kernel": "tree", "trees": a.trees, "depth": a.depth, "explanations": E,
                              "parts": P or "auto", "coalitions": te.nsamples, "background": 100,
                              "ms_per_batch": round(dt * 1e3, 3), "values_per_sec": round(E * 30 / dt, 1)}), flush=True)
    # interventional TreeSHAP of the same ensemble (exact, margin space): treeshap.hip
    from fraud_detection_amd.ops.treeshap import treeshap

    ts = EX.TreeExplainer(ens, mean, scale, B.numpy(), device="cuda")
    for E in (1000, 128):
        X, _ = separable(E, seed=93)
        Xd = X.to(dev)
        dt = timeit(lambda: treeshap(Xd, ts, sync=False), a.reps)
        print(json.dumps({"kernel": "treeshap", "trees": a.trees, "depth": a.depth, "explanations": E,
                          "background": 100, "us_per_batch": round(dt * 1e6, 1),
                          "values_per_sec": round(E * 30 / dt, 1),
                          "speedup_vs_tree_kernelshap_note": "exact Shapley (no coalition sampling)"}), flush=True)


if __name__ == "__main__":
    main()
