#!/usr/bin/env python3
"""CPU KernelSHAP baseline for BASELINE config 4 (shap is not installed here): the same algorithm
as shap.KernelExplainer (2042-coalition design, 100 background rows, identity link, efficiency-
constrained WLS) as the repo's vectorised fp64 numpy oracle (models/explainers.kernelshap_reference:
one einsum per batch instead of shap's per-explanation Python loop, so this is a FAVOURABLE CPU
number), timed on this host's CPUs for a batch of explanations.

    python tools/cpu_kernelshap_baseline.py [--expl 50] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--expl", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch

    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.explainers import cached_design, kernelshap_reference

    rng = np.random.default_rng(0)
    Xr, _ = separable(20000, seed=90)
    Xr = Xr.numpy().astype(np.float64)
    w = rng.normal(0, 0.4, 30) / Xr.std(0)
    bias = float(-2.0 - w @ Xr.mean(0))
    B = separable(100, seed=91)[0].numpy()
    X = separable(a.expl, seed=92)[0].numpy()
    Z, _, A, zM = cached_design(30, None, 0)
    kernelshap_reference(X[:2], w, bias, B, Z, A, zM)  # warm-up
    t0 = time.perf_counter()
    phi, fx, f0 = kernelshap_reference(X, w, bias, B, Z, A, zM)
    dt = time.perf_counter() - t0
    out = {"what": "CPU KernelSHAP (vectorised numpy fp64, shap.KernelExplainer algorithm)",
           "explanations": a.expl, "coalitions": int(Z.shape[0]), "background": 100, "link": "identity",
           "seconds": round(dt, 3), "values_per_sec": round(a.expl * 30 / dt, 1),
           "cpu_threads": torch.get_num_threads(), "efficiency_max_err": float(np.abs(phi.sum(1) - (fx - f0)).max())}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
