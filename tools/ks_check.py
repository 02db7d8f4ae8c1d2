#!/usr/bin/env python3
"""KernelSHAP accuracy + throughput check on the served-model setups (GPU): the reference's
shipped LR on Kaggle-like raw rows (the worker test) and a trained model on synthetic rows (the
bench), paired vs unpaired kernel, max |phi - fp64 oracle| and us per 1k batch.

    python tools/ks_check.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from _models import kaggle_like_rows
    from fraud_detection_amd.compat.safe_joblib import decode_logistic, decode_scaler
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.explainers import KernelExplainer, kernelshap_reference
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.ops import predict as P
    from fraud_detection_amd.ops.kernelshap import kernelshap

    dev = torch.device("cuda", 0)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    model = decode_logistic(os.path.join(root, "models", "logistic_model.joblib"))
    scaler = decode_scaler(os.path.join(root, "models", "scaler.joblib"))
    w = np.zeros(32)
    w[:30] = model["coef"].ravel()
    w[30] = float(model["intercept"].ravel()[0])
    a, _, bias = P.fold_scaler(w, scaler["mean_"], scaler["scale_"], None)
    setups = {"shipped_lr_kaggle_rows": (a, bias, kaggle_like_rows(100, seed=1), kaggle_like_rows(1000, seed=5))}
    # tools/kernelshap_bench.py's model: random standardized-space weights on raw features
    rng = np.random.default_rng(0)
    Xr = separable(20000, seed=90)[0].numpy().astype(np.float64)
    wb = np.zeros(32)
    wb[:30] = rng.normal(0, 0.4, 30) / Xr.std(0)
    setups["bench_tool_model"] = (wb, float(-2.0 - wb[:30] @ Xr.mean(0)), separable(100, seed=91)[0].numpy(),
                                  separable(1000, seed=92)[0].numpy())
    run(setups)
    setups = {"bench_tool_model_after_training": setups["bench_tool_model"]}
    X, y = separable(2_000_000, seed=1000, device=dev)
    res = DevicePipeline(TrainConfig(seed=42)).fit(X, y)
    a2, _, b2 = res.folded()
    setups["trained_lr_synthetic"] = (a2, b2, separable(100, seed=91)[0].numpy(), separable(1000, seed=92)[0].numpy())
    run(setups)


def run(setups):
    from fraud_detection_amd.models.explainers import KernelExplainer, kernelshap_reference
    from fraud_detection_amd.ops.kernelshap import kernelshap

    dev = torch.device("cuda", 0)
    for name, (aa, bb, B, Xe) in setups.items():
        for paired in (True, False):
            ke = KernelExplainer(aa, bb, B, device="cuda")
            Xd = torch.from_numpy(np.ascontiguousarray(Xe, np.float32)).to(dev)
            phi, fx, f0 = kernelshap(Xd, ke, paired=paired)
            ref = kernelshap_reference(Xe[:200], ke.a, ke.bias, ke.B, ke.Z, ke.A, ke.zM, "identity")
            err = np.abs(phi[:200] - ref[0])
            for _ in range(10):
                kernelshap(Xd, ke, sync=False, paired=paired)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                kernelshap(Xd, ke, sync=False, paired=paired)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 50
            zx = Xe.astype(np.float64) @ ke.a[:30] + ke.bias
            # coalition logits L_b(z) for 50 explanations (fp64 on the device)
            Zt = torch.from_numpy(ke.Z.astype(np.float64)).to(dev)
            Bt = torch.from_numpy(ke.B.astype(np.float64)).to(dev)
            at = torch.from_numpy(ke.a[:30].astype(np.float64)).to(dev)
            xt = torch.from_numpy(Xe[:50].astype(np.float64)).to(dev)
            U = at * (xt[:, None, :] - Bt[None])                         # [50, nb, d]
            Lz = torch.einsum("ebd,sd->ebs", U, Zt) + (Bt @ at + ke.bias)[None, :, None]
            frac = {f"lt{-t}": float((Lz < t).double().mean()) for t in (-44.0, -88.0, -116.0)}
            print(json.dumps({"setup": name, "paired": paired, "max_err": float(err.max()),
                              "p99_err": float(np.quantile(err, 0.99)), "mean_err": float(err.mean()),
                              "us_per_1k": round(dt * 1e6, 2), "logit_x_range": [float(zx.min()), float(zx.max())],
                              "coalition_logit_range": [float(Lz.min()), float(Lz.max())], **frac}),
                  flush=True)


if __name__ == "__main__":
    main()
