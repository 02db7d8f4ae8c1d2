#!/usr/bin/env python3
"""k-NN (SMOTE minority self-search, k=5) engine scaling on one GPU: the exact fp32 MFMA chain vs
the bf16x3 filter + exact re-score, from the 10M-row bench's 13.6k minority rows up to the 170k of
a 100M-row table (BASELINE config 5).  Minority rows of the separable generator, standardized.

    python tools/knn_bench.py [--sizes 13600,54400,170000] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="13600,27200,54400,108800,170000")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import knn as K

    dev = torch.device("cuda", 0)
    for m in (int(v) for v in a.sizes.split(",")):
        X, y = separable(2 * m + 1024, fraud_rate=0.5, seed=5, device=dev)
        xm = X[y == 1][:m]
        xm = (xm - X.mean(0)) / X.std(0)
        C = torch.zeros((xm.shape[0], 32), device=dev)
        C[:, :30] = xm
        C[:, 30] = 1.0
        res = {"minority_rows": int(C.shape[0]), "k": 5}
        ref = None
        for eng in ("fp32", "fp32lds", "bf16x3"):
            f = lambda: K.knn_topk(C, C, 5, 0, engine=eng)  # noqa: E731
            out = f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                out = f()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.reps
            res[f"{eng}_ms"] = round(dt * 1e3, 3)
            res[f"{eng}_tflops_equiv"] = round(2.0 * m * m * 32 / dt / 1e12, 1)
            if ref is None:
                ref = out
            else:
                res[f"{eng}_lists_equal_frac"] = round((out == ref).all(1).float().mean().item(), 6)
        res["speedup_lds"] = round(res["fp32_ms"] / res["fp32lds_ms"], 2)
        res["speedup_bf16x3"] = round(res["fp32_ms"] / res["bf16x3_ms"], 2)
        print(json.dumps(res), flush=True)
        del X, y, xm, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
