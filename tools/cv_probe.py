#!/usr/bin/env python3
"""The device CV job (models/cv.py DeviceCV) at the bench shape: per-run wall / device times and a
host profile of the last run -- where a fold's time goes when its device time exceeds its kernels.

    python tools/cv_probe.py [--rows-per-gpu 10000000] [--runs 4] [--solver newton] [--host-profile]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--solver", default="newton")
    ap.add_argument("--host-profile", action="store_true")
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.cv import DeviceCV
    from fraud_detection_amd.models.pipeline import TrainConfig

    dev = torch.device("cuda", 0)
    n_test = a.rows_per_gpu // 5
    X, y = separable(a.rows_per_gpu - n_test, seed=1000, device=dev)
    Xt, yt = separable(n_test, seed=5000, device=dev)
    cv = DeviceCV(TrainConfig(seed=42, solver=a.solver))
    for r in range(a.runs):
        torch.cuda.synchronize()
        last = r == a.runs - 1
        prof = cProfile.Profile() if (last and a.host_profile) else None
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        res = cv.run(X, y, Xt, yt)
        if prof:
            prof.disable()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"run": r, "wall_ms": round(ms, 3), "total_ms": round(res.total_ms, 3),
                          "prep_ms": round(res.prep_ms, 3), "fold_ms": [round(v, 3) for v in res.fold_ms],
                          "final_ms": round(res.final_ms, 3), "fold_iters": res.fold_iters,
                          "cv_auc": round(res.cv_auc_mean, 6), "test_auc": round(res.test_auc, 6)}), flush=True)
        if prof:
            s = io.StringIO()
            pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(30)
            print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
