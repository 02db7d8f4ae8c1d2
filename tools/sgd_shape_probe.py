#!/usr/bin/env python3
"""SGD schedule robustness on the device: the pipeline's SGD fit at several row
counts around the bench shape (fractions of 8M raw training rows) and data seeds -- steps run,
epoch gradient, converged -- plus the logistic CV job's per-fold steps and epoch gradients.

    python tools/sgd_shape_probe.py [--fracs 0.5,0.8,1,1.25] [--seeds 1000,1001] [--cv] [--json out]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fraud_detection_amd.data.synthetic import separable  # noqa: E402
from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fracs", default="0.5,0.8,1,1.25")
    ap.add_argument("--seeds", default="1000,1001")
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--cv", action="store_true")
    ap.add_argument("--order", action="store_true",
                    help="row-order probe: the pipeline fit on the CV job's fold-sorted rows, and both on a "
                         "shuffled Time column")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {"fits": [], "cv": None}
    for frac in [float(x) for x in a.fracs.split(",")]:
        for seed in [int(x) for x in a.seeds.split(",")]:
            X, y = separable(int(8_000_000 * frac), seed=seed, device=dev)
            pipe = DevicePipeline(TrainConfig(solver="sgd", storage=a.storage, seed=42))
            r = pipe.fit(X, y)
            f = r.fit
            row = {"frac": frac, "seed": seed, "post_smote_rows": int(r.n_train_rows), "steps": int(f.n_iter),
                   "grad_max": float(f.grad_max), "converged": bool(f.converged),
                   "epoch_batches": [int(v) for v in pipe.cfg.sgd_epoch_batches]}
            out["fits"].append(row)
            print(json.dumps(row), flush=True)
            del X, y, pipe, r
    if a.cv:
        from fraud_detection_amd.models.cv import DeviceCV

        X, y = separable(8_000_000, seed=1000, device=dev)
        cv = DeviceCV(TrainConfig(solver="sgd", storage=a.storage, seed=42))
        r = cv.run(X, y)
        out["cv"] = {"fold_iters": r.fold_iters, "fold_grad_max": [float(f.grad_max) for f in cv.fits],
                     "fold_rows": r.fold_rows, "final_steps": int(r.final.fit.n_iter),
                     "final_grad_max": float(r.final.fit.grad_max)}
        print(json.dumps(out["cv"]), flush=True)
    if a.order:
        from fraud_detection_amd.models.cv import DeviceCV

        X, y = separable(8_000_000, seed=1000, device=dev)
        cv = DeviceCV(TrainConfig(solver="sgd", storage=a.storage, seed=42))
        cv.run(X, y)
        perm = cv.perm
        res = {}
        for name, (Xo, yo) in {"orig": (X, y), "fold_sorted": (X[perm], y[perm]),
                               "row_shuffled": (lambda p: (X[p], y[p]))(torch.randperm(X.shape[0], device=dev))}.items():
            f = DevicePipeline(TrainConfig(solver="sgd", storage=a.storage, seed=42)).fit(Xo.contiguous(), yo.contiguous()).fit
            res[name] = {"steps": int(f.n_iter), "grad_max": float(f.grad_max)}
            print(name, json.dumps(res[name]), flush=True)
        # the CV job's fold-k training rows as a fresh pipeline fit (own scaler, own SMOTE) and the
        # CV's own fold fits on the same rows
        b = cv.bounds
        Xp, yp = X[perm], y[perm]
        res["fold_rows_pipeline"] = []
        for k in range(5):
            keep = torch.cat([torch.arange(0, int(b[k]), device=dev), torch.arange(int(b[k + 1]), X.shape[0], device=dev)])
            f = DevicePipeline(TrainConfig(solver="sgd", storage=a.storage, seed=42)).fit(
                Xp.index_select(0, keep).contiguous(), yp.index_select(0, keep).contiguous()).fit
            res["fold_rows_pipeline"].append({"steps": int(f.n_iter), "grad_max": float(f.grad_max)})
        res["cv_fold_fits"] = [{"steps": int(f.n_iter), "grad_max": float(f.grad_max)} for f in cv.fits]
        print("fold_rows_pipeline", json.dumps(res["fold_rows_pipeline"]), flush=True)
        print("cv_fold_fits", json.dumps(res["cv_fold_fits"]), flush=True)
        Xs = X.clone()
        Xs[:, 0] = Xs[torch.randperm(X.shape[0], device=dev), 0]
        cv2 = DeviceCV(TrainConfig(solver="sgd", storage=a.storage, seed=42))
        r2 = cv2.run(Xs, y)
        res["cv_time_shuffled"] = {"fold_iters": r2.fold_iters, "final_steps": int(r2.final.fit.n_iter),
                                   "final_grad_max": float(r2.final.fit.grad_max)}
        print("cv_time_shuffled", json.dumps(res["cv_time_shuffled"]), flush=True)
        out["order"] = res
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
