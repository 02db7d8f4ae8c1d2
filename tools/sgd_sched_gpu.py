#!/usr/bin/env python3
"""SGD schedule candidates on the device (the CV folds run the extra epoch).

For every candidate (per-epoch step scalars, momentum, minibatch counts) the pipeline's SGD fit at
several shapes / data seeds AND the logistic CV job's 5 folds + final fit: steps run, epoch gradient,
and the exact training objective of the returned weights against the Newton optimum on the same
rows (the bench's `objective_rel_gap_vs_newton`).  One JSON line per (candidate, case).

    python tools/sgd_sched_gpu.py [--json out.json] [--cands base,lr3_06,...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fraud_detection_amd.data.synthetic import separable  # noqa: E402
from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig  # noqa: E402

CANDS = {
    "base": {},
    "lr3_06": {"sgd_lr": (0.6, 0.8, 0.6)},
    "lr3_05": {"sgd_lr": (0.6, 0.8, 0.5)},
    "lr_07": {"sgd_lr": (0.6, 0.7, 0.7)},
    "lr23_09_06": {"sgd_lr": (0.6, 0.9, 0.6)},
    "mom05": {"sgd_momentum": 0.5},
    "mom06_lr3_06": {"sgd_momentum": 0.6, "sgd_lr": (0.6, 0.8, 0.6)},
    # the extra epoch (run only while not converged) with its own, smaller minibatch count
    "x2": {"sgd_epoch_batches": (4, 6, 6, 2)},
    "x3": {"sgd_epoch_batches": (4, 6, 6, 3)},
    "x4": {"sgd_epoch_batches": (4, 6, 6, 4)},
    "x3_lr06": {"sgd_epoch_batches": (4, 6, 6, 3), "sgd_lr": (0.6, 0.8, 0.8, 0.6)},
    "x3_lr04": {"sgd_epoch_batches": (4, 6, 6, 3), "sgd_lr": (0.6, 0.8, 0.8, 0.4)},
    "x3_lr03": {"sgd_epoch_batches": (4, 6, 6, 3), "sgd_lr": (0.6, 0.8, 0.8, 0.3)},
    "x4_lr04": {"sgd_epoch_batches": (4, 6, 6, 4), "sgd_lr": (0.6, 0.8, 0.8, 0.4)},
    "x6_lr04": {"sgd_lr": (0.6, 0.8, 0.8, 0.4)},
    "x6_lr05": {"sgd_lr": (0.6, 0.8, 0.8, 0.5)},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", default=",".join(CANDS))
    ap.add_argument("--shapes", default="1.0:1000,0.8:1000,1.25:1000,1.0:1001")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    names = a.cands.split(",")
    out = []
    data = {}
    for sh in a.shapes.split(","):
        frac, seed = sh.split(":")
        data[sh] = separable(int(8_000_000 * float(frac)), seed=int(seed), device=dev)
    newton_w = {}
    for sh, (X, y) in data.items():
        newton_w[sh] = DevicePipeline(TrainConfig(seed=42, deferred_check=False)).fit(X, y).w
    for name in names:
        kw = CANDS[name]
        for sh, (X, y) in data.items():
            pipe = DevicePipeline(TrainConfig(solver="sgd", seed=42, **kw))
            r = pipe.fit(X, y)
            f = r.fit
            mine = pipe.training_objective(r)["objective"]
            opt = pipe.training_objective(r, w=newton_w[sh])["objective"]
            row = {"cand": name, "case": sh, "steps": int(f.n_iter), "grad_max": float(f.grad_max),
                   "converged": bool(f.converged), "rel_gap": float((mine - opt) / opt)}
            out.append(row)
            print(json.dumps(row), flush=True)
            del pipe, r
        from fraud_detection_amd.models.cv import DeviceCV

        X, y = data[a.shapes.split(",")[0]]
        cv = DeviceCV(TrainConfig(solver="sgd", seed=42, **kw))
        r = cv.run(X, y)
        row = {"cand": name, "case": "cv", "fold_iters": list(r.fold_iters),
               "fold_grad_max": [round(float(f.grad_max), 6) for f in cv.fits], "final_steps": int(r.final.fit.n_iter),
               "cv_auc_mean": float(r.cv_auc_mean) if hasattr(r, "cv_auc_mean") else None}
        out.append(row)
        print(json.dumps(row), flush=True)
        del cv, r
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
