#!/usr/bin/env python3
"""GBDT (K11) throughput on one GPU: xgboost-config boosting (100 trees, depth 5, eta 0.1) on
credit_card-shaped synthetic rows after SMOTE, plus test AUC and inference rate.

    python tools/gbdt_bench.py [--rows 10000000] [--trees 100] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.gbdt import GBDTPipeline
    from fraud_detection_amd.models.pipeline import TrainConfig
    from fraud_detection_amd.ops import gbdt as gb

    dev = torch.device("cuda", 0)
    n_test = a.rows // 5
    X, y = separable(a.rows - n_test, seed=1000, device=dev)
    Xt, yt = separable(n_test, seed=5000, device=dev)
    pipe = GBDTPipeline(TrainConfig(), gb.GBDTParams(n_estimators=a.trees, max_depth=a.depth))
    GBDTPipeline(TrainConfig(), gb.GBDTParams(n_estimators=2, max_depth=a.depth)).fit(X, y)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = pipe.fit(X, y)
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    ev = res.evaluate(Xt, yt)
    Xs = res.standardize(Xt)
    res.predict_margin(Xt)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        gb.predict_margin(Xs, res.ensemble, res._dens)
    torch.cuda.synchronize()
    pred_s = (time.perf_counter() - t1) / 5
    out = {"rows_train_post_smote": res.n_train_rows, "trees": a.trees, "depth": a.depth,
           "fit_s": round(fit_s, 4), "prep_s": round(res.timings["prep"], 4), "boost_s": round(res.timings["boost"], 4),
           "ms_per_tree": round(1000 * res.timings["boost"] / max(a.trees, 1), 3),
           "row_trees_per_s": round(res.n_train_rows * a.trees / res.timings["boost"], 1),
           "auc": round(ev["auc"], 6), "predict_rows_per_s": round(n_test / pred_s, 1),
           "scale_pos_weight": round(res.scale_pos_weight, 3)}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
