#!/usr/bin/env python3
"""Minimal driver for PMC runs on the solver pass: the stored-row pass over 2n rows and the
virtual-SMOTE pass over n stored + n rebuilt rows, each --reps times (rocprofv3 --pmc target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import knn as K
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops import scaler as S
    from fraud_detection_amd.ops.native import native, stream_of

    nat = native()
    dev = torch.device("cuda", 0)
    X, y = separable(n, seed=1, device=dev)
    st = S.scaler_fit(X)
    rows2 = torch.empty((2 * n, 32), device=dev, dtype=torch.bfloat16)
    S.scale_cast(X, st, labels=y, out=rows2[:n])
    S.scale_cast(X, st, labels=y, out=rows2[n:])
    idx = S.compact_indices(y, 1)
    xmin = S.scale_cast(X, st, labels=y, out_dtype="f32", idx=idx)
    nbr = K.knn_topk(xmin, xmin, 5, 0)
    vr = L.VirtualRows(K.smote_parents(xmin), nbr, 0, n, seed=42)
    vr.ensure_plan()
    ws = L.LRWorkspace(dev)
    ws.reset(np.r_[np.random.default_rng(0).normal(0, 0.2, 30), -3.0, 0.0])
    s = stream_of(X)
    for _ in range(reps):
        L._pass(nat, rows2, ws, 0, 0, 2 * n, 4.0, s, done=False)
        L._pass(nat, rows2[:n], ws, 0, 0, 2 * n, 4.0, s, done=False, vrows=vr)
    torch.cuda.synchronize()
    print("pass_probe done")


if __name__ == "__main__":
    main()
