#!/usr/bin/env python3
"""Phase timing of the on-device Newton update (logreg.hip newton_update_kernel<31>) from s_memtime
stamps: load -> affine map -> gradient/objective -> Cholesky -> substitutions -> state write.

    python tools/newton_stamps.py [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["global loads -> LDS", "affine map of the sums", "gradient / objective / decision",
          "Cholesky factorization", "triangular solves", "state write-back"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops import scaler as S
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    nat = native()
    dev = torch.device("cuda", 0)
    X, y = separable(2_000_000, seed=1, device=dev)
    rows = torch.empty((X.shape[0], 32), device=dev, dtype=torch.bfloat16)
    st = S.scaler_fit_cast(X, y, rows)
    ws = L.LRWorkspace(dev)
    w0 = np.r_[np.random.default_rng(0).normal(0, 0.1, 30), -3.0, 0.0]
    s = stream_of(X)
    stamps = torch.zeros(8, dtype=torch.int64, device=dev)
    per = []
    for r in range(a.reps):
        ws.reset(w0)
        nat.logreg_fold(ptr(ws.state), ptr(st.aff), ptr(ws.w32), s)
        L._pass(nat, rows, ws, 1, 0, rows.shape[0], 4.0, s, done=False)
        nat.newton_update_stamped(ptr(ws.red), ptr(ws.state), ptr(ws.w32), ptr(ws.done), 1.0, ptr(st.aff),
                                  ptr(stamps), s)
        torch.cuda.synchronize()
        t = stamps.cpu().numpy().astype(np.int64)
        if r >= 5:
            per.append(np.diff(t[:7]))
    per = np.array(per)
    med = np.median(per, 0)
    print(f"newton_update_kernel<31> phases (s_memtime ticks, median of {len(per)}; total {med.sum():.0f})")
    for name, v in zip(PHASES, med):
        print(f"  {name:34s} {v:8.0f}")


if __name__ == "__main__":
    main()
