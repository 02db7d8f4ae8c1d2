#!/usr/bin/env python3
"""k-NN (SMOTE self-search, k=5) at the bench shapes: engines x candidate slices.

    python tools/knn_lab.py [--reps 20] [--engines fp32,bf16x3r] [--json out.json]

Shapes: DP1 (the 10M-row bench's 13.6k minority rows against themselves) and the DP=8 global-scope
rank (its 13.6k minority rows against all 8 ranks' 108.8k).  For every nsplit the event-timed
median of the whole knn_topk call (prep + search + merge) and whether the lists equal the
auto-split lists exactly.  (r4: a pilot search seeding every slice's threshold was measured here
too, 1-3% slower at every split count -- profiles/r4_g/knn_lab.json -- and removed.)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--splits", default="1,2,4,8,16,32")
    ap.add_argument("--engines", default="fp32")
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import knn as K
    from fraud_detection_amd.ops.native import native

    dev = torch.device("cuda", 0)
    m1, world = 13600, 8
    X, y = separable(2 * m1 * world + 4096, fraud_rate=0.5, seed=5, device=dev)
    xm = X[y == 1][: m1 * world]
    xm = (xm - X.mean(0)) / X.std(0)
    C = torch.zeros((xm.shape[0], 32), device=dev)
    C[:, :30] = xm
    C[:, 30] = 1.0
    shapes = {"dp1_self": (C[:m1].contiguous(), C[:m1].contiguous(), 0),
              "dp8_global_rank3": (C[3 * m1: 4 * m1].contiguous(), C, 3 * m1)}
    out = {"reps": a.reps, "flush": os.environ.get("FDX_KNN_FLUSH", "4"), "shapes": {}}

    def timed(fn):
        for _ in range(3):
            fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
        ev[0].record()
        for i in range(a.reps):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize()
        return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]))

    splitter = {"fp32": "knn_splits", "fp32lds": "knn_lds_splits", "bf16x3": "knn3_splits",
                "bf16x3r": "knn3r_splits", "b3top": "knn_b3top_splits"}
    for name, (Q, Cc, off) in shapes.items():
        mq, mc = Q.shape[0], Cc.shape[0]
        ref = K.knn_topk(Q, Cc, 5, off, engine="fp32")
        for eng in a.engines.split(","):
            mqp = (mq + 31) // 32 * 32 if eng != "fp32lds" else (mq + 127) // 128 * 128
            auto = getattr(native(), splitter[eng])(mqp, (mc + 31) // 32 * 32)
            rec = {"engine": eng, "mq": mq, "mc": mc, "auto_nsplit": int(auto), "cases": []}
            for ns in sorted({int(v) for v in a.splits.split(",")} | {int(auto)}):
                f = lambda: K.knn_topk(Q, Cc, 5, off, engine=eng, nsplit=ns)  # noqa: E731
                got = f()
                ms = timed(f)
                if eng in ("bf16x3r", "b3top"):
                    dg = {}
                    K.knn_topk(Q, Cc, 5, off, engine=eng, nsplit=ns, _diag=dg)
                    dg.pop("counts", None)
                    print(json.dumps({name: {"engine": eng, "nsplit": ns, "lists": dg}}), flush=True)
                case = {"engine": eng, "nsplit": ns, "ms": round(ms, 4),
                        "lists_match_frac": float((got == ref).all(1).float().mean().item()),
                        "tflops_equiv": round(2.0 * mq * mc * 32 / (ms * 1e-3) / 1e12, 1),
                        "lists_equal": bool((got == ref).all().item())}
                rec["cases"].append(case)
                print(json.dumps({name: case}), flush=True)
            best = min(rec["cases"], key=lambda c: c["ms"])
            base = [c for c in rec["cases"] if c["nsplit"] == auto][0]
            rec["best"], rec["auto"] = best, base
            out["shapes"][f"{name}:{eng}"] = rec
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
