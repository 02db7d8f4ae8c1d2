#!/usr/bin/env python3
"""Virtual-SMOTE bucket sort (smote.hip, three launches) at the bench shape: event-timed median of
VirtualSmote.prepare().  (r4: swept over the level-2 bin size with a since-removed knob -- ~2048
samples per bin 117 us, ~4096 91 us: profiles/r4_m/bucket*.log.)

    python tools/bucket_lab.py [--reps 30]
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
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops.native import native

    dev = torch.device("cuda", 0)
    X, y = separable(8_000_000, seed=1000, device=dev)
    pipe = DevicePipeline(TrainConfig(seed=42), None)
    pipe.fit(X, y)
    pipe.settle()
    v0 = pipe._virtual
    ws = L.BucketWorkspace()
    ref = L.VirtualSmote(v0.parents, v0.nbr, v0.n_new, seed=v0.seed).prepare(ws)
    cnt0 = ref.cnt.clone()
    ts = []
    for i in range(a.reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v = L.VirtualSmote(v0.parents, v0.nbr, v0.n_new, seed=v0.seed).prepare(ws)
        e1.record()
        e1.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    same = bool(torch.equal(v.cnt, cnt0))  # (off: bins take their room in arrival order)
    R, n = int(v0.nbr.numel()), int(v0.n_new)
    m = native()
    print(json.dumps({"picks": R, "samples": n,
                      "bins": int(m.smote_bucket_bins(R, n)), "us_median": round(float(np.median(ts)), 2),
                      "counts_equal_first": same}), flush=True)


if __name__ == "__main__":
    main()
