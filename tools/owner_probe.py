#!/usr/bin/env python3
"""GPU-owner batch latency probe: one small zero-copy predict launch (rows in mapped pinned host
memory, results written to mapped pinned memory) and its wait, by wait method and batch size.

    python tools/owner_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from fraud_detection_amd.ops import predict as P
    from fraud_detection_amd.serve.engine import InferenceEngine

    eng = InferenceEngine.from_paths(device="cuda")
    m = P.native()
    cap = 1024
    eng.owner_input(cap)
    X = np.random.default_rng(0).normal(size=(cap, 30)).astype(np.float32)
    eng._owner_in[0][:cap].copy_(torch.from_numpy(X))
    out = {}
    for n in (1, 8, 64, 256):
        for mode in ("sync", "spin"):
            ts = []
            for i in range(2000):
                t0 = time.perf_counter()
                h = eng.run_staged_async(n, False, 0)
                if mode == "spin":
                    m.event_spin(eng._oevents[0])
                else:
                    m.event_sync(eng._oevents[0])
                ts.append(time.perf_counter() - t0)
            a = np.array(ts[200:]) * 1e6
            out[f"n{n}_{mode}"] = {"p50_us": round(float(np.percentile(a, 50)), 2), "p99_us": round(float(np.percentile(a, 99)), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
