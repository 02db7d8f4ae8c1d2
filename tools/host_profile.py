"""Host-side (Python) cost of one bench fit: cProfile over K back-to-back fits of the bench
configuration (10M rows, bf16, Newton), functions by own time and by cumulative time per fit.

The device timeline (tools/timeline.py) shows the GPU idle only at the fit boundary, while the
host returns from the Newton loop and enqueues the next fit's first kernels; this tool says which
Python calls that host path spends its time in.

    python tools/host_profile.py [--steps 30] [--rows 10000000] [--storage bf16]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--solver", default="sgd")
    a = ap.parse_args()
    import torch

    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig

    dev = torch.device("cuda", 0)
    n_train = a.rows - a.rows // 5
    X, y = separable(n_train, seed=1000, device=dev)
    pipe = DevicePipeline(TrainConfig(solver=a.solver, storage=a.storage, seed=42, smote_scope="global"))
    for _ in range(3):
        pipe.fit(X, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pipe.fit(X, y)
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / a.steps
    # host time spent inside fit() per call, back to back (the device queue never drains if this
    # stays below the device time per fit), and the same with the device idle at every call
    host = []
    for _ in range(a.steps):
        t1 = time.perf_counter()
        pipe.fit(X, y)
        host.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    idle = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pipe.fit(X, y)
        idle.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    import numpy as np
    print(f"[host_profile] host time in fit(), back to back: median {np.median(host) * 1e3:.4f} ms; "
          f"from an idle device: median {np.median(idle) * 1e3:.4f} ms (blocks on the minority count)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        pipe.fit(X, y)
    torch.cuda.synchronize()
    pr.disable()
    print(f"[host_profile] plain {plain * 1e3:.4f} ms/fit over {a.steps} fits (profiled run below is slower)")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        st = pstats.Stats(pr, stream=s)
        st.sort_stats(key).print_stats(a.top)
        print(f"==== by {key} (totals over {a.steps} fits) ====")
        print(s.getvalue())


if __name__ == "__main__":
    main()
