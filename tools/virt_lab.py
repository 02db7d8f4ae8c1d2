"""Virtual-SMOTE attribution lab (event timings, one GPU): the bench shape's logistic passes over
(a) the stored real rows only, (b) the real rows + virtual samples (ops/logreg.VirtualSmote),
(c) the real rows + materialised SMOTE rows, and the bucket sort's stages.

    python tools/virt_lab.py [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops.native import native, ptr, stream_of


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(float(np.median(ts)), 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-real", type=int, default=8_000_000)
    ap.add_argument("--n-new", type=int, default=7_972_800)
    ap.add_argument("--mq", type=int, default=13_600)
    ap.add_argument("--json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    real = (torch.randn(a.n_real, 32, generator=g) * 0.5).to(torch.bfloat16)
    real[:, 30] = 1.0
    real[:, 31] = (torch.rand(a.n_real, generator=g) < 0.002).to(torch.bfloat16)
    real = real.to(dev)
    par = (torch.randn(a.mq, 32, generator=g) + 1.0).to(torch.bfloat16)
    par[:, 30] = 1.0
    par[:, 31] = 1.0
    par = par.to(dev)
    nbr = torch.randint(0, a.mq, (a.mq, 5), generator=g, dtype=torch.int32).to(dev)
    v = L.VirtualSmote(par, nbr, a.n_new).prepare()
    full = torch.empty((a.n_real + a.n_new, 32), dtype=torch.bfloat16, device=dev)
    full[: a.n_real] = real
    v.materialize(full[a.n_real:])
    m = native()
    ws = L.LRWorkspace(dev)
    ws.reset(np.r_[np.random.default_rng(1).normal(0, 0.1, 30), -1.0, 0.0])
    s = stream_of(real)
    n_all = a.n_real + a.n_new
    out = {}
    for h, name in ((8, "hess8"), (0, "grad")):
        out[f"{name}_real_only_us"] = timed(lambda: L._pass(m, real, ws, h, 0, a.n_real, 4.0, s, done=False))
        out[f"{name}_virtual_us"] = timed(lambda: L._pass(m, real, ws, h, 0, n_all, 4.0, s, done=False, virtual=v))
        out[f"{name}_stored_us"] = timed(lambda: L._pass(m, full, ws, h, 0, n_all, 4.0, s, done=False))
    out["sub16_virtual_us"] = timed(lambda: L._pass(m, real, ws, 16, 0, n_all, 4.0, s, done=False, sub=16, virtual=v))
    out["sub16_stored_us"] = timed(lambda: L._pass(m, full, ws, 16, 0, n_all, 4.0, s, done=False, sub=16))
    out["prepare_us"] = timed(lambda: L.VirtualSmote(par, nbr, a.n_new).prepare())
    out["smote_generate_us"] = timed(lambda: v.materialize(full[a.n_real:]))
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
