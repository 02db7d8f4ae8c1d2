#!/usr/bin/env python3
"""Host <-> device transfer probe for config 2's host-to-host batch predict (1M x 30 fp32 =
120 MB in, 8 MB out): what each way of getting pageable caller memory onto the GPU costs.

    python tools/h2d_probe.py [--rows 1000000]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import time

import numpy as np
import torch


def t_med(fn, reps=7):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X = np.random.default_rng(0).normal(size=(a.rows, 30)).astype(np.float32)
    nb = X.nbytes
    out = {"bytes": nb}
    d = torch.empty((a.rows, 30), dtype=torch.float32, device=dev)
    pin = torch.empty((a.rows, 30), dtype=torch.float32, pin_memory=True)
    src = torch.from_numpy(X)
    out["pageable_h2d_GBps"] = nb / t_med(lambda: d.copy_(src)) / 1e9
    out["pinned_h2d_GBps"] = nb / t_med(lambda: d.copy_(pin, non_blocking=True)) / 1e9
    out["np_copy_to_pinned_1thr_GBps"] = nb / t_med(lambda: np.copyto(pin.numpy(), X)) / 1e9
    for T in (4, 8, 16):
        ex = cf.ThreadPoolExecutor(T)
        pv = pin.numpy()
        sl = [slice(i * a.rows // T, (i + 1) * a.rows // T) for i in range(T)]

        def par():
            list(ex.map(lambda s: np.copyto(pv[s], X[s]), sl))
        out[f"np_copy_to_pinned_{T}thr_GBps"] = nb / t_med(par) / 1e9
        ex.shutdown()
    rt = torch.cuda.cudart()

    def reg():
        assert int(rt.cudaHostRegister(X.ctypes.data, nb, 0)) == 0
        assert int(rt.cudaHostUnregister(X.ctypes.data)) == 0
    out["host_register_unregister_ms"] = t_med(reg) * 1e3
    rt.cudaHostRegister(X.ctypes.data, nb, 0)
    out["registered_h2d_GBps"] = nb / t_med(lambda: d.copy_(src, non_blocking=True)) / 1e9
    rt.cudaHostUnregister(X.ctypes.data)
    o = torch.empty(a.rows * 2, dtype=torch.float32, device=dev)
    ho = torch.empty(a.rows * 2, dtype=torch.float32, pin_memory=True)
    out["pinned_d2h_8MB_GBps"] = o.numel() * 4 / t_med(lambda: ho.copy_(o, non_blocking=True)) / 1e9
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
