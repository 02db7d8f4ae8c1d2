#!/usr/bin/env python3
"""Idle gaps between back-to-back kernels after a kernel that stores to mapped pinned host memory
(the count scan's total word, the state export) -- run under rocprofv3 --kernel-trace.

    rocprofv3 --kernel-trace --output-format csv -d out -o run -- python3 tools/gap_probe.py
    python tools/gap_probe.py --report out/run_kernel_trace.csv

Each round enqueues, with the host far ahead of the device: count -> scan (total to a mapped word,
or to device memory only) -> fused scaler pass -> state export (to a mapped slot, or a device
copy) -> a short kernel.  The report prints the median gap in front of the kernel that follows
each variant.
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch

    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import scaler as S
    from fraud_detection_amd.ops.layout import NCOLS
    from fraud_detection_amd.ops.native import native, ptr, stream_of

    dev = torch.device("cuda", 0)
    m = native()
    X, y = separable(8_000_000, seed=1, device=dev)
    rows = torch.empty((X.shape[0], NCOLS), dtype=torch.bfloat16, device=dev)
    n = y.shape[0]
    nb = 512
    counts = torch.empty(nb, device=dev, dtype=torch.int64)
    total = torch.empty(1, device=dev, dtype=torch.int64)
    word = torch.empty(1, dtype=torch.int64, pin_memory=True)
    hdev = int(m.host_device_pointer(word.data_ptr()))
    st = torch.zeros(256, dtype=torch.float64, device=dev)
    slot = torch.empty(256, dtype=torch.float64, pin_memory=True)
    sdev = int(m.host_device_pointer(slot.data_ptr()))
    dcopy = torch.empty(256, dtype=torch.float64, device=dev)
    s = stream_of(y)
    S.scaler_fit_cast(X, y, rows)
    torch.cuda.synchronize()
    for r in range(40):
        mapped = r % 2 == 0
        m.compact_count(ptr(y), n, 1, ptr(counts), nb, s)
        m.exclusive_scan_small(ptr(counts), nb, ptr(total), s, hdev if mapped else 0)
        S.scaler_fit_cast(X, y, rows)       # "after scan, mapped" / "after scan, device"
        if mapped:
            m.logreg_export(ptr(st), sdev, s)
        else:
            dcopy.copy_(st)
        m.compact_count(ptr(y), n, 1, ptr(counts), nb, s)  # "after export, ..."
    torch.cuda.synchronize()
    print("gap_probe done", flush=True)


def report(path: str):
    import numpy as np

    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    scan, exp_mapped, copy_dev = [], [], []
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        g = (s1 - e0) / 1e3
        if "exclusive_scan_small" in n0 and "scaler_stats_cast" in n1:
            scan.append(g)
        elif "logreg_export" in n0 and "compact_count" in n1:
            exp_mapped.append(g)
        elif "compact_count" in n1 and "scaler" not in n0:
            copy_dev.append(g)
    gaps = {"scan(mapped) -> scaler": scan[0::2], "scan(device) -> scaler": scan[1::2],
            "export(mapped) -> count": exp_mapped, "copy(device) -> count": copy_dev}
    for k, v in gaps.items():
        if v:
            print(f"{k:28s} n={len(v):3d} median {np.median(v):7.2f} us  max {np.max(v):7.2f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--report", default=None)
    a = ap.parse_args()
    if a.report:
        report(a.report)
    else:
        run()
