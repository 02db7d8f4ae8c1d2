#!/usr/bin/env python3
"""One bench step from a rocprofv3 kernel trace, in launch order, with the idle gap before each
kernel (the host-latency view of a fit).

    python tools/timeline.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--step -1] [--anchor NAME]

A step starts at each launch of the anchor kernel (default: the fused scaler pass)."""
import argparse
import csv
import re


def short(name: str) -> str:
    n = name.replace("void ", "").replace("fdx::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1)
    ap.add_argument("--anchor", default="scaler_stats_cast_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if a.anchor in k[2]]
    if not starts:
        raise SystemExit("anchor kernel not found")
    i0 = starts[a.step]
    nxt = [i for i in starts if i > i0]
    i1 = nxt[0] if nxt else len(ks)
    # include the launches just before the anchor that belong to the step (same fit: < 100 us gap)
    while i0 > 0 and ks[i0][0] - ks[i0 - 1][1] < 100_000 and "fdx" in ks[i0 - 1][2]:
        i0 -= 1
    t0 = ks[i0][0]
    busy = gaps = 0
    prev = None
    print(f"{'start_us':>9} {'gap_us':>7} {'dur_us':>8}  kernel")
    for s, e, n in ks[i0:i1]:
        gap = 0 if prev is None else max(0, s - prev)
        busy += e - s
        gaps += gap
        print(f"{(s - t0) / 1e3:9.1f} {gap / 1e3:7.1f} {(e - s) / 1e3:8.1f}  {short(n)}")
        prev = e
    print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle gaps {gaps / 1e3:.1f} us")


if __name__ == "__main__":
    main()
