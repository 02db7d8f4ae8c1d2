#!/usr/bin/env python3
"""Attribute the one-GPU two-process rehearsal's intermittent fit stall.

Run with two ranks on ONE GPU (FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo) under
``rocprofv3 --marker-trace --kernel-trace``: every rank runs --fits synchronised fits of the bench
pipeline (global-scope SMOTE), each inside a roctx range ``fit<i>:<solver>``, and prints its host
time per fit.  ``--analyze <dir>`` then reads the traces of both processes and, for every fit
window, reports the device time the rank's kernels used, the longest kernel, the idle time inside
the window and the other rank's kernels that overlapped it -- i.e. whether a stalled fit waited
with an idle device (host or collective wait) or ran a kernel long (the card time-sliced between
the two processes).

    FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        tools/stall_probe.py --fits 12
    python tools/stall_probe.py --analyze <rocprofv3 output dir> [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch

    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.obs.tracing import roctx_range
    from fraud_detection_amd.parallel.comm import Communicator

    os.environ.setdefault("FDX_COMM_TIMING", "1")  # per-collective host times of the staged path

    def cpu_stat():  # cgroup v2 CPU accounting: throttling of the box's CPU quota
        try:
            with open("/sys/fs/cgroup/cpu.stat") as fh:
                return {k: int(v) for k, v in (ln.split() for ln in fh if ln.strip())}
        except OSError:
            return {}

    def cpu_max():
        try:
            with open("/sys/fs/cgroup/cpu.max") as fh:
                return fh.read().strip()
        except OSError:
            return ""
    st0 = cpu_stat()
    local = 0 if os.environ.get("FDX_BENCH_ONE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = Communicator(backend=os.environ.get("FDX_BENCH_BACKEND") or None, device=dev)
    n_train = a.rows - a.rows // 5
    X, y = separable(n_train, seed=1000 + comm.rank, device=dev)
    out = {}
    for solver in a.solvers.split(","):
        pipe = DevicePipeline(TrainConfig(seed=42, solver=solver, smote_scope="global"), comm)
        for _ in range(2):
            pipe.fit(X, y)
        pipe.settle()
        torch.cuda.synchronize()
        comm.barrier()
        ms, thr = [], []
        for i in range(a.fits):
            c0 = cpu_stat().get("nr_throttled", 0)
            t0 = time.perf_counter()
            with roctx_range(f"fit{i}:{solver}"):
                pipe.fit(X, y)
                pipe.settle()
                torch.cuda.synchronize()
            ms.append(round((time.perf_counter() - t0) * 1e3, 3))
            thr.append(cpu_stat().get("nr_throttled", 0) - c0)  # CPU-quota throttles inside the fit
            comm.barrier()
        out[solver] = ms
        out[solver + "_throttled_periods"] = thr
    st1 = cpu_stat()
    thr = {k: st1[k] - st0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec") if k in st1}
    print(json.dumps({"rank": comm.rank, "pid": os.getpid(), "fit_ms": out, "cgroup_cpu_max": cpu_max(),
                      "cgroup_throttling_delta": thr, "collectives": comm.collective_summary()}), flush=True)
    comm.close()


def _rows(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def analyze(a):
    kern = _rows(os.path.join(a.analyze, "**", "*kernel_trace.csv"))
    mark = _rows(os.path.join(a.analyze, "**", "*marker_api_trace.csv"))
    by_pid = {}
    for r in kern:
        pid = r.get("Process_Id") or r.get("Thread_Id")  # kernel rows carry the dispatching thread
        by_pid.setdefault(pid, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                           r["Kernel_Name"][:60]))
    for v in by_pid.values():
        v.sort()
    fits = []
    for r in mark:
        nm = r.get("Function") or r.get("Marker_Name") or r.get("Operation") or ""
        if not nm.startswith("fit"):
            continue
        fits.append((r.get("Process_Id") or r.get("Thread_Id"), nm, int(r["Start_Timestamp"]),
                     int(r["End_Timestamp"])))
    res = []
    for pid, nm, t0, t1 in sorted(fits, key=lambda x: (x[1], x[0])):
        mine = [(max(s, t0), min(e, t1), k) for s, e, k in by_pid.get(pid, []) if e > t0 and s < t1]
        busy = 0
        last = t0
        idle = 0
        for s, e, _ in mine:
            if s > last:
                idle += s - last
            busy += max(0, e - max(s, last))
            last = max(last, e)
        idle += max(0, t1 - last)
        longest = max(mine, key=lambda x: x[1] - x[0]) if mine else (0, 0, "")
        other = [(s, e) for p, v in by_pid.items() if p != pid for s, e, _ in v if e > t0 and s < t1]
        res.append({"pid": pid, "fit": nm, "window_ms": round((t1 - t0) / 1e6, 3),
                    "own_kernel_busy_ms": round(busy / 1e6, 3), "idle_ms": round(idle / 1e6, 3),
                    "longest_kernel": longest[2], "longest_kernel_ms": round((longest[1] - longest[0]) / 1e6, 3),
                    "other_rank_kernels_overlapping": len(other),
                    "other_rank_busy_ms": round(sum(min(e, t1) - max(s, t0) for s, e in other) / 1e6, 3)})
    med = sorted(r["window_ms"] for r in res)[len(res) // 2] if res else 0
    stalled = [r for r in res if r["window_ms"] > 2.0 * med]
    summary = {"fits": len(res), "median_window_ms": med, "stalled": stalled,
               "verdict": ("no stalled fit in this run" if not stalled else
                           "stalled windows: compare idle_ms (device idle: a host / collective wait) with "
                           "longest_kernel_ms (a kernel ran long: the card time-sliced)")}
    print(json.dumps(summary, indent=1))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"summary": summary, "fits": res}, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--fits", type=int, default=12)
    ap.add_argument("--solvers", default="sgd,newton")
    ap.add_argument("--analyze", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
