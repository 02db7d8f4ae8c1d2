#!/usr/bin/env python3
"""Attribute the cost of global-scope vs shard-scope SMOTE under data parallelism.

Run under torchrun (the one-GPU rehearsal: FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo, two ranks
on cuda:0).  For each scope rank 0 prints one JSON line with:
  * per-fit wall times of back-to-back fits (no sync between them) and of synchronised fits;
  * the per-phase device-synchronised times of one profiled fit (DevicePipeline profile=True);
  * the collective breakdown of the timed fits (Communicator stats);
  * the top host functions by own time over the timed fits (cProfile, rank 0).

    torchrun --nproc-per-node 2 tools/dp_scope_probe.py [--rows 2000000] [--fits 5]
"""
import argparse
import cProfile
import gc
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--fits", type=int, default=5)
    ap.add_argument("--scopes", default="shard,global")
    ap.add_argument("--solver", default="newton")
    ap.add_argument("--storage", default="bf16")
    ap.add_argument("--smote-virtual", type=int, default=1, help="0: stored SMOTE rows (smote_generate + streamed)")
    ap.add_argument("--phases", type=int, default=0, help="1: per-phase synced times of every synced fit")
    ap.add_argument("--gc-freeze", type=int, default=0, help="1: gc.freeze() after the warm-up fits")
    a = ap.parse_args()
    gc_pauses = []  # (generation, ms) of every collection: a host pause that stalls one rank
    gc_t0 = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t0[0] = time.perf_counter()
        else:
            gc_pauses.append((info["generation"], (time.perf_counter() - gc_t0[0]) * 1e3))
    gc.callbacks.append(_gc_cb)
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.parallel.comm import Communicator

    local = 0 if os.environ.get("FDX_BENCH_ONE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = Communicator(backend=os.environ.get("FDX_BENCH_BACKEND") or None, device=dev)
    n_train = a.rows - a.rows // 5
    X, y = separable(n_train, seed=1000 + comm.rank, device=dev)
    for scope in a.scopes.split(","):
        pipe = DevicePipeline(TrainConfig(seed=42, solver=a.solver, smote_scope=scope, storage=a.storage,
                                       virtual_smote=bool(a.smote_virtual)), comm)
        for _ in range(2):
            pipe.fit(X, y)
        if a.gc_freeze:
            gc.collect()
            gc.freeze()
        comm.barrier()
        torch.cuda.synchronize(dev)
        comm.stats.reset()
        gc_pauses.clear()
        prof = cProfile.Profile()
        prof.enable()
        t0 = time.perf_counter()
        for _ in range(a.fits):
            r = pipe.fit(X, y)
        torch.cuda.synchronize(dev)
        back_to_back = (time.perf_counter() - t0) / a.fits
        prof.disable()
        coll = comm.collective_summary()
        synced, phased = [], []
        comm.stats.reset()
        from fraud_detection_amd.ops import logreg as L
        L.FLAG_WAITS.clear()
        for _ in range(a.fits):
            comm.barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            r = pipe.fit(X, y, profile=bool(a.phases))
            pipe.settle()  # every rank verifies its pending fit here (a deferred check waits)
            torch.cuda.synchronize(dev)
            synced.append(round((time.perf_counter() - t1) * 1e3, 3))
            if a.phases:
                phased.append({k: round(v * 1e3, 3) for k, v in r.timings.items()})
        coll_synced = comm.collective_summary()
        flag_waits = sorted(L.FLAG_WAITS, reverse=True)[:5]
        gcs = sorted(gc_pauses, key=lambda g: -g[1])[:5]
        p = pipe.fit(X, y, profile=True)
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(18)
        out = {"scope": scope, "rank": comm.rank, "ms_back_to_back": round(back_to_back * 1e3, 3),
               "ms_synced": synced, "phase_ms": {k: round(v * 1e3, 3) for k, v in p.timings.items()},
               "n_train_rows": int(r.n_train_rows), "n_synthetic": int(r.n_synthetic),
               "newton_iters": int(r.fit.n_iter), "virtual_smote": pipe._virtual is not None,
               "collectives": coll, "storage": a.storage, "solver": a.solver,
               "collectives_synced_fits": coll_synced, "longest_flag_waits_ms": [round(x * 1e3, 3) for x in flag_waits],
               "gc_collections": len(gc_pauses), "longest_gc_pauses_ms": [[g, round(t, 3)] for g, t in gcs],
               "gc_freeze": bool(a.gc_freeze)}
        if phased:
            out["phases_synced"] = phased
        print(json.dumps(out), flush=True)  # every rank: the two ranks share one GPU
        if comm.rank == 0:
            print(s.getvalue(), file=sys.stderr, flush=True)
    comm.close()


if __name__ == "__main__":
    main()
