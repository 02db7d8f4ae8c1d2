#!/usr/bin/env python3
"""Per-fit wall times of DevicePipeline under DP with and without the deferred Newton check
(rehearsal: every rank on cuda:0, gloo).  Run under torch.distributed.run, e.g.

    FDX_BENCH_ONE_GPU=1 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/dp_defer_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.parallel.comm import Communicator

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(backend=os.environ.get("FDX_PROBE_BACKEND", "gloo"), device=dev)
    X, y = separable(1_600_000, seed=1000 + comm.rank, device=dev)
    for defer in (False, True):
        pipe = DevicePipeline(TrainConfig(seed=42, smote_scope="shard", deferred_check=defer), comm)
        ts = []
        for i in range(6):
            comm.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = pipe.fit(X, y)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ts.append((round((t1 - t0) * 1e3, 2), round((t2 - t0) * 1e3, 2)))
        pipe.settle()
        it = r.fit.n_iter
        if comm.rank == 0:
            print(f"defer={defer} (host ms, host+sync ms) per fit: {ts} n_iter={it} pred={pipe._full_pred}", flush=True)
    comm.close()


if __name__ == "__main__":
    main()
