#!/usr/bin/env python3
"""Collective sequence of ONE data-parallel fit (FDX_COMM_TRACE): run under torchrun, e.g. two
ranks on one GPU over gloo (FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo) as a rehearsal of the
8-GPU RCCL run.  Rank 0 prints one JSON line: the ordered (op, path, bytes) list per fit and the
Newton iteration count, for the bench's bf16 Newton and SGD configurations.

    torchrun --nproc-per-node 2 tools/dp_trace.py [--rows 2000000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("FDX_COMM_TRACE", "1")

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig
    from fraud_detection_amd.parallel.comm import Communicator

    local = 0 if os.environ.get("FDX_BENCH_ONE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = Communicator(backend=os.environ.get("FDX_BENCH_BACKEND") or None, device=dev)
    X, y = separable(a.rows, seed=1000 + comm.rank, device=dev)
    out = {}
    for name, kw in (("newton_shard", dict(solver="newton", smote_scope="shard")),
                     ("sgd_shard", dict(solver="sgd", smote_scope="shard")),
                     ("newton_global", dict(solver="newton", smote_scope="global"))):
        pipe = DevicePipeline(TrainConfig(seed=42, **kw), comm)
        pipe.fit(X, y)  # warm-up
        torch.cuda.synchronize(dev)
        comm.trace.clear()
        res = pipe.fit(X, y)
        pipe.settle()
        torch.cuda.synchronize(dev)
        out[name] = {"collectives": len(comm.trace), "trace": [list(t) for t in comm.trace],
                     "newton_iters": int(res.fit.n_iter)}
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
