"""Native RCCL communicator on the one GPU a test box has (world_size 1): init through a
torch.distributed store, all-reduce / all-gather / variable-count all-gather / broadcast on the
compute stream."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_native_rccl_single_rank(dev):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from fraud_detection_amd.parallel.rccl import NativeRCCL

        nat = NativeRCCL(0, 1, 0)
        assert nat.verify()
        x = torch.arange(1088, dtype=torch.float64, device=dev)
        nat.all_reduce_(x)
        g = nat.all_gather(torch.ones(5, device=dev))
        nat.broadcast_(x)
        torch.cuda.synchronize()
        assert torch.equal(x.cpu(), torch.arange(1088, dtype=torch.float64))
        assert g.shape == (1, 5)
        # variable-count all-gather (C3): minority rows and int32 neighbour lists, compact output
        rows = torch.randn(37, 32, device=dev)
        out = nat.all_gatherv(rows, [37])
        nbr = torch.randint(0, 37, (37, 5), dtype=torch.int32, device=dev)
        nout = nat.all_gatherv(nbr, [37])
        empty = nat.all_gatherv(torch.empty((0, 32), device=dev), [0])
        torch.cuda.synchronize()
        assert torch.equal(out, rows) and torch.equal(nout, nbr) and empty.shape == (0, 32)
        nat.close()
    finally:
        dist.destroy_process_group()


def test_communicator_gathers_rows_on_the_native_path(dev, monkeypatch):
    """Communicator.all_gather_rows takes the native grouped send/recv path when the native
    communicator is up (world 1 here: the trace shows the rccl path, the result is exact)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from fraud_detection_amd.parallel.comm import Communicator
        from fraud_detection_amd.parallel.rccl import NativeRCCL

        c = Communicator(device=dev)
        c.world_size = 1  # a world-1 group never takes collectives: attach the native comm by hand
        c._native = NativeRCCL(0, 1, 0)
        c.trace = []
        x = torch.randn(11, 32, device=dev)
        got, counts = c._native_gather(x, [11])
        torch.cuda.synchronize()
        assert torch.equal(got, x) and counts == [11]
        c.close()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


class _World1AsDP:
    """A world-1 native RCCL communicator presented as a 2-rank one: drives the data-parallel code
    path (lean SGD step: pass -> native all-reduce -> update) on one GPU, the reduction an identity."""

    def __init__(self, nat):
        self._native, self.world_size, self.rank = nat, 2, 0

    def all_reduce_scalar(self, x, op="sum"):
        return x

    def all_reduce_(self, t, op="sum"):
        return self._native.all_reduce_(t)


def test_dp_sgd_hipgraph_replay_is_bitwise_the_eager_fit(dev, monkeypatch):
    """the DP SGD schedule captured into hipGraphs (with the native RCCL all-reduces)
    replays bitwise the eager DP fit, and the eager DP fit equals the single-process persistent fit
    (integer step sums); a second fit on the same buffers replays the cached graphs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from fraud_detection_amd.ops import logreg as L
        from fraud_detection_amd.parallel.rccl import NativeRCCL

        g = torch.Generator().manual_seed(3)
        real = torch.randn(1_200_000, 32, generator=g)
        real[:, 30] = 1.0
        real[:, 31] = (torch.rand(1_200_000, generator=g) < 0.03).float()
        par = torch.randn(400, 32, generator=g) + 0.7
        par[:, 30] = 1.0
        par[:, 31] = 1.0
        nbr = torch.stack([torch.randperm(400, generator=g)[:5] for _ in range(400)]).to(torch.int32)
        rows = real.to(torch.bfloat16).to(dev)
        v = L.VirtualSmote(par.to(torch.bfloat16).to(dev), nbr.to(dev), 1_000_000, seed=3)
        comm = _World1AsDP(NativeRCCL(0, 1, 0))
        kw = dict(virtual=v, epoch_batches=L.SGD_EPOCH_BATCHES, subsample=L.SGD_SUB,
                  extra_epochs=L.SGD_EXTRA_EPOCHS, avg_from=L.SGD_AVG_FROM)
        monkeypatch.setenv("FDX_DP_GRAPH", "0")  # eager (the default)
        eager = L.sgd_fit(rows, comm=comm, workspace=L.LRWorkspace(dev), **kw).as_fit_info()
        monkeypatch.setenv("FDX_DP_GRAPH", "1")
        ws = L.LRWorkspace(dev)
        a = L.sgd_fit(rows, comm=comm, workspace=ws, **kw).as_fit_info()
        assert len(ws._dp_graphs) == 1
        b = L.sgd_fit(rows, comm=comm, workspace=ws, **kw).as_fit_info()  # cached graphs replayed
        assert len(ws._dp_graphs) == 1
        single = L.sgd_fit(rows, **kw).as_fit_info()
        for f in (a, b, single):
            assert np.array_equal(f.w, eager.w) and f.n_iter == eager.n_iter, (f.n_iter, eager.n_iter)
            assert f.objective == eager.objective and f.grad_max == eager.grad_max
        comm._native.close()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
