"""Native RCCL communicator on the one GPU a test box has (world_size 1): init through a
torch.distributed store, all-reduce / all-gather / variable-count all-gather / broadcast on the
compute stream."""
import os
import socket

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
