"""Native RCCL communicator on the one GPU a test box has (world_size 1): init through a
torch.distributed store, all-reduce / all-gather / broadcast on the compute stream."""
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
        nat.close()
    finally:
        dist.destroy_process_group()
