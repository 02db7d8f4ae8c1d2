"""Shared-memory sum all-reduce of the host-staged collectives (parallel/shm_reduce.py): exact int64
sums, identical fp64 sums on every rank, back-to-back collectives of both slot parities, and a
bounded wait when a rank stops participating."""
import multiprocessing as mp

import numpy as np
import pytest

from fraud_detection_amd.parallel.shm_reduce import ShmAllReduce


def _rank(r, world, name, q, rounds):
    a = ShmAllReduce(r, world, 1 << 14, name=name, timeout_s=20)
    got = []
    for i in range(rounds):
        v = np.full(37, (r + 1) * 1000003 + i, np.int64)
        a.all_reduce_(v)
        f = np.linspace(0.1, 1.0, 9) * (r + 1) + i * 1e-3
        a.all_reduce_(f)
        got.append((int(v[0]), f.tobytes()))
    q.put((r, got))
    a.close()


def _expected(world, rounds):
    out = []
    for i in range(rounds):
        iv = sum((r + 1) * 1000003 + i for r in range(world))
        acc = np.linspace(0.1, 1.0, 9) * 1 + i * 1e-3
        for r in range(1, world):  # rank order, as every rank sums
            acc = acc + (np.linspace(0.1, 1.0, 9) * (r + 1) + i * 1e-3)
        out.append((iv, acc.tobytes()))
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_shm_all_reduce_matches_rank_order_sums(world):
    ctx = mp.get_context("spawn")
    owner = ShmAllReduce(0, world, 1 << 14, timeout_s=20)
    q = ctx.Queue()
    rounds = 50
    ps = [ctx.Process(target=_rank, args=(r, world, owner.name, q, rounds)) for r in range(1, world)]
    for p in ps:
        p.start()
    got0 = []
    for i in range(rounds):
        v = np.full(37, 1000003 + i, np.int64)
        owner.all_reduce_(v)
        f = np.linspace(0.1, 1.0, 9) + i * 1e-3
        owner.all_reduce_(f)
        got0.append((int(v[0]), f.tobytes()))
    res = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    owner.close()
    exp = _expected(world, rounds)
    assert got0 == exp
    for r in range(1, world):
        assert res[r] == exp  # bitwise the same fp64 sums on every rank


def test_shm_all_reduce_times_out_without_peers():
    a = ShmAllReduce(0, 2, 1 << 10, timeout_s=0.5)
    try:
        with pytest.raises(RuntimeError, match="stopped participating"):
            a.all_reduce_(np.ones(4))
        with pytest.raises(ValueError):
            a.all_reduce_(np.ones(1 << 12))
    finally:
        a.close()
