"""N>1 read path on CPU (gloo, world_size 2): slab partition + gather assemble exactly the subset
rank 0 would have read alone; LPT partition is balanced and deterministic. The per-rank decode is
a numpy stand-in here (the GPU decode itself is covered by the -m gpu parity tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zarrs_amd.distributed import (gather_slabs, lpt_partition, retrieve_array_subset_distributed,
                                   slab_partition)


class FakeArray:
    """retrieve_array_subset_into over an in-memory reference array (decode stand-in)."""
    def __init__(self, a):
        self.a = a
        self.dtype = a.dtype

    def retrieve_array_subset_into(self, start, shape, out):
        sl = tuple(slice(s, s + n) for s, n in zip(start, shape))
        out.copy_(torch.from_numpy(np.ascontiguousarray(self.a[sl])))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = (np.arange(37 * 11 * 5, dtype=np.float32) * 1.5).reshape(37, 11, 5)
        arr = FakeArray(a)
        res = {}
        for name, (start, shape) in {"even": ([2, 1, 0], [20, 9, 5]), "ragged": ([3, 0, 1], [31, 11, 3]),
                                     "tiny": ([5, 5, 2], [1, 2, 2])}.items():
            got = retrieve_array_subset_distributed(arr, start, shape, device="cpu")
            if rank == 0:
                sl = tuple(slice(s, s + n) for s, n in zip(start, shape))
                res[name] = bool(np.array_equal(got.numpy(), a[sl]))
            else:
                res[name] = got is None
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_slab_partition_covers_subset():
    for ext, world in ((768, 8), (10, 3), (2, 4)):
        slabs = slab_partition([200, 5, 7], [ext, 3, 4], world)
        assert sum(sh[0] for _, sh in slabs) == ext
        assert slabs[0][0][0] == 200
        for (s0, sh0), (s1, _) in zip(slabs, slabs[1:]):
            assert s0[0] + sh0[0] == s1[0]
        assert max(sh[0] for _, sh in slabs) - min(sh[0] for _, sh in slabs) <= 1


def test_lpt_partition_balanced_and_deterministic():
    rng = np.random.default_rng(0)
    costs = rng.integers(1000, 100000, size=500).tolist()
    parts = lpt_partition(costs, 8)
    assert sorted(i for p in parts for i in p) == list(range(500))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)
    assert parts == lpt_partition(costs, 8)


def test_gather_single_rank_passthrough():
    t = torch.arange(6).reshape(2, 3)
    assert gather_slabs(t, slab_partition([0, 0], [2, 3], 1)) is t


def test_two_rank_gloo_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[0].values()), out
    assert all(out[1].values()), out
