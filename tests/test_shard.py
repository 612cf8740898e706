"""Multi-rank control plane of the sharded RTI (sdf-nmpc_amd/shard.py) with world_size 2 over gloo
on the CPU: instance ranges cover the batch exactly once, the weight blob broadcast is byte-exact,
u_0 rows gather back in instance order, and the step time is the max over ranks."""
import hashlib
import os
import socket

import numpy as np
import pytest

from sdf_nmpc_amd.shard import instance_range, plan


@pytest.mark.parametrize("total,world", [(1024, 1), (1024, 8), (8192, 8), (1000, 3), (5, 8), (0, 2)])
def test_instance_ranges_partition(total, world):
    seen = np.zeros(total, int)
    sizes = []
    for r in range(world):
        lo, hi = instance_range(total, world, r)
        seen[lo:hi] += 1
        sizes.append(hi - lo)
    assert (seen == 1).all() and max(sizes) - min(sizes) <= 1


def test_plan_occupancy_gate():
    """shard.plan: G = min(devices, ceil(total / capacity)) contiguous parts; capacity 0 is refused."""
    assert plan(1024, 1024, 8) == [(0, 0, 1024)]
    assert plan(1025, 1024, 8) == [(0, 0, 513), (1, 513, 1025)]
    assert [p[0] for p in plan(8192, 1024, 8)] == list(range(8))
    assert len(plan(100000, 1024, 4)) == 4
    with pytest.raises(ValueError):
        plan(10, 0, 2)
    with pytest.raises(ValueError):
        plan(10, 1024, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sdf_nmpc_amd import shard, weights as W
    dev = torch.device("cpu")
    blob = W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=3)) if rank == 0 else None
    got = shard.broadcast_blob(blob, dev)
    lo, hi = shard.instance_range(total, world, rank)
    u0 = torch.arange(lo * 4, hi * 4, dtype=torch.float64).reshape(-1, 4)  # row i holds instance i
    full = shard.gather_rows(u0, total)
    t = shard.max_over_ranks(0.5 + rank, dev)
    q.put((rank, len(got), hashlib.sha256(got).hexdigest(), None if full is None else full.numpy(), t))
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [10, 7])
def test_two_rank_control_plane(total):
    import torch.multiprocessing as mp
    from sdf_nmpc_amd import weights as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blob = W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=3))
    for rank, n, h, full, t in res:
        assert n == len(blob) and h == hashlib.sha256(blob).hexdigest() and t == 1.5
        if rank == 0:
            np.testing.assert_array_equal(full, np.arange(total * 4, dtype=float).reshape(-1, 4))
        else:
            assert full is None
