"""Instance sharding across the GPUs of one node.

MPC instances never interact, so the data path has no collective: rank g owns the contiguous
instance range [g*B/G, (g+1)*B/G) and runs the whole RTI iteration on it.  The only collectives
are control-plane ones: the packed SDF weights broadcast once at start-up, the max-over-ranks step
time, and (for a controller that serves all instances from rank 0) a gather of the u_0 rows.
Works with any torch.distributed backend: "nccl" (= RCCL over xGMI on ROCm) on the GPU box,
"gloo" for the CPU tests.
"""
from __future__ import annotations


def instance_range(total: int, world: int, rank: int):
    """Contiguous, balanced [lo, hi) of `total` instances for `rank` of `world` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def plan(total: int, capacity: int, n_devices: int):
    """The north_star's occupancy gate: shard the batch over more GPUs only when it exceeds what the GPUs
    in use already run concurrently -- G = min(n_devices, ceil(total / capacity)) devices, each with a
    contiguous instance_range.  `capacity` = instances one GPU solves in one wave of QP workgroups, from
    the library and the device (sdfnmpc_qp_capacity, _lib.Context.qp_capacity).
    Returns [(device_slot, lo, hi)]."""
    if n_devices < 1:
        raise ValueError("no device to plan on")
    if capacity < 1:
        raise ValueError("the QP does not fit one GPU at this horizon (capacity 0)")
    G = max(1, min(n_devices, -(-total // capacity)))
    return [(g,) + instance_range(total, G, g) for g in range(G)]


def broadcast_blob(blob, device, src=0):
    """bytes on `src` -> the same bytes on every rank (two broadcasts: length, payload)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    if dist.get_backend() == "gloo":  # gloo broadcasts host tensors
        device = "cpu"
    n = torch.tensor([len(blob) if rank == src else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device))
    dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def gather_rows(t, total: int, dst=0):
    """Concatenate every rank's [rows_g, ...] shard (instance_range layout) on `dst`; None elsewhere."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    rows = max(instance_range(total, world, r)[1] - instance_range(total, world, r)[0] for r in range(world))
    pad = torch.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    if dist.get_backend() == "gloo":
        dist.gather(pad, parts, dst=dst)
    else:  # RCCL has no gather: all_gather and keep dst's copy
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
    if rank != dst:
        return None
    return torch.cat([parts[r][: instance_range(total, world, r)[1] - instance_range(total, world, r)[0]]
                      for r in range(world)])


def max_over_ranks(seconds: float, device) -> float:
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "gloo":  # gloo reduces host tensors
        device = "cpu"
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
