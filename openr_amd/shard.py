"""Source sharding across ranks (one process per GPU) and the result all-gather.

Units (sources, (link, source) what-if pairs, (src, dst) KSP2 pairs) are
independent, so each rank holds a full CSR replica and solves a contiguous block
of units with no collective during compute. The only exchange is
the optional all-gather of the dense result shards over RCCL (torch.distributed
"nccl" backend = RCCL on ROCm).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n_units: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced block [lo, hi) of n_units for `rank` of `world`."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(n_units, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def shard_sizes(n_units: int, world: int):
    return [shard_range(n_units, r, world)[1] - shard_range(n_units, r, world)[0] for r in range(world)]


def allgather_results(dist_shard, nh_shard, n_units: int, world: int):
    """All-gather per-rank [n_r, V] distance and [n_r, V, B] next-hop shards.

    Shards may be uneven (n_units % world != 0); each is padded to the largest
    shard for the collective and trimmed afterwards. Returns full tensors.
    """
    import torch
    import torch.distributed as dist

    sizes = shard_sizes(n_units, world)
    m = max(sizes)
    outs = []
    for t in (dist_shard, nh_shard):
        if t is None:
            outs.append(None)
            continue
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        full = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(full, pad)
        parts = [full[r * m : r * m + sizes[r]] for r in range(world)]
        outs.append(torch.cat(parts, dim=0))
    return outs[0], outs[1]


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a host scalar over all ranks (bench timing: the slowest rank's clock);
    the identity without an initialised process group."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
