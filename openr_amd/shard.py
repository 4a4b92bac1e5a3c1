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
    """All-gather per-rank [n_r, V] distance and [n_r, V, B] next-hop shards (uneven
    shards allowed); returns the full [n_units, ...] tensors (or None for a None shard)."""
    gb = GatherBuffers(dist_shard, nh_shard, n_units, world)
    gb.allgather()
    return (gb.full_dist() if dist_shard is not None else None,
            gb.full_nh() if nh_shard is not None else None)


class GatherBuffers:
    """Preallocated all-gather of per-rank result shards (the config-3 exchange step).

    ``dist_shard`` [n_r, V] / ``nh_shard`` [n_r, V, B] are this rank's rows (device
    tensors for RCCL, host tensors for gloo). ``allgather()`` fills ``full`` buffers of
    [world * max_shard, ...] with one ``all_gather_into_tensor`` per array; shards
    smaller than the largest are staged through a padded send buffer. Rows of rank r
    sit at [r * max_shard, r * max_shard + n_r).
    """

    def __init__(self, dist_shard, nh_shard, n_units: int, world: int) -> None:
        import torch

        self.sizes = shard_sizes(n_units, world)
        self.m = max(self.sizes) if self.sizes else 0
        self.world = world
        self.parts = []
        for t in (dist_shard, nh_shard):
            if t is None:
                self.parts.append(None)
                continue
            tail = tuple(t.shape[1:])
            send = t if t.shape[0] == self.m and t.is_contiguous() else torch.zeros((self.m,) + tail, dtype=t.dtype,
                                                                                    device=t.device)
            full = torch.empty((world * self.m,) + tail, dtype=t.dtype, device=t.device)
            self.parts.append((t, send, full))

    def allgather(self) -> None:
        import torch.distributed as dist

        for p in self.parts:
            if p is None:
                continue
            src, send, full = p
            if send is not src:
                send[: src.shape[0]].copy_(src)
            dist.all_gather_into_tensor(full, send)

    def _rows(self, i):
        import torch

        full = self.parts[i][2]
        return torch.cat([full[r * self.m: r * self.m + self.sizes[r]] for r in range(self.world)], dim=0)

    def full_dist(self):
        return self._rows(0)

    def full_nh(self):
        return self._rows(1)


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
