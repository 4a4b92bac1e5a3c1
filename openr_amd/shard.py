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


class CompactGather:
    """The config-3 exchange in level form: on a uniform-cost graph (every
    usable edge costs ``cost``, or useLinkMetric=false) every finite distance of
    LinkState::runSpf is level x cost, so a rank sends its rows as levels — u8 when every
    finite level is <= 254, else u16 (all ones = unreached, i.e. UINT64_MAX) — plus its
    next-hop rows, instead of u64 distances: 1 + B instead of 8 + B bytes per (source,
    node). Receivers keep the gathered level rows and expand u64 distances on demand
    (``full_dist``), bit-identical to the senders' rows.

    ``dist_shard`` [n_r, V] int64 (UINT64_MAX viewed as -1) and ``nh_shard`` [n_r, V, B]
    are this rank's engine rows (device tensors for RCCL, host tensors for gloo);
    ``max_level`` bounds every finite level of the whole job (e.g. the largest finite
    distance / cost, measured once outside any timed region).
    """

    def __init__(self, dist_shard, nh_shard, n_units: int, world: int, cost: int, max_level: int) -> None:
        import torch

        if cost < 1:
            raise ValueError("cost must be >= 1")
        if max_level > 65534:
            raise ValueError("levels do not fit u16: use GatherBuffers")
        self.cost = int(cost)
        self.dtype = torch.uint8 if max_level <= 254 else torch.int16  # int16 holds u16 bit patterns
        self.sentinel = 0xFF if self.dtype == torch.uint8 else -1  # all ones
        self.dist_shard = dist_shard
        self.sizes = shard_sizes(n_units, world)
        self.m = max(self.sizes) if self.sizes else 0
        self.world = world
        V = dist_shard.shape[1]
        dev = dist_shard.device
        self.lv_send = torch.zeros((self.m, V), dtype=self.dtype, device=dev)
        self.lv_full = torch.empty((world * self.m, V), dtype=self.dtype, device=dev)
        self.nh = None
        if nh_shard is not None:
            tail = tuple(nh_shard.shape[1:])
            send = nh_shard if nh_shard.shape[0] == self.m and nh_shard.is_contiguous() else torch.zeros(
                (self.m,) + tail, dtype=nh_shard.dtype, device=dev)
            self.nh = (nh_shard, send, torch.empty((world * self.m,) + tail, dtype=nh_shard.dtype, device=dev))
        nb = 0
        if nh_shard is not None:
            nb = nh_shard.element_size()
            for x in nh_shard.shape[2:]:
                nb *= int(x)
        self.bytes_per_rank = self.m * V * (self.lv_send.element_size() + nb)

    @classmethod
    def native(cls, nh_shard, n_units: int, world: int, cost: int, max_level: int, V: int, device):
        """The fused form: the solve writes this rank's level rows itself
        (openr_spf_solve_device with OPENR_SPF_EMIT_LEVELS8 / 16 into ``level_send``), so
        the exchange reads no u64 rows and there is no encode pass. ``level_bytes`` is the
        flag the solve needs; ``level_send`` [m, V] (m = the largest shard) is its output
        buffer (rows past this rank's shard stay zero)."""
        import torch

        obj = cls.__new__(cls)
        if cost < 1:
            raise ValueError("cost must be >= 1")
        if max_level > 65534:
            raise ValueError("levels do not fit u16: use GatherBuffers")
        obj.cost = int(cost)
        obj.dtype = torch.uint8 if max_level <= 254 else torch.int16
        obj.sentinel = 0xFF if obj.dtype == torch.uint8 else -1
        obj.level_bytes = 1 if obj.dtype == torch.uint8 else 2
        obj.dist_shard = None
        obj.sizes = shard_sizes(n_units, world)
        obj.m = max(obj.sizes) if obj.sizes else 0
        obj.world = world
        obj.lv_send = torch.zeros((obj.m, V), dtype=obj.dtype, device=device)
        obj.level_send = obj.lv_send
        obj.lv_full = torch.empty((world * obj.m, V), dtype=obj.dtype, device=device)
        obj.nh = None
        nb = 0
        if nh_shard is not None:
            tail = tuple(nh_shard.shape[1:])
            send = nh_shard if nh_shard.shape[0] == obj.m and nh_shard.is_contiguous() else torch.zeros(
                (obj.m,) + tail, dtype=nh_shard.dtype, device=device)
            obj.nh = (nh_shard, send, torch.empty((world * obj.m,) + tail, dtype=nh_shard.dtype, device=device))
            nb = nh_shard.element_size()
            for x in nh_shard.shape[2:]:
                nb *= int(x)
        obj.bytes_per_rank = obj.m * V * (obj.lv_send.element_size() + nb)
        return obj

    def encode(self) -> None:
        """This rank's u64 rows -> level rows (on the rows' device); nothing to do in the
        native form (the solve wrote them)."""
        import torch

        d = self.dist_shard
        if d is None:
            return
        n = d.shape[0]
        if n == 0:
            return
        lv = torch.div(d, self.cost, rounding_mode="floor")
        lv = torch.where(d == -1, torch.full_like(lv, self.sentinel), lv)
        self.lv_send[:n].copy_(lv.to(self.dtype))

    def allgather(self) -> None:
        import torch
        import torch.distributed as dist

        self.encode()
        # byte views: u16 level rows travel as bytes (gloo has no 16-bit integer type)
        dist.all_gather_into_tensor(self.lv_full.view(torch.uint8), self.lv_send.view(torch.uint8))
        if self.nh is not None:
            src, send, full = self.nh
            if send is not src:
                send[: src.shape[0]].copy_(src)
            dist.all_gather_into_tensor(full, send)

    def _rows(self, full):
        import torch

        return torch.cat([full[r * self.m: r * self.m + self.sizes[r]] for r in range(self.world)], dim=0)

    def full_levels(self):
        return self._rows(self.lv_full)

    def full_dist(self):
        """The gathered rows expanded to u64 distances (int64 view, UINT64_MAX = -1)."""
        import torch

        lv = self.full_levels()
        unreached = lv == self.sentinel
        d = lv.to(torch.int64)
        if self.dtype != torch.uint8:
            d = d & 0xFFFF
        d = d * self.cost
        return torch.where(unreached, torch.full_like(d, -1), d)

    def full_nh(self):
        return self._rows(self.nh[2]) if self.nh is not None else None


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
