"""The engine in more than one rank, and in one context over a multi-entry device list.

Config 3 (G100 all-pairs sharded by source across GPUs + all-gather) and config 5 (KSP2
all pairs across GPUs) run one process per GPU, each holding a CSR replica and solving a
contiguous block of units (shard.py), with the result shards all-gathered. The 1-GPU
box cannot host two RCCL ranks on one device, so here both ranks put the ENGINE on
cuda:0 and exchange their shards over gloo (host tensors); the per-rank code path —
shard_range, SpfEngine.solve / ksp2 on the rank's block, GatherBuffers and the compact
level-row CompactGather — is the one bench.py runs over RCCL. The gathered rows must equal the oracle's, bit for bit.
"""
import os
import socket

import numpy as np
import pytest

from openr_amd import shard
from openr_amd import topology as T

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph(name):
    return {"grid40": lambda: T.grid_fast(40), "fabric": lambda: T.fabric(288 + 2 * 56)}[name]()


def _rank_main(rank, world, port, gname, out_dir):
    import torch
    import torch.distributed as dist

    torch.cuda.init()  # torch's HIP runtime first (see tests/conftest.py)
    from openr_amd.engine import SpfEngine

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = _graph(gname)
    V = g.num_nodes
    eng = SpfEngine([0])
    eng.set_graph(g)
    lo, hi = shard.shard_range(V, rank, world)
    d, nh, _ = eng.solve(np.arange(lo, hi, dtype=np.uint32), True)
    d_t, nh_t = torch.from_numpy(d.view(np.int64).copy()), torch.from_numpy(nh.copy())
    full_d, full_nh = shard.allgather_results(d_t, nh_t, V, world)
    # the compact exchange bench.py runs by default (u8 level rows + next hops; unit metrics)
    cg = shard.CompactGather(d_t, nh_t, V, world, cost=1, max_level=254)
    cg.allgather()
    # KSP2 pairs sharded the same way (config 5): this rank's sources x a destination sample
    ks = np.arange(lo, hi, max(1, (hi - lo) // 5), dtype=np.uint32)
    dst = np.arange(0, V, 7, dtype=np.uint32)
    t1, t2 = eng.ksp2_tokens(np.repeat(ks, len(dst)), np.tile(dst, len(ks)), 256)
    np.save(os.path.join(out_dir, f"ksp_src_{rank}.npy"), ks)
    np.save(os.path.join(out_dir, f"ksp_t1_{rank}.npy"), t1)
    np.save(os.path.join(out_dir, f"ksp_t2_{rank}.npy"), t2)
    if rank == 0:
        np.save(os.path.join(out_dir, "dist.npy"), full_d.numpy())
        np.save(os.path.join(out_dir, "nh.npy"), full_nh.numpy())
        np.save(os.path.join(out_dir, "cdist.npy"), cg.full_dist().numpy())
        np.save(os.path.join(out_dir, "cnh.npy"), cg.full_nh().numpy())
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("gname,world", [("grid40", 2), ("fabric", 2), ("grid40", 3)])
def test_engine_ranks_shard_and_allgather(tmp_path, gname, world):
    import torch.multiprocessing as mp

    from openr_amd.engine import decode_paths
    from oracle import Oracle

    mp.start_processes(_rank_main, args=(world, _free_port(), gname, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    g = _graph(gname)
    V = g.num_nodes
    o = Oracle(g)
    d, nh = o.all_sources(np.arange(V, dtype=np.uint32), True, nthreads=8)
    np.testing.assert_array_equal(np.load(tmp_path / "dist.npy").view(np.uint64), d)
    np.testing.assert_array_equal(np.load(tmp_path / "nh.npy"), nh)
    np.testing.assert_array_equal(np.load(tmp_path / "cdist.npy").view(np.uint64), d)
    np.testing.assert_array_equal(np.load(tmp_path / "cnh.npy"), nh)
    dst = np.arange(0, V, 7, dtype=np.uint32)
    for r in range(world):
        ks = np.load(tmp_path / f"ksp_src_{r}.npy")
        t1, t2 = np.load(tmp_path / f"ksp_t1_{r}.npy"), np.load(tmp_path / f"ksp_t2_{r}.npy")
        o1, o2 = o.ksp2_tokens(np.repeat(ks, len(dst)), np.tile(dst, len(ks)), 256)
        for i in range(len(t1)):
            assert decode_paths(t1[i]) == decode_paths(o1[i]) and decode_paths(t2[i]) == decode_paths(o2[i]), (r, i)


def test_context_over_repeated_device_list():
    """openr_spf_create with two device entries (the same ordinal twice on a 1-GPU box):
    the sources of one call are split in blocks across the two device slots
    (spf_capi.hip), each with its own stream and buffers; results equal a single-device
    context's and the oracle's."""
    from openr_amd.engine import SpfEngine
    from oracle import Oracle

    g = T.fabric(288 + 2 * 56)
    one, two = SpfEngine([0]), SpfEngine([0, 0])
    try:
        srcs = np.arange(g.num_nodes, dtype=np.uint32)
        for e in (one, two):
            e.set_graph(g)
        d1, n1, t1 = one.solve(srcs, True, want_tight=True)
        d2, n2, t2 = two.solve(srcs, True, want_tight=True)
        np.testing.assert_array_equal(d1, d2)
        np.testing.assert_array_equal(n1, n2)
        np.testing.assert_array_equal(t1, t2)
        od, onh = Oracle(g).all_sources(srcs, True, nthreads=8)
        np.testing.assert_array_equal(d2, od)
        np.testing.assert_array_equal(n2, onh)
        assert two.stats().spf_runs == len(srcs)
        # ignore sets and the KSP2 batch split across the two slots too
        rng = np.random.default_rng(3)
        ign = [sorted(set(rng.integers(0, g.num_links, 6).tolist())) for _ in range(40)]
        s40 = rng.integers(0, g.num_nodes, 40).tolist()
        a, _, _ = one.solve(s40, True, ignore=ign)
        b, _, _ = two.solve(s40, True, ignore=ign)
        np.testing.assert_array_equal(a, b)
        pairs_s = rng.integers(0, g.num_nodes, 300)
        pairs_d = rng.integers(0, g.num_nodes, 300)
        k1a, k2a = one.ksp2_tokens(pairs_s, pairs_d, 256)
        k1b, k2b = two.ksp2_tokens(pairs_s, pairs_d, 256)
        from openr_amd.engine import decode_paths

        for i in range(300):
            assert decode_paths(k1a[i]) == decode_paths(k1b[i]) and decode_paths(k2a[i]) == decode_paths(k2b[i])
        wl = np.arange(0, g.num_links, 11)
        c1, _ = one.whatif(wl, s40[:8], True)
        c2, _ = two.whatif(wl, s40[:8], True)
        np.testing.assert_array_equal(c1, c2)
    finally:
        one.close()
        two.close()


def _whatif_rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    torch.cuda.init()
    from openr_amd.engine import SpfEngine

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = T.wan(400, 1200, 64, seed=5)
    V, L = g.num_nodes, g.num_links
    eng = SpfEngine([0])
    eng.set_graph(g)
    # config 4's strong split (bench.py whatif_main): rank r takes links shard_range(L, r, N)
    lo, hi = shard.shard_range(L, rank, world)
    srcs = np.arange(0, V, 3, dtype=np.uint32)
    changed, _ = eng.whatif(np.arange(lo, hi, dtype=np.uint32), srcs, True)
    # bench.py's self-check: every rank's rows as a 64-bit digest, all-gathered
    import hashlib

    digest = hashlib.blake2b(changed.tobytes(), digest_size=8).hexdigest()
    t = torch.tensor([int(digest, 16) - (1 << 63)], dtype=torch.int64)
    digs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(digs, t)
    # the rows themselves, gathered to rank 0 (padded to the largest shard)
    sizes = shard.shard_sizes(L, world)
    buf = np.zeros((max(sizes), len(srcs)), dtype=np.int64)
    buf[: hi - lo] = changed
    parts = [torch.zeros(buf.shape, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(buf))
    if rank == 0:
        full = np.concatenate([p.numpy()[:n] for p, n in zip(parts, sizes)]).astype(np.uint32)
        np.save(os.path.join(out_dir, "whatif.npy"), full)
        np.save(os.path.join(out_dir, "digests.npy"), np.array([int(x.item()) for x in digs], dtype=np.int64))
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_engine_ranks_whatif_link_shards(tmp_path, world):
    """Config 4 across ranks: each rank sweeps its block of links (shard_range) for the
    same sources on its own engine; the gathered changed rows equal the oracle's
    re-solves runSpf(src, true, {link}), and each rank's all-gathered digest equals a
    single-rank recomputation of that shard (the check bench.py's what-if line carries)."""
    import hashlib

    import torch.multiprocessing as mp

    from openr_amd.engine import SpfEngine
    from oracle import Oracle

    mp.start_processes(_whatif_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    g = T.wan(400, 1200, 64, seed=5)
    V, L = g.num_nodes, g.num_links
    srcs = np.arange(0, V, 3, dtype=np.uint32)
    full = np.load(tmp_path / "whatif.npy")
    want = Oracle(g).whatif(np.arange(L, dtype=np.uint32), srcs, True)
    np.testing.assert_array_equal(full, want)
    digs = np.load(tmp_path / "digests.npy")
    eng = SpfEngine([0])
    eng.set_graph(g)
    for r in range(world):
        lo, hi = shard.shard_range(L, r, world)
        c, _ = eng.whatif(np.arange(lo, hi, dtype=np.uint32), srcs, True)
        d = hashlib.blake2b(c.tobytes(), digest_size=8).hexdigest()
        assert int(d, 16) - (1 << 63) == int(digs[r]), f"rank {r} digest"
    eng.close()
