"""The config-3 exchange over RCCL on device tensors (the leg bench.py runs
for N > 1 had never executed). One rank, world size 1 — the 1-GPU box cannot host two
RCCL ranks on one device — with torch.distributed's "nccl" backend (RCCL on ROCm), the
G100 shard of one 8-GPU rank (1 250 sources), and the device-resident buffers bench.py
uses: GatherBuffers (u64 rows), CompactGather with the device-side encode of u64 rows,
and the fused form whose solve writes the u8 level rows itself
(OPENR_SPF_EMIT_LEVELS8). Every gathered row is compared with the oracle, bit for bit;
the u16 form and the u8 overflow status are checked on a deeper graph.
"""
import os
import socket

import numpy as np
import pytest

from openr_amd import topology as T

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, port, out_dir):
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    from openr_amd.engine import SpfEngine
    from openr_amd.shard import CompactGather, GatherBuffers

    g = T.grid_fast(100)
    V = g.num_nodes
    n = 1250  # one rank's shard of an 8-GPU strong-scaling run
    eng = SpfEngine([0])
    eng.set_graph(g)
    nb = eng.nh_bytes
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    src = torch.arange(0, n, dtype=torch.int32, device=dev)
    d_dist = torch.empty((n, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((n, V, nb), dtype=torch.uint8, device=dev)
    eng.solve_device(src.data_ptr(), n, d_dist.data_ptr(), d_nh.data_ptr(), nb, True, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    # u64 rows over RCCL
    gb = GatherBuffers(d_dist, d_nh, n, 1)
    gb.allgather()
    torch.cuda.synchronize(dev)
    np.save(os.path.join(out_dir, "full_dist.npy"), gb.full_dist().cpu().numpy())
    np.save(os.path.join(out_dir, "full_nh.npy"), gb.full_nh().cpu().numpy())
    # compact rows, encoded on the device from the u64 rows
    cg = CompactGather(d_dist, d_nh, n, 1, cost=1, max_level=198)
    cg.allgather()
    torch.cuda.synchronize(dev)
    np.save(os.path.join(out_dir, "enc_dist.npy"), cg.full_dist().cpu().numpy())
    np.save(os.path.join(out_dir, "enc_nh.npy"), cg.full_nh().cpu().numpy())
    # fused: the solve writes the u8 level rows (no u64 rows at all)
    d_nh2 = torch.zeros((n, V, nb), dtype=torch.uint8, device=dev)
    fg = CompactGather.native(d_nh2, n, 1, cost=1, max_level=198, V=V, device=dev)
    assert fg.level_bytes == 1
    eng.solve_device(src.data_ptr(), n, fg.level_send.data_ptr(), d_nh2.data_ptr(), nb, True,
                     stream=stream.cuda_stream, level_bytes=fg.level_bytes)
    fg.allgather()
    torch.cuda.synchronize(dev)
    assert eng.take_status() == 0
    np.save(os.path.join(out_dir, "fused_levels.npy"), fg.full_levels().cpu().numpy())
    np.save(os.path.join(out_dir, "fused_dist.npy"), fg.full_dist().cpu().numpy())
    np.save(os.path.join(out_dir, "fused_nh.npy"), fg.full_nh().cpu().numpy())
    eng.close()
    dist.destroy_process_group()


def test_rccl_world1_g100_shard(tmp_path):
    import torch.multiprocessing as mp

    from oracle import Oracle

    mp.start_processes(_rank_main, args=(_free_port(), str(tmp_path)), nprocs=1, join=True, start_method="spawn")
    g = T.grid_fast(100)
    d, nh = Oracle(g).all_sources(np.arange(1250, dtype=np.uint32), True, nthreads=8)
    for tag in ("full", "enc", "fused"):
        np.testing.assert_array_equal(np.load(tmp_path / f"{tag}_dist.npy").view(np.uint64), d, err_msg=tag)
        np.testing.assert_array_equal(np.load(tmp_path / f"{tag}_nh.npy"), nh, err_msg=tag)
    lv = np.load(tmp_path / "fused_levels.npy")
    exp = np.where(d == np.uint64(2**64 - 1), 0xFF, d).astype(np.uint8)
    np.testing.assert_array_equal(lv, exp)


@pytest.mark.parametrize("wave", ["0", "1"])
def test_level_rows_u8_u16_and_overflow(monkeypatch, wave):
    """EMIT_LEVELS8 / 16 on a graph with levels past 254 (a 300-node chain hanging off a
    grid): u16 rows hold every level, u8 rows hold 0xFE past 254 and raise
    OPENR_SPF_STATUS_LEVEL_OVERFLOW; both on the lean and on the wave pass (and their u16
    re-run), against the oracle."""
    import torch

    from openr_amd.engine import STATUS_LEVEL_OVERFLOW, SpfEngine, SpfError
    from oracle import Oracle

    monkeypatch.setenv("OPENR_SPF_BFS_WAVE", wave)
    monkeypatch.setenv("OPENR_SPF_BFS_FAMILY", "lvl")
    n, tail = 20, 300
    names = [f"g{r:02d}-{c:02d}" for r in range(n) for c in range(n)] + [f"z{i:03d}" for i in range(tail)]
    links = [(r * n + c, r * n + c + 1) for r in range(n) for c in range(n - 1)]
    links += [(r * n + c, (r + 1) * n + c) for r in range(n - 1) for c in range(n)]
    links += [(n * n - 1, n * n)] + [(n * n + i, n * n + i + 1) for i in range(tail - 1)]
    g = T.csr_from_links(names, np.array(links))
    V = g.num_nodes
    srcs = np.array([0, 7, n * n - 1, n * n + 5, V - 1] + list(range(0, n * n, 13)), dtype=np.uint32)
    od, onh = Oracle(g).all_sources(srcs, True)
    eng = SpfEngine([0])
    try:
        eng.set_graph(g)
        nb = eng.nh_bytes
        dev = torch.device("cuda", 0)
        s = torch.from_numpy(srcs.astype(np.int32)).to(dev)
        unreached = od == np.uint64(2**64 - 1)
        for lb, dt in ((2, torch.int16), (1, torch.uint8)):
            rows = torch.zeros((len(srcs), V), dtype=dt, device=dev)
            nh = torch.zeros((len(srcs), V, nb), dtype=torch.uint8, device=dev)
            eng.solve_device(s.data_ptr(), len(srcs), rows.data_ptr(), nh.data_ptr(), nb, True, level_bytes=lb)
            st = eng.take_status()
            got = rows.cpu().numpy()
            np.testing.assert_array_equal(nh.cpu().numpy(), onh)
            if lb == 2:
                exp = np.where(unreached, 0xFFFF, od).astype(np.uint16)
                np.testing.assert_array_equal(got.view(np.uint16), exp)
                assert st == 0
            else:
                exp = np.where(unreached, 0xFF, np.minimum(od, 0xFE)).astype(np.uint8)
                np.testing.assert_array_equal(got, exp)
                assert st == STATUS_LEVEL_OVERFLOW  # the chain's far end lies past level 254
        # level rows need the level family: an ignore set is refused
        with pytest.raises(SpfError):
            rows = torch.zeros((1, V), dtype=torch.uint8, device=dev)
            ip = torch.tensor([0, 1], dtype=torch.int32, device=dev)
            il = torch.tensor([0], dtype=torch.int32, device=dev)
            eng.solve_device(s.data_ptr(), 1, rows.data_ptr(), 0, nb, True, d_ignore_ptr=ip.data_ptr(),
                             d_ignore_links=il.data_ptr(), level_bytes=1)
    finally:
        eng.close()
