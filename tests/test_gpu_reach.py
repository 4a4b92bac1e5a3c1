"""GPU parity of the all-sources level passes (spf_allsrc.hip: msbfs_kernel — bit-parallel
multi-source BFS — and bfs_reach_kernel, each followed by nh_from_levels_kernel), the
all-sources path on graphs whose rows hold <= 4 edges (G100, BASELINE config 3).

The passes solve levels only and derive every next-hop set from the level rows of the
source's neighbours (closed form of LinkState::runSpf for uniform cost,
/root/reference/openr/decision/LinkState.cpp:808-882). These tests check every row of
whole batches against the oracle on the graphs where that derivation has corner cases:
overloaded nodes (sinks, next hop of themselves only), down links, parallel links,
disconnected parts, non-unit uniform cost, hop count on weighted graphs, and the
fallbacks — solves deeper than 253 levels or wider than a queue half, and sources whose
neighbour rows are missing from the batch — which the u16 full-order pass re-runs.
openr_spf_last_kernels proves which kernels ran.
"""
import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.engine import SpfEngine
from oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = SpfEngine()
    yield e
    e.close()


PASS_KERNEL = {"wreach": "bfs_wreach_kernel", "msbfs": "msbfs_tile_kernel", "msbfs_dense": "msbfs_kernel",
               "reach": "bfs_reach_kernel"}


@pytest.fixture(autouse=True, params=["wreach", "msbfs", "msbfs_dense", "reach"])
def level_pass(request, monkeypatch):
    """Every test runs on every level pass (forced: also on batches smaller than V): the
    wave-reach pass (one wavefront per source, graph in LDS; partial batches extended with
    halo rows), the tile-active multi-source BFS, the dense-pull one and the per-source
    reach pass."""
    monkeypatch.setenv("OPENR_SPF_BFS_FAMILY", "lvl")
    monkeypatch.setenv("OPENR_SPF_BFS_WREACH", "1" if request.param == "wreach" else "0")
    monkeypatch.setenv("OPENR_SPF_BFS_MSBFS", "0" if request.param in ("reach", "wreach") else "1")
    monkeypatch.setenv("OPENR_SPF_MSBFS_TILE", "0" if request.param == "msbfs_dense" else "1")
    monkeypatch.setenv("OPENR_SPF_BFS_REACH", "1")
    return request.param


def grid_links(n):
    links = [(r * n + c, r * n + c + 1) for r in range(n) for c in range(n - 1)]
    links += [(r * n + c, (r + 1) * n + c) for r in range(n - 1) for c in range(n)]
    return links


def check_batch(eng, g, sources, use_metric=True, nh_bytes=None, kernel=None):
    eng.set_graph(g)
    o = Oracle(g)
    src = np.asarray(sources, dtype=np.uint32)
    dist, nh, _ = eng.solve(src, use_metric, nh_bytes=nh_bytes)
    ran = eng.last_kernels()
    if kernel:
        assert kernel in ran, ran
    odist, onh = o.all_sources(src, use_metric, nthreads=16)
    bad = np.nonzero(np.any(dist != odist, axis=1))[0]
    assert bad.size == 0, f"dist differs for sources {src[bad[:8]].tolist()} ({ran})"
    nb = o.nh_bytes
    bad = np.nonzero(np.any(nh[:, :, :nb] != onh, axis=(1, 2)))[0]
    assert bad.size == 0, f"next hops differ for sources {src[bad[:8]].tolist()} ({ran})"
    if nh.shape[2] > nb:
        assert not nh[:, :, nb:].any(), "bytes past the next-hop set must be zero"
    return dist, nh, ran


@pytest.mark.parametrize("dist_phase", ["1", "2"])
def test_grid_all_sources(eng, monkeypatch, dist_phase, level_pass):
    """A 40 x 40 grid, all sources in one batch; distance rows written by phase 1 (default)
    or by the streaming next-hop pass (OPENR_SPF_REACH_DIST=2)."""
    monkeypatch.setenv("OPENR_SPF_REACH_DIST", dist_phase)
    n = 40
    g = T.grid_fast(n)
    _, _, ran = check_batch(eng, g, range(n * n), kernel=PASS_KERNEL[level_pass])
    assert "nh_from_levels_kernel" in ran


def test_grid_overloads_down_links_parallel_links(eng, level_pass):
    """Overloaded nodes (incl. sources' neighbours and sources themselves), 5 % down
    links and parallel links (rows of <= 4 edges): every row of the all-sources batch."""
    n = 36
    rng = np.random.default_rng(7)
    names = [f"g{r:02d}-{c:02d}" for r in range(n) for c in range(n)]
    links = grid_links(n)
    # parallel links along the first column (degree stays <= 4: column nodes lose no edge
    # but get a second link to the node below only where they have no left neighbour)
    links += [(r * n, (r + 1) * n) for r in range(0, n - 1, 3)]
    ovl = (rng.random(n * n) < 0.06).astype(np.uint8)
    up = (rng.random(len(links)) > 0.05).astype(np.uint8)
    g = T.csr_from_links(names, np.array(links), overloaded=ovl, link_up=up)
    assert max(np.diff(g.row_ptr)) <= 4
    check_batch(eng, g, range(n * n), kernel=PASS_KERNEL[level_pass])


def test_disconnected_parts_and_isolated_nodes(eng):
    """Two grids with no link between them plus nodes whose every link is down: unreached
    nodes keep UINT64_MAX and empty sets, isolated sources reach only themselves."""
    n = 20
    names = [f"a{i:03d}" for i in range(n * n)] + [f"b{i:03d}" for i in range(n * n)] + ["x0", "x1"]
    links = grid_links(n) + [(n * n + a, n * n + b) for a, b in grid_links(n)] + [(2 * n * n, 2 * n * n + 1)]
    up = np.ones(len(links), dtype=np.uint8)
    up[-1] = 0
    g = T.csr_from_links(names, np.array(links), link_up=up)
    check_batch(eng, g, range(g.num_nodes))


def test_uniform_non_unit_cost_and_hop_count(eng):
    """Every metric 7 (dist = 7 x level), and a random-metric graph of degree <= 4 solved
    with useLinkMetric=false (hop count: uniform cost 1 on a weighted graph)."""
    n = 24
    links = np.array(grid_links(n))
    names = [str(i) for i in range(n * n)]
    g = T.csr_from_links(names, links, metric_uv=np.full(len(links), 7), metric_vu=np.full(len(links), 7))
    dist, _, _ = check_batch(eng, g, range(n * n))
    assert int(dist[0, n * n - 1]) == 7 * 2 * (n - 1)
    rng = np.random.default_rng(3)
    g2 = T.csr_from_links(names, links, metric_uv=rng.integers(1, 64, len(links)),
                          metric_vu=rng.integers(1, 64, len(links)))
    check_batch(eng, g2, range(n * n), use_metric=False)


def test_depth_overflow_rerun(eng):
    """A 30 x 30 grid plus a 300-node chain: chain sources run deeper than 253 levels, are
    flagged by the reach pass and re-run by the u16 full-order pass — and so are the
    sources whose neighbour rows were flagged (their next hops need those rows)."""
    n, tail = 30, 300
    names = [f"g{i:03d}" for i in range(n * n)] + [f"z{i:03d}" for i in range(tail)]
    links = grid_links(n) + [(n * n + i, n * n + i + 1) for i in range(tail - 1)] + [(n * n - 1, n * n)]
    g = T.csr_from_links(names, np.array(links))
    dist, _, ran = check_batch(eng, g, range(g.num_nodes))
    assert "bfs_lvl_kernel<full,u16>:rerun" in ran, ran
    assert int(dist[0, g.num_nodes - 1]) == 2 * (n - 1) + tail


def test_queue_half_overflow_rerun(eng, monkeypatch, level_pass):
    """A forced 16-entry queue half (reach pass): wide levels overflow it, those solves and
    their neighbours' next-hop rows go to the re-run."""
    if level_pass not in ("reach", "wreach"):
        pytest.skip("the per-source passes' queues")
    monkeypatch.setenv("OPENR_SPF_REACH_QHALF", "16")
    g = T.grid_fast(24)
    check_batch(eng, g, range(g.num_nodes))


def test_partial_batches_missing_neighbours(eng, monkeypatch, level_pass):
    """Forced onto batches that do not hold every neighbour (a strong-scaling shard, a
    strided sample, duplicates, sources in random order): sources with a missing
    neighbour row are re-run, the others use the derivation."""
    monkeypatch.setenv("OPENR_SPF_BFS_REACH", "1")
    g = T.grid_fast(30)
    V = g.num_nodes
    check_batch(eng, g, range(100, 250), kernel=PASS_KERNEL[level_pass])
    check_batch(eng, g, range(0, V, 3))
    rng = np.random.default_rng(1)
    perm = rng.permutation(V)
    check_batch(eng, g, np.concatenate([perm, perm[:50]]))


def test_wider_nh_stride_zero_padded(eng):
    """A caller stride of 3 next-hop bytes per node: byte 0 holds the set, the rest are zero."""
    g = T.grid_fast(16)
    check_batch(eng, g, range(g.num_nodes), nh_bytes=3)


def test_grid100_full_batch(eng, monkeypatch, level_pass):
    """All 10 000 G100 sources in one call with the pass in auto mode run it; a sample of
    rows vs the oracle (test_gpu_configs.py checks every row)."""
    if level_pass == "reach":
        pytest.skip("the reach pass has no auto mode for full batches")
    monkeypatch.setenv("OPENR_SPF_BFS_WREACH", "2" if level_pass == "wreach" else "0")
    monkeypatch.setenv("OPENR_SPF_BFS_MSBFS", "0" if level_pass == "wreach" else "2")
    monkeypatch.delenv("OPENR_SPF_BFS_REACH")
    g = T.grid_fast(100)
    eng.set_graph(g)
    src = np.arange(10000, dtype=np.uint32)
    dist, nh, _ = eng.solve(src, True)
    ran = eng.last_kernels()
    assert PASS_KERNEL[level_pass] in ran and "nh_from_levels_kernel" in ran, ran
    o = Oracle(g)
    pick = np.array([0, 99, 4950, 5050, 9900, 9999, 1234, 7777], dtype=np.uint32)
    od, on = o.all_sources(pick, True, nthreads=8)
    np.testing.assert_array_equal(dist[pick], od)
    np.testing.assert_array_equal(nh[pick], on)
