"""Full-size HIP-vs-oracle parity on every BASELINE.json config, one test per config.

Each test is named after the config it covers (BASELINE.json "configs")
so config coverage reads directly from the test log:

  config1  G10  (10x10 benchmark grid), all-sources getSpfResult      — every source
  config2  FAB  (intended fabric, 4 992 nodes), all-sources + ECMP    — every source
  config3  G100 (100x100 grid, 10 000 nodes), all-pairs               — every source
  config4  WAN  (1k nodes, 3 000 links, U[1,64]) what-if sweep        — all links x 16 sources
  config5  FAB  KSP2 getKthPaths(k=1,2)                               — every destination of
                                                                         an SSW, FSW and RSW source

The oracle (oracle/spf_oracle.c, LinkState.cpp:762-882 restated) runs on host threads
as the checker; every engine call goes through the C-ABI. The multi-GPU halves of
configs 3 and 5 (source sharding + RCCL all-gather) are covered by
tests/test_gpu_multirank.py.
"""
import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.engine import SpfEngine, decode_paths
from openr_amd.spf_result import tight_in_edges
from oracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = SpfEngine()
    yield e
    e.close()


def all_sources_vs_oracle(eng, g, chunk, use_metric=True, expect_kernel=None, check_chunk=2500):
    """Every source of g: engine dist + next-hop rows == oracle rows. The engine solves
    `chunk` sources per call (one launch, as bench.py does at chunk = V); the rows are
    compared against the oracle `check_chunk` at a time. expect_kernel: the kernel every
    call must have run (openr_spf_last_kernels)."""
    eng.set_graph(g)
    o = Oracle(g)
    assert eng.nh_bytes == o.nh_bytes
    V = g.num_nodes
    for lo in range(0, V, chunk):
        srcs = np.arange(lo, min(V, lo + chunk), dtype=np.uint32)
        dist, nh, _ = eng.solve(srcs, use_metric)
        if expect_kernel is not None:
            ran = eng.last_kernels()
            assert expect_kernel in ran, ran
        for clo in range(0, len(srcs), check_chunk):
            sub = srcs[clo:clo + check_chunk]
            odist, onh = o.all_sources(sub, use_metric, nthreads=16)
            d, n = dist[clo:clo + check_chunk], nh[clo:clo + check_chunk]
            bad = np.nonzero(np.any(d != odist, axis=1))[0]
            assert bad.size == 0, f"dist differs for sources {sub[bad[:8]].tolist()}"
            bad = np.nonzero(np.any(n != onh, axis=(1, 2)))[0]
            assert bad.size == 0, f"next hops differ for sources {sub[bad[:8]].tolist()}"


def pathlinks_vs_oracle(eng, g, sources, use_metric=True):
    eng.set_graph(g)
    o = Oracle(g)
    dist, _, tight = eng.solve(sources, use_metric, want_tight=True)
    for i, s in enumerate(sources):
        run = o.run_spf(int(s), use_metric)
        pe = tight_in_edges(g, dist[i], tight[i])
        for v in np.nonzero(run.reachable())[0].tolist():
            assert pe.get(v, []) == run.pl_edge[run.pl_ptr[v]: run.pl_ptr[v + 1]].tolist(), (s, v)


def test_config1_grid10_all_sources():
    """DecisionBenchmark 10x10 grid (RoutingBenchmarkUtils.cpp:205-240): all 100 sources,
    link metric and hop count, dist + next hops + pathLinks."""
    e = SpfEngine()
    try:
        g = T.grid(10)
        for use_metric in (True, False):
            all_sources_vs_oracle(e, g, 100, use_metric)
            pathlinks_vs_oracle(e, g, list(range(100)), use_metric)
        a = np.arange(100)
        dist, _, _ = e.solve(a, True)
        assert np.array_equal(dist.astype(np.int64), np.abs(a[:, None] % 10 - a % 10) + np.abs(a[:, None] // 10 - a // 10))
    finally:
        e.close()


@pytest.mark.parametrize("faithful", [False, True], ids=["intended", "reference-faithful"])
def test_config2_fabric5000_all_sources(eng, faithful):
    """Fabric ~5k nodes (84 pods x 8 planes x 36 SSWs), every one of the
    4 992 sources, ECMP next-hop sets up to 84 bits wide; both generator variants."""
    g = T.fabric(5000, faithful=faithful)
    assert g.num_nodes == 4992 and g.num_links == (56448 if not faithful else 32544)
    # all 4 992 sources in one call, as bench.py launches them
    all_sources_vs_oracle(eng, g, 4992, check_chunk=1248)
    pathlinks_vs_oracle(eng, g, [0, 287, 288, 959, 960, 4991])


def test_config3_grid100_all_sources(eng):
    """100x100 grid, all 10 000 sources in ONE launch (the benchmarked configuration:
    bench.py solves them in one call, which runs the default all-sources pass
    CONFIG3_KERNEL), every row against the oracle; plus pathLinks of a source sample."""
    g = T.grid_fast(100)
    all_sources_vs_oracle(eng, g, 10000, expect_kernel=CONFIG3_KERNEL)
    pathlinks_vs_oracle(eng, g, [0, 99, 4950, 5050, 9900, 9999, 1234, 7777])


# the pass a full G100 batch takes by default (spf_bfs_lvl.hip)
CONFIG3_KERNEL = "bfs_ell_kernel"


@pytest.mark.parametrize("chunk,env,kernel", [
    (10000, {"OPENR_SPF_LEAN_DELTA": "0"}, "bfs_ell_kernel"),
    (10000, {"OPENR_SPF_BFS_WAVE": "1"}, "bfs_wave_kernel"),
    (1250, {}, "bfs_wave_kernel"),
    (1250, {"OPENR_SPF_BFS_WAVE": "0"}, "bfs_ell_kernel"),
], ids=["full-batch-lean-ellv", "full-batch-wave", "shard1250-auto", "shard1250-lean"])
def test_config3_grid100_pass_variants(eng, monkeypatch, chunk, env, kernel):
    """Config 3's other launch shapes, every row against the oracle: the full batch on the
    round-2 lean pass (16-byte ellv rows instead of the default delta rows) and on the wave
    pass, and the 1 250-source shards of an 8-GPU strong-scaling run (per-GPU step: the
    wave pass by default; the lean pass)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    all_sources_vs_oracle(eng, T.grid_fast(100), chunk, expect_kernel=kernel)


@pytest.mark.parametrize("mode", ["group", "group-lds", "group-d32", "group-cap", "group-cap1", "incr", "solve"])
def test_config4_wan_whatif_all_links(eng, mode, monkeypatch):
    """Per-link-failure sweep on the 1k-node WAN (U[1,64] asymmetric metrics): every one
    of the 3 000 links x 16 sources, changed-node counts vs oracle re-solves
    runSpf(src, true, {link}); grouped repair (default: u16 distances, global graph; LDS
    graph; u32 distances), per-unit repair and re-solve modes."""
    if mode == "group-lds":
        monkeypatch.setenv("OPENR_SPF_WHATIF_LDSG", "1")
    if mode == "group-d32":
        monkeypatch.setenv("OPENR_SPF_WHATIF_D32", "1")
    if mode == "group-cap":  # 8 dirty slots: larger units take the seeded re-solve
        monkeypatch.setenv("OPENR_SPF_WHATIF_CAP", "8")
    if mode == "group-cap1":  # 1 slot: nearly every affected unit is re-solved
        monkeypatch.setenv("OPENR_SPF_WHATIF_CAP", "1")
    monkeypatch.setenv("OPENR_SPF_WHATIF", mode.split("-")[0])
    g = T.wan(1000, 3000, 64, seed=1)
    eng.set_graph(g)
    links = np.arange(g.num_links, dtype=np.uint32)
    sources = np.linspace(0, g.num_nodes - 1, 16).astype(np.uint32)
    changed, solved = eng.whatif(links, sources, True)
    want = Oracle(g).whatif(links, sources, True)
    bad = np.argwhere(changed != want)
    assert bad.size == 0, f"(link, source) units differ: {bad[:8].tolist()}"
    assert changed.sum() > 0 and solved >= len(sources)


def test_config4_wan_whatif_full_workload(eng):
    """The whole benchmarked what-if workload — every one of the 3 000 links x every one
    of the 1 000 sources, 3 M units — in the default mode (grouped repair + seeded
    re-solves), each unit's changed-node count against the oracle's re-solve
    runSpf(src, true, {link}) (the oracle runs on the host's worker threads)."""
    g = T.wan(1000, 3000, 64, seed=1)
    eng.set_graph(g)
    links = np.arange(g.num_links, dtype=np.uint32)
    sources = np.arange(g.num_nodes, dtype=np.uint32)
    changed, solved = eng.whatif(links, sources, True)
    want = Oracle(g).whatif(links, sources, True)
    bad = np.argwhere(changed != want)
    assert bad.size == 0, f"{len(bad)} (link, source) units differ: {bad[:8].tolist()}"
    assert changed.shape == (3000, 1000) and changed.sum() > 0


def test_config4_wan_whatif_delta(eng):
    """openr_spf_whatif_delta on the config-4 WAN: all 3 000 links x 16 sources, each
    unit's changed nodes with their new u64 distance and next-hop bits, against oracle
    re-solves runSpf(src, true, {link}) through the oracle's per-unit digest, plus entry
    for entry on the first 150 links x 4 sources."""
    from oracle import delta_digest
    from test_gpu_parity import check_delta_rows

    g = T.wan(1000, 3000, 64, seed=1)
    eng.set_graph(g)
    links = np.arange(g.num_links, dtype=np.uint32)
    sources = np.linspace(0, g.num_nodes - 1, 16).astype(np.uint32)
    changed, ptr, node, dist, nh, _ = eng.whatif_delta(links, sources, True)
    want, dig = Oracle(g).whatif_delta_digest(links, sources, nh.shape[1], True)
    np.testing.assert_array_equal(changed, want)
    got = delta_digest(ptr, node, dist, nh).reshape(changed.shape)
    bad = np.argwhere(got != dig)
    assert bad.size == 0, f"{len(bad)} units' deltas differ: {bad[:8].tolist()}"
    n150 = 150 * len(sources)
    sub = [0, 5, 10, 15]
    sel = np.array([i * len(sources) + j for i in range(150) for j in sub])
    ptr2 = np.concatenate([[0], np.cumsum(changed.ravel()[sel])]).astype(np.uint64)
    take = np.concatenate([np.arange(int(ptr[u]), int(ptr[u + 1])) for u in sel]).astype(np.int64)
    check_delta_rows(g, links[:150], sources[sub], True, changed[:150][:, sub], ptr2, node[take], dist[take], nh[take])
    assert n150 > 0 and changed.sum() > 0


def test_config4_wan_whatif_delta_full_workload(eng):
    """The whole config-4 workload (3 000 links x 1 000 sources, 3 M units) with the
    delta: every unit's digest against the oracle's (host worker threads)."""
    from oracle import delta_digest

    g = T.wan(1000, 3000, 64, seed=1)
    eng.set_graph(g)
    links = np.arange(g.num_links, dtype=np.uint32)
    sources = np.arange(g.num_nodes, dtype=np.uint32)
    changed, ptr, node, dist, nh, _ = eng.whatif_delta(links, sources, True)
    want, dig = Oracle(g).whatif_delta_digest(links, sources, nh.shape[1], True)
    np.testing.assert_array_equal(changed, want)
    got = delta_digest(ptr, node, dist, nh).reshape(changed.shape)
    bad = np.argwhere(got != dig)
    assert bad.size == 0, f"{len(bad)} units' deltas differ: {bad[:8].tolist()}"


def test_config5_fabric_ksp2_more_sources(eng):
    """KSP2 on the fabric for 40 more sources spread over the id range (SSWs, FSWs and
    RSWs of many pods) x every destination: 199 680 pairs (0.8 % of the benchmarked 24.9 M),
    both path lists edge for edge against the oracle."""
    g = T.fabric(5000)
    eng.set_graph(g)
    V = g.num_nodes
    srcs = np.linspace(1, V - 2, 40).astype(np.uint32)
    src = np.repeat(srcs, V)
    dst = np.tile(np.arange(V, dtype=np.uint32), len(srcs))
    t1, t2 = eng.ksp2_tokens(src, dst, 1024)
    o1, o2 = Oracle(g).ksp2_tokens(src, dst, 1024)
    for i in range(len(src)):
        for k, (a, b) in enumerate(((t1, o1), (t2, o2))):
            assert decode_paths(a[i]) == decode_paths(b[i]), (int(src[i]), int(dst[i]), k + 1)


def test_config5_fabric_ksp2_all_destinations(eng):
    """KSP2 on the fabric: getKthPaths(src, dst, 1) and (.., 2) for EVERY destination of an
    SSW, an FSW and an RSW source (3 x 4 992 pairs), traced on the device, edge for edge
    against the oracle."""
    g = T.fabric(5000)
    eng.set_graph(g)
    V = g.num_nodes
    ssw, fsw, rsw = 0, 288, 288 + 84 * 8
    assert g.names[ssw].startswith("1-") and g.names[fsw].startswith("2-") and g.names[rsw].startswith("3-")
    src = np.repeat(np.array([ssw, fsw, rsw], dtype=np.uint32), V)
    dst = np.tile(np.arange(V, dtype=np.uint32), 3)
    t1, t2 = eng.ksp2_tokens(src, dst, 1024)
    o1, o2 = Oracle(g).ksp2_tokens(src, dst, 1024)
    for i in range(len(src)):
        for k, (a, b) in enumerate(((t1, o1), (t2, o2))):
            assert decode_paths(a[i]) == decode_paths(b[i]), (int(src[i]), int(dst[i]), k + 1)
    n2 = np.array([int(r[0]) for r in t2])
    assert (n2[dst != src] > 0).mean() > 0.5  # most pairs have edge-disjoint second paths
