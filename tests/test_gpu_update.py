"""Incremental mirror updates on the GPU: openr_spf_patch_graph + openr_spf_refresh.

Rows solved on graph G, then patched to G' (metric changes, link down/up, node overload
toggles — the attribute changes LinkState::updateAdjacencyDatabase / decrementHolds
report as topology changes, LinkState.cpp:564-719, 500-514) and refreshed in place,
must equal the oracle's runSpf on G' (dist, next-hop sets, pathLinks via tight edges)
and a fresh engine solve on G', bit for bit. The BM_DecisionGrid / BM_DecisionFabric
update loops of the reference benchmark (RoutingBenchmarkUtils.cpp:407-479: toggle a
random node's overload bit, then revert it) are replayed on the full-size topologies.
"""
import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.engine import EINVAL, SpfEngine, SpfError
from openr_amd.spf_result import tight_in_edges
from oracle import Oracle
from test_gpu_parity import random_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = SpfEngine()
    yield e
    e.close()


@pytest.fixture(params=["auto", "lvl", "code"])
def family(request, monkeypatch):
    if request.param != "auto":
        monkeypatch.setenv("OPENR_SPF_BFS_FAMILY", request.param)
    return request.param


def random_patch(g, rng, n_edges=3, n_links=2, n_nodes=1, max_metric=9):
    e = rng.choice(g.num_dir_edges, n_edges, replace=False) if n_edges else np.zeros(0, np.int64)
    m = rng.integers(1, max_metric + 1, len(e)).astype(np.uint64)
    lk = rng.choice(g.num_links, n_links, replace=False) if n_links else np.zeros(0, np.int64)
    lu = rng.integers(0, 2, len(lk)).astype(np.uint8)
    nd = rng.choice(g.num_nodes, n_nodes, replace=False) if n_nodes else np.zeros(0, np.int64)
    no = (1 - g.node_overloaded[nd]).astype(np.uint8)  # toggle
    return dict(edges=e, metrics=m, links=lk, link_up=lu, nodes=nd, node_overloaded=no)


def check_rows(eng, g, sources, dist, nh, tight, use_metric=True, oracle_rows=None):
    """Refreshed rows == fresh engine solve == oracle (on `oracle_rows` of them)."""
    fd, fn, ft = eng.solve(sources, use_metric, want_nh=True, want_tight=tight is not None)
    np.testing.assert_array_equal(dist, fd)
    np.testing.assert_array_equal(nh, fn)
    if tight is not None:
        np.testing.assert_array_equal(tight, ft)
    o = Oracle(g)
    idx = range(len(sources)) if oracle_rows is None else oracle_rows
    for i in idx:
        run = o.run_spf(int(sources[i]), use_metric)
        np.testing.assert_array_equal(dist[i], run.dist, err_msg=f"dist src={sources[i]}")
        np.testing.assert_array_equal(nh[i], run.nh, err_msg=f"nh src={sources[i]}")
        if tight is not None:
            pe = tight_in_edges(g, dist[i], tight[i])
            for v in np.nonzero(run.reachable())[0].tolist():
                assert pe.get(v, []) == run.pl_edge[run.pl_ptr[v] : run.pl_ptr[v + 1]].tolist()


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("max_metric", [1, 9])
@pytest.mark.parametrize("with_tight", [True, False], ids=["tight", "exact"])
def test_random_patches_match_oracle(eng, family, seed, max_metric, with_tight):
    """Rows with tight-edge rows refresh through the first-stage filter; rows without
    through the exact second stage too (only rows whose dist / next hops move are
    re-solved, spf_update.hip refresh_exact)."""
    g = random_graph(200 + seed, 80 + 20 * seed, 200 + 40 * seed, max_metric)
    eng.set_graph(g)
    srcs = list(range(g.num_nodes))
    rng = np.random.default_rng(seed)
    dist, nh, tight = eng.solve(srcs, True, want_tight=with_tight)
    for step in range(4):
        p = random_patch(g, rng, max_metric=max_metric if step % 2 else 1)
        eng.patch(**p)
        g = eng.g
        n = eng.refresh(srcs, dist, nh, tight)
        assert 0 <= n <= len(srcs)
        check_rows(eng, g, srcs, dist, nh, tight)


@pytest.mark.parametrize("seed", range(3))
def test_hop_count_refresh(eng, seed):
    """useLinkMetric=false rows: metric-only patches re-solve nothing."""
    g = random_graph(300 + seed, 120, 300, 20)
    eng.set_graph(g)
    srcs = list(range(g.num_nodes))
    rng = np.random.default_rng(seed)
    dist, nh, _ = eng.solve(srcs, False)
    eng.patch(**random_patch(g, rng, n_edges=8, n_links=0, n_nodes=0, max_metric=20))
    assert eng.refresh(srcs, dist, nh, use_link_metric=False) == 0
    eng.patch(**random_patch(eng.g, rng, n_edges=0, n_links=3, n_nodes=2))
    eng.refresh(srcs, dist, nh, use_link_metric=False)
    check_rows(eng, eng.g, srcs, dist, nh, None, use_metric=False)


def test_grid_overload_toggle_benchmark_loop(eng):
    """BM_DecisionGrid update loop (RoutingBenchmarkUtils.cpp:455-479) on G100: overload a
    random node, refresh all-sources rows, revert it, refresh again."""
    g = T.grid_fast(100)
    eng.set_graph(g)
    srcs = np.arange(g.num_nodes, dtype=np.uint32)
    dist, nh, _ = eng.solve(srcs, True)
    base_d, base_n = dist.copy(), nh.copy()
    rng = np.random.default_rng(5)
    sample = rng.choice(g.num_nodes, 24, replace=False).tolist()
    for node in (int(rng.integers(0, g.num_nodes)), 0, 9999):
        eng.patch(nodes=[node], node_overloaded=[1])
        n = eng.refresh(srcs, dist, nh)
        assert n <= g.num_nodes
        check_rows(eng, eng.g, srcs, dist, nh, None, oracle_rows=sample)
        eng.patch(nodes=[node], node_overloaded=[0])
        eng.refresh(srcs, dist, nh)
        np.testing.assert_array_equal(dist, base_d)
        np.testing.assert_array_equal(nh, base_n)


@pytest.mark.parametrize("delta", ["1", "0"], ids=["delta8", "ellv"])
def test_grid_link_patches_lean_rows(eng, monkeypatch, delta):
    """Links going down and up on a grid, solved by the lean level pass from each form of
    its rows (byte deltas, 16-byte rows): the patched rows (a down link's slot becomes
    delta 0) and the refreshed rows equal the oracle's."""
    monkeypatch.setenv("OPENR_SPF_BFS_WAVE", "0")
    monkeypatch.setenv("OPENR_SPF_LEAN_DELTA", delta)
    g = T.grid_fast(40)
    eng.set_graph(g)
    srcs = np.arange(g.num_nodes, dtype=np.uint32)
    dist, nh, _ = eng.solve(srcs, True)
    rng = np.random.default_rng(int(delta) + 11)
    sample = rng.choice(g.num_nodes, 16, replace=False).tolist()
    for step in range(3):
        lk = rng.choice(g.num_links, 6, replace=False)
        eng.patch(links=lk, link_up=np.full(len(lk), step % 2, np.uint8))
        eng.refresh(srcs, dist, nh)
        check_rows(eng, eng.g, srcs, dist, nh, None, oracle_rows=sample)


def test_fabric_rsw_overload_toggle(eng):
    """BM_DecisionFabric update loop (RoutingBenchmarkUtils.cpp:407-446): an RSW's overload
    bit affects only sources that transit it (SSWs, FSWs), not the RSWs."""
    g = T.fabric(1200)
    eng.set_graph(g)
    srcs = np.arange(g.num_nodes, dtype=np.uint32)
    dist, nh, tight = eng.solve(srcs, True, want_tight=True)
    rsw = [i for i, nm in enumerate(g.names) if nm.startswith("3-")][7]
    eng.patch(nodes=[rsw], node_overloaded=[1])
    n = eng.refresh(srcs, dist, nh, tight)
    n_rsw = sum(1 for nm in g.names if nm.startswith("3-"))
    assert 0 < n <= g.num_nodes - n_rsw + 1
    check_rows(eng, eng.g, srcs, dist, nh, tight, oracle_rows=range(0, g.num_nodes, 37))


def test_fabric_rsw_overload_exact_filter(eng, monkeypatch):
    """Without tight rows the exact second stage re-solves only the rows the RSW toggle
    really moves (the pod's FSWs lose the RSW as a next hop towards the pod's other-plane
    FSWs; SSWs keep theirs through the other RSWs): far fewer than the first stage lists,
    and every row equals a fresh solve."""
    g = T.fabric(1200)
    eng.set_graph(g)
    srcs = np.arange(g.num_nodes, dtype=np.uint32)
    dist, nh, _ = eng.solve(srcs, True)
    rsw = [i for i, nm in enumerate(g.names) if nm.startswith("3-")][7]
    counts = []
    for exact in ("0", "1"):
        monkeypatch.setenv("OPENR_SPF_REFRESH_EXACT", exact)
        d, n = dist.copy(), nh.copy()
        eng.patch(nodes=[rsw], node_overloaded=[1])
        counts.append(eng.refresh(srcs, d, n))
        check_rows(eng, eng.g, srcs, d, n, None, oracle_rows=range(0, g.num_nodes, 37))
        eng.patch(nodes=[rsw], node_overloaded=[0])
        eng.refresh(srcs, d, n)
        np.testing.assert_array_equal(d, dist)
        np.testing.assert_array_equal(n, nh)
    assert 0 < counts[1] < counts[0] // 4, counts


def test_uniform_to_general_metric_switches_kernel(eng):
    """A metric change on a unit-metric grid moves solves from the BFS to the general kernel."""
    g = T.grid_fast(12)
    eng.set_graph(g)
    srcs = list(range(g.num_nodes))
    dist, nh, tight = eng.solve(srcs, True, want_tight=True)
    eng.patch(edges=[5, g.num_dir_edges - 3], metrics=[4, 2])
    n = eng.refresh(srcs, dist, nh, tight)
    assert 0 < n < len(srcs)
    check_rows(eng, eng.g, srcs, dist, nh, tight)
    eng.patch(edges=[5, g.num_dir_edges - 3], metrics=[1, 1])  # back to uniform
    eng.refresh(srcs, dist, nh, tight)
    check_rows(eng, eng.g, srcs, dist, nh, tight)


def test_wan_metric_changes(eng):
    g = T.wan(1000, 3000, 64, seed=1)
    eng.set_graph(g)
    srcs = np.arange(0, g.num_nodes, 3, dtype=np.uint32)
    dist, nh, _ = eng.solve(srcs, True)
    rng = np.random.default_rng(3)
    for _ in range(3):
        eng.patch(**random_patch(eng.g, rng, n_edges=4, n_links=1, n_nodes=0, max_metric=64))
        eng.refresh(srcs, dist, nh)
        check_rows(eng, eng.g, srcs, dist, nh, None, oracle_rows=range(0, len(srcs), 29))


def test_refresh_device_form(eng):
    import torch

    g = random_graph(77, 150, 400, 5)
    eng.set_graph(g)
    srcs = np.arange(g.num_nodes, dtype=np.uint32)
    dist, nh, _ = eng.solve(srcs, True)
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(srcs.astype(np.int32)).to(dev)
    d_d = torch.from_numpy(dist.view(np.int64)).to(dev)
    d_n = torch.from_numpy(nh).to(dev)
    eng.patch(**random_patch(g, np.random.default_rng(1)))
    n = eng.refresh_device(d_s.data_ptr(), len(srcs), d_d.data_ptr(), d_n.data_ptr(), nh.shape[2])
    torch.cuda.synchronize()
    n2 = eng.refresh(srcs, dist, nh)  # same delta, host form
    assert n == n2
    np.testing.assert_array_equal(d_d.cpu().numpy().view(np.uint64), dist)
    np.testing.assert_array_equal(d_n.cpu().numpy(), nh)
    check_rows(eng, eng.g, srcs, dist, nh, None)


def test_patch_errors(eng):
    g = T.grid_fast(6)
    eng.set_graph(g)
    d, n, _ = eng.solve([0, 1], True)
    with pytest.raises(SpfError) as ei:
        eng.refresh([0, 1], d, n)  # no patch since set_graph
    assert ei.value.code == EINVAL
    with pytest.raises(SpfError) as ei:
        eng.patch(edges=[g.num_dir_edges], metrics=[3])
    assert ei.value.code == EINVAL
    with pytest.raises(SpfError) as ei:
        eng.patch(nodes=[g.num_nodes], node_overloaded=[1])
    assert ei.value.code == EINVAL
    eng.patch(edges=[0], metrics=[0])  # a zero metric: every row re-solved by the exact kernel
    assert eng.refresh([0, 1], d, n) == 2
    check_rows(eng, eng.g, [0, 1], d, n, None)
    eng.patch()  # empty patch after a zero-metric graph: rows re-solved again
    assert eng.refresh([0, 1], d, n) == 2
    eng.patch(edges=[0], metrics=[1])  # back to positive metrics: rows from the exact kernel refreshed
    assert eng.refresh([0, 1], d, n) == 2
    check_rows(eng, eng.g, [0, 1], d, n, None)
    eng.patch()  # empty patch: nothing to re-solve
    eng.patch(edges=[0], metrics=[1])
    assert eng.refresh([0, 1], d, n) >= 0
    check_rows(eng, eng.g, [0, 1], d, n, None)


def test_two_patches_one_refresh(eng, family):
    """Patches with no refresh in between accumulate their delta: one refresh of the rows
    of the original graph brings them to the twice-patched graph (edges changed and changed
    back drop out; edges changed twice keep their original state)."""
    g = random_graph(77, 120, 320, 9)
    eng.set_graph(g)
    srcs = list(range(g.num_nodes))
    dist, nh, tight = eng.solve(srcs, True, want_tight=True)
    rng = np.random.default_rng(77)
    e = rng.choice(g.num_dir_edges, 6, replace=False)
    eng.patch(edges=e, metrics=rng.integers(1, 10, 6).astype(np.uint64))
    eng.patch(edges=e[:3], metrics=g.metric[e[:3]])  # three of them back to the original
    lk = rng.choice(g.num_links, 2, replace=False)
    eng.patch(links=lk, link_up=np.zeros(2, np.uint8))
    eng.refresh(srcs, dist, nh, tight)
    check_rows(eng, eng.g, srcs, dist, nh, tight, oracle_rows=range(0, len(srcs), 7))
    # after a refresh the next patch starts a new delta
    eng.patch(links=lk, link_up=np.ones(2, np.uint8))
    eng.refresh(srcs, dist, nh, tight)
    check_rows(eng, eng.g, srcs, dist, nh, tight, oracle_rows=range(0, len(srcs), 7))
