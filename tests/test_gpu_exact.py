"""GPU parity of the exact-order kernel (spf_exact.hip) against the oracle, bit-exact.

The exact-order kernel replays LinkState::runSpf's heap process (LinkState.cpp:808-882)
where the fast kernels' assumptions fail: zero metrics and i32-negative metrics (stored
as u64, sums wrapping mod 2^64 — SURVEY.md Appendix A.2: the pop order then depends on
the relaxation history), next-hop sets wider than 256 bits, and graphs larger than the
LDS-resident layouts. Compared per solve: dist, next hops, the pathLinks edge set with
its order rebuilt from the kernel's pop index, and the pop index itself. Forced runs
(OPENR_SPF_FORCE_EXACT) on ordinary graphs check the kernel against the fast path's
inputs too; both the LDS-resident and the global-memory slot layouts are covered.
"""
import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.engine import ENOTSUP, SpfEngine, SpfError
from openr_amd.spf_result import tight_in_edges
from oracle import Oracle

pytestmark = pytest.mark.gpu

U64 = 2**64


@pytest.fixture(scope="module")
def eng():
    e = SpfEngine()
    yield e
    e.close()


@pytest.fixture(params=["lds", "global"])
def slot(request, monkeypatch):
    if request.param == "global":
        monkeypatch.setenv("OPENR_SPF_EXACT_GLOBAL", "1")
    return request.param


def random_graph(seed, V, L, metrics, p_ovl=0.08, p_down=0.05, p_par=0.1):
    """Random connected multigraph whose directed metrics are drawn from `metrics`."""
    rng = np.random.default_rng(seed)
    names = [f"r{rng.integers(0, 10**6)}-{i}" for i in range(V)]
    links = [(int(rng.integers(0, i)), i) for i in range(1, V)]
    while len(links) < L:
        a, b = rng.integers(0, V, 2)
        if a != b:
            links.append((int(a), int(b)))
    for _ in range(int(p_par * L)):
        links.append(links[int(rng.integers(0, len(links)))])
    pool = np.array([m % U64 for m in metrics], dtype=np.uint64)
    m_uv = pool[rng.integers(0, len(pool), len(links))]
    m_vu = pool[rng.integers(0, len(pool), len(links))]
    up = (rng.random(len(links)) >= p_down).astype(np.uint8)
    ovl = (rng.random(V) < p_ovl).astype(np.uint8)
    return T.csr_from_links(names, np.array(links), m_uv, m_vu, ovl, up)


def pop_index(run, V):
    pop = np.full(V, 0xFFFFFFFF, dtype=np.uint32)
    pop[run.order] = np.arange(len(run.order), dtype=np.uint32)
    return pop


def check_exact(eng, g, sources, use_metric=True, ignore=None):
    """solve_order == oracle: dist, nh, pop index, pathLinks (tight set in pop order);
    the plain solve returns the same dist / nh."""
    eng.set_graph(g)
    o = Oracle(g)
    V = g.num_nodes
    dist, nh, tight, order = eng.solve_order(sources, use_metric, want_tight=True, ignore=ignore)
    for i, s in enumerate(sources):
        run = o.run_spf(int(s), use_metric, ignore[i] if ignore else None)
        np.testing.assert_array_equal(dist[i], run.dist, err_msg=f"dist src={s}")
        np.testing.assert_array_equal(nh[i], run.nh, err_msg=f"nh src={s}")
        np.testing.assert_array_equal(order[i], pop_index(run, V), err_msg=f"pop order src={s}")
        pe = tight_in_edges(g, dist[i], tight[i], pop=order[i])
        for v in np.nonzero(run.reachable())[0].tolist():
            assert pe.get(v, []) == run.pl_edge[run.pl_ptr[v]: run.pl_ptr[v + 1]].tolist(), (s, v)
    d2, n2, _ = eng.solve(sources, use_metric, ignore=ignore)
    np.testing.assert_array_equal(d2, dist)
    np.testing.assert_array_equal(n2, nh)


ZERO = [0, 1, 2, 3]
WRAPPED = [0, 1, 5, 2**31 - 1, U64 - 1, U64 - 3, U64 - 2**31]  # i32 -1, -3, INT32_MIN


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("metrics", [ZERO, WRAPPED, [0]], ids=["zero", "wrapped", "all-zero"])
def test_zero_and_wrapped_metrics_all_sources(eng, slot, seed, metrics):
    g = random_graph(seed, 40 + 30 * seed, 90 + 60 * seed, metrics)
    check_exact(eng, g, list(range(g.num_nodes)), True)


def test_zero_metrics_with_ignore_sets(eng):
    g = random_graph(9, 120, 300, ZERO)
    rng = np.random.default_rng(9)
    srcs = rng.integers(0, g.num_nodes, 48).tolist()
    ignore = [sorted(set(rng.integers(0, g.num_links, int(rng.integers(0, 12))).tolist())) for _ in srcs]
    check_exact(eng, g, srcs, True, ignore)


def test_zero_metric_hop_count_uses_fast_kernels(eng):
    """useLinkMetric=false ignores metrics: the fast kernels serve it, same answers."""
    g = random_graph(3, 80, 200, ZERO)
    eng.set_graph(g)
    o = Oracle(g)
    srcs = list(range(g.num_nodes))
    dist, nh, _ = eng.solve(srcs, False)
    odist, onh = o.all_sources(np.array(srcs, dtype=np.uint32), False)
    np.testing.assert_array_equal(dist, odist)
    np.testing.assert_array_equal(nh, onh)


@pytest.mark.parametrize("graph", ["grid", "fabric", "random"])
def test_forced_exact_matches_fast_path(eng, slot, graph, monkeypatch):
    """The exact kernel on graphs the fast kernels serve: identical rows, pathLinks in the
    (dist, name) order the fast path documents."""
    g = {"grid": lambda: T.grid_fast(12), "fabric": lambda: T.fabric(288 + 56),
         "random": lambda: random_graph(5, 150, 400, list(range(1, 40)))}[graph]()
    srcs = list(range(0, g.num_nodes, max(1, g.num_nodes // 64)))
    eng.set_graph(g)
    fast = eng.solve(srcs, True, want_tight=True)
    monkeypatch.setenv("OPENR_SPF_FORCE_EXACT", "1")
    ex = eng.solve(srcs, True, want_tight=True)
    for a, b in zip(fast, ex):
        np.testing.assert_array_equal(a, b)
    check_exact(eng, g, srcs, True)


def test_more_than_256_next_hops(eng, slot):
    """A hub with 300 distinct neighbours (next-hop rows of 38 bytes): served by the exact
    kernel instead of being refused."""
    rng = np.random.default_rng(4)
    V = 420
    links = [(0, v) for v in range(1, 301)]  # hub 0
    links += [(int(rng.integers(1, 301)), v) for v in range(301, V)]  # second tier
    links += [(int(a), int(b)) for a, b in rng.integers(1, V, (200, 2)) if a != b]
    links = np.array(links)
    m = rng.integers(1, 6, len(links)).astype(np.uint64)
    names = [f"x{rng.integers(0, 10**6)}-{i}" for i in range(V)]
    g = T.csr_from_links(names, links, m, m, np.zeros(V, np.uint8))
    assert g.max_distinct_degree() == 300
    eng.set_graph(g)
    assert eng.nh_bytes == 38
    srcs = [0, 1, 2, 150, 300, 301, V - 1]
    check_exact(eng, g, srcs, True)
    check_exact(eng, g, srcs, False)


def test_graph_beyond_lds_layouts(eng):
    """A 300x300 grid (90 000 nodes) exceeds the LDS-resident kernels: the exact kernel
    solves it from global-memory slots (sampled sources vs the oracle + Manhattan check)."""
    n = 300
    g = T.grid_fast(n)
    eng.set_graph(g)
    srcs = [0, n * n - 1, n * (n // 2) + n // 2, 12345]
    dist, nh, _ = eng.solve(srcs, True)
    a = np.arange(n * n)
    for i, s in enumerate(srcs):
        want = np.abs(s % n - a % n) + np.abs(s // n - a // n)
        assert np.array_equal(dist[i].astype(np.int64), want)
    o = Oracle(g)
    for i, s in enumerate(srcs[:2]):
        run = o.run_spf(s, True)
        np.testing.assert_array_equal(nh[i], run.nh)


@pytest.mark.parametrize("metrics", [ZERO, WRAPPED], ids=["zero", "wrapped"])
def test_whatif_zero_and_wrapped_metrics(eng, metrics):
    """Per-link-failure sweep on graphs outside the fast kernels' domain: every unit with an
    up link is re-solved on the exact kernel; changed counts vs the oracle."""
    g = random_graph(21, 90, 220, metrics)
    eng.set_graph(g)
    links = np.arange(g.num_links, dtype=np.uint32)
    sources = np.arange(0, g.num_nodes, 7, dtype=np.uint32)
    changed, _ = eng.whatif(links, sources, True)
    want = Oracle(g).whatif(links, sources, True)
    np.testing.assert_array_equal(changed, want)


def test_ksp2_refuses_zero_metrics(eng):
    g = random_graph(2, 30, 60, ZERO)
    eng.set_graph(g)
    with pytest.raises(SpfError) as ei:
        eng.ksp2_tokens([0], [1], 64)
    assert ei.value.code == ENOTSUP
