"""CPU check of the affected-row rule behind openr_spf_refresh (spf_update.hip).

For random graphs and attribute patches (metrics, link up/down, node overload), every
source the rule declares unaffected must have exactly the same oracle runSpf result
(dist, next-hop sets, pathLinks) before and after the patch — the rule is what lets the
engine skip re-solving that row. Also checks CsrGraph.patched against a rebuilt graph.
"""
import numpy as np
import pytest

from openr_amd import topology as T
from oracle import Oracle
from test_gpu_parity import random_graph

U64_MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


def affected(g0, g1, src, dist0, use_metric=True):
    """The refresh filter of spf_update.hip, restated: row src is affected iff a changed
    directed edge u->v was tight before or may be tight / shorter after."""
    owner = g0.edge_owner()
    for e in range(g0.num_dir_edges):
        u, v = int(owner[e]), int(g0.col[e])
        w0 = int(g0.metric[e]) if use_metric else 1
        w1 = int(g1.metric[e]) if use_metric else 1
        a0 = bool(g0.edge_up[e]) and (u == src or not g0.node_overloaded[u])
        a1 = bool(g1.edge_up[e]) and (u == src or not g1.node_overloaded[u])
        if a0 == a1 and w0 == w1:
            continue
        du = dist0[u]
        if du == U64_MAX:
            continue
        dv = int(dist0[v])
        if (a0 and int(du) + w0 == dv) or (a1 and int(du) + w1 <= dv):
            return True
    return False


def random_patch(g, rng, max_metric):
    e = rng.choice(g.num_dir_edges, 2, replace=False)
    m = rng.integers(1, max_metric + 1, 2).astype(np.uint64)
    lk = rng.choice(g.num_links, 1, replace=False)
    lu = rng.integers(0, 2, 1).astype(np.uint8)
    nd = rng.choice(g.num_nodes, 1, replace=False)
    no = (1 - g.node_overloaded[nd]).astype(np.uint8)
    return e, m, lk, lu, nd, no


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("max_metric", [1, 6])
def test_unaffected_rows_are_unchanged(seed, max_metric):
    g0 = random_graph(500 + seed, 40, 90, max_metric)
    rng = np.random.default_rng(seed)
    skipped = 0
    for use_metric in (True, False):
        g1 = g0.patched(*random_patch(g0, rng, max_metric))
        o0, o1 = Oracle(g0), Oracle(g1)
        for s in range(g0.num_nodes):
            r0 = o0.run_spf(s, use_metric)
            if affected(g0, g1, s, r0.dist, use_metric):
                continue
            skipped += 1
            r1 = o1.run_spf(s, use_metric)
            np.testing.assert_array_equal(r0.dist, r1.dist)
            np.testing.assert_array_equal(r0.nh, r1.nh)
            np.testing.assert_array_equal(r0.pl_ptr, r1.pl_ptr)
            np.testing.assert_array_equal(r0.pl_edge, r1.pl_edge)
    assert skipped > 0


def test_patched_graph_matches_rebuild():
    names = [str(i) for i in range(5)]
    links = np.array([(0, 1), (1, 2), (2, 3), (3, 4), (1, 3)])
    m = np.ones(len(links), dtype=np.uint64)
    g = T.csr_from_links(names, links, m, m)
    e = int(np.nonzero(g.link_id == 4)[0][0])
    p = g.patched([e], [7], [2], [0], [3], [1])
    assert p.metric[e] == 7 and g.metric[e] == 1
    assert (p.edge_up[g.link_id == 2] == 0).all() and (p.edge_up[g.link_id != 2] == 1).all()
    assert p.node_overloaded.tolist() == [0, 0, 0, 1, 0]
    assert p.row_ptr is g.row_ptr and p.col is g.col
