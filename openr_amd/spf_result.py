"""Host-side materialisation of engine outputs into the reference's SPF views.

The engine returns dense arrays (include/openr_spf.h). This module rebuilds the
reference structures from them:

* ``NodeSpfResult`` (LinkState.h:203-257): metric, nextHops (neighbour names),
  pathLinks [(link, prevNode)] in the reference's order — tight in-edges of v
  sorted by (dist[u], name of u) = the settle order of u (DijkstraQ pop order,
  LinkState.h:488-498), then by position in row u (= linksFromNode(u) order).
* ``get_kth_paths`` (LinkState.cpp:762-791): k=1 traces the base SPF; k>=2 runs
  one GPU solve that ignores every link of the paths for i<k
  (openr_spf_solve_ignore), then ``trace_one_path`` (LinkState.cpp:398-419)
  greedily extracts edge-disjoint paths on the host.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np

U64_MAX = 0xFFFFFFFFFFFFFFFF


@dataclass
class NodeSpfResult:
    metric: int
    next_hops: Set[str] = field(default_factory=set)
    path_links: List[Tuple[int, str]] = field(default_factory=list)  # (link id, prevNode)
    path_edges: List[int] = field(default_factory=list)  # directed edge ids (prev = row owner)


def nh_names(g, src: int, nh_row: np.ndarray, nbrs: Sequence[int]) -> Set[str]:
    out = set()
    for i, nb in enumerate(nbrs):
        if (int(nh_row[i >> 3]) >> (i & 7)) & 1:
            out.add(g.names[int(nb)])
    return out


def tight_in_edges(g, dist: np.ndarray, tight: np.ndarray, owner: Optional[np.ndarray] = None,
                   pop: Optional[np.ndarray] = None) -> Dict[int, List[int]]:
    """Per node v: tight in-edges (u->v) in the reference's pathLinks order: the settle
    order of u ((dist, name), or the exact kernel's pop index `pop`), then row position."""
    if owner is None:
        owner = g.edge_owner()
    E = g.num_dir_edges
    bits = np.unpackbits(tight.view(np.uint8), bitorder="little")[:E].astype(bool)
    edges = np.nonzero(bits)[0]
    per: Dict[int, List[int]] = {}
    if edges.size == 0:
        return per
    us = owner[edges].astype(np.int64)
    vs = g.col[edges].astype(np.int64)
    if pop is not None:
        order = np.lexsort((edges, pop[us]))
    else:
        order = np.lexsort((edges, g.name_rank[us], dist[us]))  # settle order of u, then row position
    for idx in order.tolist():
        per.setdefault(int(vs[idx]), []).append(int(edges[idx]))
    return per


def materialize(g, src: int, dist: np.ndarray, nh: np.ndarray, nbrs: Sequence[int],
                tight: Optional[np.ndarray] = None, pop: Optional[np.ndarray] = None) -> Dict[str, NodeSpfResult]:
    """Dense outputs of one solve -> SpfResult (name -> NodeSpfResult)."""
    owner = g.edge_owner()
    pls = tight_in_edges(g, dist, tight, owner, pop) if tight is not None else {}
    res: Dict[str, NodeSpfResult] = {}
    reached = (pop != 0xFFFFFFFF) if pop is not None else (dist != np.uint64(U64_MAX))  # wrapped sums may be U64_MAX
    for v in np.nonzero(reached)[0].tolist():
        r = NodeSpfResult(int(dist[v]), nh_names(g, src, nh[v], nbrs))
        for e in pls.get(v, []):
            r.path_edges.append(e)
            r.path_links.append((int(g.link_id[e]), g.names[int(owner[e])]))
        res[g.names[v]] = r
    return res


def trace_one_path(g, owner: np.ndarray, src: int, dest: int, path_edges: Dict[int, List[int]],
                   visited: Set[int]) -> Optional[List[int]]:
    """LinkState::traceOnePath (LinkState.cpp:398-419), explicit stack."""
    if src == dest:
        return []
    stack = [[dest, 0, -1]]  # node, next pathLink index, edge taken
    while stack:
        f = stack[-1]
        if f[0] == src:
            return [fr[2] for fr in reversed(stack[:-1])]
        pls = path_edges.get(f[0], [])
        pushed = False
        while f[1] < len(pls):
            e = pls[f[1]]
            f[1] += 1
            link = int(g.link_id[e])
            if link not in visited:
                visited.add(link)
                f[2] = e
                stack.append([int(owner[e]), 0, -1])
                pushed = True
                break
        if not pushed:
            stack.pop()
    return None


def get_kth_paths(engine, src: int, dest: int, k: int) -> List[List[int]]:
    """LinkState::getKthPaths on the GPU engine; paths as directed edge ids (src->dest)."""
    if k < 1:
        raise ValueError("k must be >= 1 (CHECK_GE(k, 1), LinkState.cpp:765)")
    g = engine.g
    owner = g.edge_owner()
    ignore: List[int] = []
    paths: List[List[int]] = []
    for level in range(1, k + 1):
        if ignore:
            dist, _, tight = engine.solve([src], True, want_nh=False, want_tight=True, ignore=[sorted(set(ignore))])
        else:
            dist, _, tight = engine.solve([src], True, want_nh=False, want_tight=True)
        paths = []
        if dist[0, dest] != np.uint64(U64_MAX):
            pe = tight_in_edges(g, dist[0], tight[0], owner)
            visited: Set[int] = set()
            while True:
                p = trace_one_path(g, owner, src, dest, pe, visited)
                if not p:
                    break
                paths.append(p)
        if level < k:
            for p in paths:
                ignore.extend(int(g.link_id[e]) for e in p)
    return paths


def path_a_in_path_b(a: Sequence[int], b: Sequence[int]) -> bool:
    """LinkState::pathAInPathB (LinkState.h:395-410) over link ids."""
    if len(a) > len(b):
        return False
    for i in range(len(b) - len(a) + 1):
        if list(b[i : i + len(a)]) == list(a):
            return True
    return False
