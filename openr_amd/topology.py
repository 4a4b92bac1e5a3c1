"""Topology model and CSR mirror for the SPF engine.

Mirrors how ``openr::LinkState`` turns AdjacencyDatabases into links
(/root/reference/openr/decision/LinkState.cpp:531-547 ``maybeMakeLink``,
:564-719 ``updateAdjacencyDatabase``) and packs the result into the CSR layout
the C-ABI consumes (include/openr_spf.h ``openr_spf_graph``):

* a link exists iff both ends advertise each other with matching
  ``ifName``/``otherIfName``; parallel links are distinct links;
* directed edge u->v carries ``metric`` = u's advertised metric as u64
  (``Adjacency.metric`` is i32, LinkState.cpp:151-152: negative values wrap);
* ``edge_up`` = ``Link::isUp()`` = neither side's adjacency overload bit set
  (LinkState.cpp:233-236; hold TTLs are zero for generated topologies);
* row u lists u's links in the order of u's adjacency list. (The C++ host
  mirror, openr_amd/csrc/host, captures the live ``linksFromNode`` order
  instead; see DESIGN.md "Row order".)

Generators restate the reference's benchmark topologies
(/root/reference/openr/decision/tests/RoutingBenchmarkUtils.cpp:82-134,
155-400) plus the WAN topology defined in SURVEY.md §8d.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

U64_MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


@dataclass
class Adjacency:
    """Subset of ``thrift::Adjacency`` (openr/if/Lsdb.thrift:71-105) used by SPF."""

    other_node: str
    if_name: str
    other_if_name: str
    metric: int = 1
    is_overloaded: bool = False
    adj_label: int = 0


@dataclass
class AdjacencyDatabase:
    """Subset of ``thrift::AdjacencyDatabase`` (openr/if/Lsdb.thrift:109-129)."""

    node: str
    adjacencies: List[Adjacency] = field(default_factory=list)
    is_overloaded: bool = False
    node_label: int = 0


@dataclass
class CsrGraph:
    """Dense-id CSR mirror of a LinkState (layout of ``openr_spf_graph``)."""

    names: List[str]
    row_ptr: np.ndarray  # u32 [V+1]
    col: np.ndarray  # u32 [E]
    metric: np.ndarray  # u64 [E]
    link_id: np.ndarray  # u32 [E]
    edge_up: np.ndarray  # u8  [E]
    node_overloaded: np.ndarray  # u8 [V]
    name_rank: np.ndarray  # u32 [V]
    num_links: int
    link_ends: List[Tuple[Tuple[str, str], Tuple[str, str]]] = field(default_factory=list)
    index: Dict[str, int] = field(default_factory=dict)

    @property
    def num_nodes(self) -> int:
        return len(self.names)

    @property
    def num_dir_edges(self) -> int:
        return int(self.col.shape[0])

    def id(self, name: str) -> int:
        return self.index[name]

    def row(self, u: int) -> range:
        return range(int(self.row_ptr[u]), int(self.row_ptr[u + 1]))

    def distinct_neighbors(self, u: int) -> List[int]:
        """Next-hop bit i of a solve from u <-> this list's i-th entry."""
        seen: List[int] = []
        for e in self.row(u):
            v = int(self.col[e])
            if v not in seen:
                seen.append(v)
        return seen

    def max_distinct_degree(self) -> int:
        best = 0
        for u in range(self.num_nodes):
            d = int(self.row_ptr[u + 1] - self.row_ptr[u])
            if d <= best:
                continue
            best = max(best, len(set(self.col[self.row_ptr[u] : self.row_ptr[u + 1]].tolist())))
        return best

    def nh_bytes(self) -> int:
        return max(1, (self.max_distinct_degree() + 7) // 8)

    def edge_owner(self) -> np.ndarray:
        return np.repeat(np.arange(self.num_nodes, dtype=np.uint32), np.diff(self.row_ptr))

    def patched(self, edges, metrics, links, link_up, nodes, node_overloaded) -> "CsrGraph":
        """Copy with the attributes of ``openr_spf_patch_graph`` applied (same structure)."""
        metric = self.metric.copy()
        up = self.edge_up.copy()
        ovl = self.node_overloaded.copy()
        metric[np.asarray(edges, dtype=np.int64)] = np.asarray(metrics, dtype=np.uint64)
        if len(links):
            lk = set(int(x) for x in links)
            want = dict(zip((int(x) for x in links), (1 if x else 0 for x in link_up)))
            for e in np.nonzero(np.isin(self.link_id, list(lk)))[0]:
                up[e] = want[int(self.link_id[e])]
        ovl[np.asarray(nodes, dtype=np.int64)] = np.asarray(node_overloaded, dtype=np.uint8) != 0
        return CsrGraph(self.names, self.row_ptr, self.col, metric, self.link_id, up, ovl, self.name_rank,
                        self.num_links, self.link_ends, self.index)

    def ctypes_struct(self, struct_type):
        """Fill a ctypes mirror of ``openr_spf_graph``/``oracle_graph``; keeps refs alive."""
        arrs = [
            np.ascontiguousarray(self.row_ptr, dtype=np.uint32),
            np.ascontiguousarray(self.col, dtype=np.uint32),
            np.ascontiguousarray(self.metric, dtype=np.uint64),
            np.ascontiguousarray(self.link_id, dtype=np.uint32),
            np.ascontiguousarray(self.edge_up, dtype=np.uint8),
            np.ascontiguousarray(self.node_overloaded, dtype=np.uint8),
            np.ascontiguousarray(self.name_rank, dtype=np.uint32),
        ]
        s = struct_type()
        s.num_nodes = self.num_nodes
        s.num_dir_edges = self.num_dir_edges
        s.num_links = self.num_links
        s.row_ptr = arrs[0].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        s.col = arrs[1].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        s.metric = arrs[2].ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        s.link_id = arrs[3].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        s.edge_up = arrs[4].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        s.node_overloaded = arrs[5].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        s.name_rank = arrs[6].ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        s._keepalive = arrs  # type: ignore[attr-defined]
        return s


def _to_u64(metric: int) -> int:
    # i32 -> LinkStateMetric (uint64_t) conversion of Link::Link (LinkState.cpp:151)
    return metric & 0xFFFFFFFFFFFFFFFF


def build_csr(dbs: Iterable[AdjacencyDatabase]) -> CsrGraph:
    """AdjacencyDatabases -> CSR mirror following LinkState's link rules."""
    dbs = list(dbs)
    by_name: Dict[str, AdjacencyDatabase] = {}
    for db in dbs:
        by_name[db.node] = db  # later publication replaces earlier (updateAdjacencyDatabase)
    names = list(by_name.keys())
    index = {n: i for i, n in enumerate(names)}

    # link identity = unordered pair of (node, ifName) ends (LinkState.cpp:138-142)
    link_ids: Dict[Tuple[Tuple[str, str], Tuple[str, str]], int] = {}
    link_ends: List[Tuple[Tuple[str, str], Tuple[str, str]]] = []
    rows: List[List[Tuple[int, int, int, int]]] = [[] for _ in names]  # (v, metric, link, up)

    def reverse_adj(node: str, adj: Adjacency) -> Optional[Adjacency]:
        other = by_name.get(adj.other_node)
        if other is None:
            return None
        for oadj in other.adjacencies:
            if (
                oadj.other_node == node
                and adj.other_if_name == oadj.if_name
                and adj.if_name == oadj.other_if_name
            ):
                return oadj  # first match, as maybeMakeLink
        return None

    for name in names:
        db = by_name[name]
        seen_ends = set()
        for adj in db.adjacencies:
            radj = reverse_adj(name, adj)
            if radj is None:
                continue
            key = tuple(sorted([(name, adj.if_name), (adj.other_node, radj.if_name)]))
            if key in seen_ends:
                continue  # duplicate advertisement of the same link
            seen_ends.add(key)
            lid = link_ids.get(key)
            if lid is None:
                lid = len(link_ends)
                link_ids[key] = lid
                link_ends.append(key)  # type: ignore[arg-type]
            up = int(not adj.is_overloaded and not radj.is_overloaded)
            rows[index[name]].append((index[adj.other_node], _to_u64(adj.metric), lid, up))

    row_ptr = np.zeros(len(names) + 1, dtype=np.uint32)
    for i, r in enumerate(rows):
        row_ptr[i + 1] = row_ptr[i] + len(r)
    flat = [x for r in rows for x in r]
    col = np.array([x[0] for x in flat], dtype=np.uint32)
    metric = np.array([x[1] for x in flat], dtype=np.uint64)
    lid = np.array([x[2] for x in flat], dtype=np.uint32)
    up = np.array([x[3] for x in flat], dtype=np.uint8)
    ovl = np.array([int(by_name[n].is_overloaded) for n in names], dtype=np.uint8)
    return CsrGraph(
        names=names,
        row_ptr=row_ptr,
        col=col,
        metric=metric,
        link_id=lid,
        edge_up=up,
        node_overloaded=ovl,
        name_rank=name_ranks(names),
        num_links=len(link_ends),
        link_ends=link_ends,  # type: ignore[arg-type]
        index=index,
    )


def name_ranks(names: Sequence[str]) -> np.ndarray:
    """Rank of each name under std::string operator< (bytewise compare)."""
    order = sorted(range(len(names)), key=lambda i: names[i].encode())
    rank = np.empty(len(names), dtype=np.uint32)
    rank[np.array(order, dtype=np.int64)] = np.arange(len(names), dtype=np.uint32)
    return rank


# ---------------------------------------------------------------------------
# Fast array-based builder for large synthetic topologies
# ---------------------------------------------------------------------------
def csr_from_links(
    names: Sequence[str],
    links: np.ndarray,
    metric_uv: Optional[np.ndarray] = None,
    metric_vu: Optional[np.ndarray] = None,
    overloaded: Optional[np.ndarray] = None,
    link_up: Optional[np.ndarray] = None,
) -> CsrGraph:
    """Undirected link list (L,2) -> CSR; row order = link order (stable).

    Equivalent to ``build_csr`` on the adjacency databases in which every node
    advertises its links in link order (used for the bench-size topologies).
    """
    V = len(names)
    links = np.asarray(links, dtype=np.int64).reshape(-1, 2)
    L = links.shape[0]
    if metric_uv is None:
        metric_uv = np.ones(L, dtype=np.uint64)
    if metric_vu is None:
        metric_vu = metric_uv
    if link_up is None:
        link_up = np.ones(L, dtype=np.uint8)
    src = np.concatenate([links[:, 0], links[:, 1]])
    dst = np.concatenate([links[:, 1], links[:, 0]])
    w = np.concatenate([np.asarray(metric_uv, dtype=np.uint64), np.asarray(metric_vu, dtype=np.uint64)])
    lid = np.concatenate([np.arange(L), np.arange(L)]).astype(np.uint32)
    up = np.concatenate([link_up, link_up]).astype(np.uint8)
    # row-major, and within a row by link id (advertisement order)
    order = np.lexsort((lid, src))
    row_ptr = np.zeros(V + 1, dtype=np.uint32)
    np.cumsum(np.bincount(src, minlength=V), out=row_ptr[1:])
    ovl = np.zeros(V, dtype=np.uint8) if overloaded is None else np.asarray(overloaded, dtype=np.uint8)
    return CsrGraph(
        names=list(names),
        row_ptr=row_ptr,
        col=dst[order].astype(np.uint32),
        metric=w[order],
        link_id=lid[order],
        edge_up=up[order],
        node_overloaded=ovl,
        name_rank=name_ranks(names),
        num_links=L,
        index={n: i for i, n in enumerate(names)},
    )


def grid(n: int) -> CsrGraph:
    """Grid via the adjacency-database path (row order = advertisement order)."""
    return build_csr(grid_dbs(n))


def grid_dbs(n: int, test_form: bool = False) -> List[AdjacencyDatabase]:
    """Adjacency DBs of the benchmark grid (RoutingBenchmarkUtils.cpp:205-240)
    or, with ``test_form``, of DecisionTest.cpp:4207-4265 (ifnames 0/1..0/4,
    nodeLabel node+1)."""
    dbs = []
    for r in range(n):
        for c in range(n):
            u = r * n + c
            adjs = []
            nbrs = [(r, c + 1, "0/1", "0/3"), (r - 1, c, "0/2", "0/4"), (r, c - 1, "0/3", "0/1"), (r + 1, c, "0/4", "0/2")]
            if not test_form:
                nbrs = [(r, c + 1, None, None), (r, c - 1, None, None), (r - 1, c, None, None), (r + 1, c, None, None)]
            for rr, cc, ifn, oifn in nbrs:
                if 0 <= rr < n and 0 <= cc < n:
                    v = rr * n + cc
                    if ifn is None:
                        ifn, oifn = f"if_{u}_{v}", f"if_{v}_{u}"
                    adjs.append(Adjacency(str(v), ifn, oifn, 1, False, 100001 + v))
            dbs.append(AdjacencyDatabase(str(u), adjs, False, u + 1 if test_form else 0))
    return dbs


# Fabric (RoutingBenchmarkUtils.h:53-58, RoutingBenchmarkUtils.cpp:248-400)
SSWS_PER_PLANE = 36
FSWS_PER_POD = 8
RSWS_PER_POD = 48


def fabric_pods(num_switches: int) -> int:
    planes = FSWS_PER_POD
    return (num_switches - planes * SSWS_PER_PLANE) // (FSWS_PER_POD + RSWS_PER_POD)


def fabric(num_switches: int = 5000, faithful: bool = False) -> CsrGraph:
    """Clos fabric: SSW "1-{plane}-{i}", FSW "2-{pod}-{plane}", RSW "3-{pod}-{i}".

    ``faithful=True`` reproduces the reference generator's ``emplace`` bug
    (RoutingBenchmarkUtils.cpp:256-273): each SSW keeps only its pod-0 FSW.
    """
    pods = fabric_pods(num_switches)
    planes = FSWS_PER_POD
    names: List[str] = []
    ids: Dict[Tuple[int, int, int], int] = {}

    def add(marker: int, a: int, b: int) -> None:
        ids[(marker, a, b)] = len(names)
        names.append(f"{marker}-{a}-{b}")

    for p in range(planes):
        for s in range(SSWS_PER_PLANE):
            add(1, p, s)
    for pod in range(pods):
        for f in range(FSWS_PER_POD):
            add(2, pod, f)
    for pod in range(pods):
        for r in range(RSWS_PER_POD):
            add(3, pod, r)
    # Per-node advertisement order: SSW -> FSW(pod, plane) by pod; FSW -> its
    # plane's SSWs then its pod's RSWs; RSW -> its pod's FSWs.
    adj: List[List[int]] = [[] for _ in names]
    for p in range(planes):
        for s in range(SSWS_PER_PLANE):
            u = ids[(1, p, s)]
            for pod in range(pods):
                adj[u].append(ids[(2, pod, p)])
    for pod in range(pods):
        for f in range(FSWS_PER_POD):
            u = ids[(2, pod, f)]
            for s in range(SSWS_PER_PLANE):
                adj[u].append(ids[(1, f, s)])
            for r in range(RSWS_PER_POD):
                adj[u].append(ids[(3, pod, r)])
    for pod in range(pods):
        for r in range(RSWS_PER_POD):
            u = ids[(3, pod, r)]
            for f in range(FSWS_PER_POD):
                adj[u].append(ids[(2, pod, f)])
    if faithful:
        for p in range(planes):
            for s in range(SSWS_PER_PLANE):
                u = ids[(1, p, s)]
                adj[u] = adj[u][:1]
    return _csr_from_adjacency_lists(names, adj)


def _csr_from_adjacency_lists(names: List[str], adj: List[List[int]], metric=None) -> CsrGraph:
    """Bidirectional-only links from per-node neighbour lists (no parallels)."""
    V = len(names)
    adjsets = [set(a) for a in adj]
    link_of: Dict[Tuple[int, int], int] = {}
    rows_c, rows_l = [], []
    for u in range(V):
        for v in adj[u]:
            if u not in adjsets[v]:
                continue  # not bidirectional -> no Link
            key = (u, v) if u < v else (v, u)
            lid = link_of.setdefault(key, len(link_of))
            rows_c.append(v)
            rows_l.append(lid)
    row_ptr = np.zeros(V + 1, dtype=np.uint32)
    cnt = [sum(1 for v in adj[u] if u in adjsets[v]) for u in range(V)]
    np.cumsum(np.array(cnt, dtype=np.uint32), out=row_ptr[1:])
    E = len(rows_c)
    return CsrGraph(
        names=names,
        row_ptr=row_ptr,
        col=np.array(rows_c, dtype=np.uint32),
        metric=np.ones(E, dtype=np.uint64) if metric is None else metric,
        link_id=np.array(rows_l, dtype=np.uint32),
        edge_up=np.ones(E, dtype=np.uint8),
        node_overloaded=np.zeros(V, dtype=np.uint8),
        name_rank=name_ranks(names),
        num_links=len(link_of),
        index={n: i for i, n in enumerate(names)},
    )


def wan(num_nodes: int = 1000, num_links: int = 3000, max_metric: int = 64, seed: int = 1,
        parallel_fraction: float = 0.0) -> CsrGraph:
    """WAN-like topology of BASELINE config 4: ring +
    uniform random chords, asymmetric metrics 1 + rng() % max_metric per direction,
    optional parallel links. The links and metrics come from the C++ generator
    (openr_topogen_wan, std::mt19937_64(seed), include/openr_topogen.h); only the CSR
    packing happens here."""
    from openr_amd import adjdb

    lib = adjdb.load_library()
    npar = int(parallel_fraction * num_links)
    L = num_links + npar
    ends = np.zeros(2 * L, dtype=np.uint32)
    m_uv = np.zeros(L, dtype=np.uint32)
    m_vu = np.zeros(L, dtype=np.uint32)
    rc = lib.openr_topogen_wan(num_nodes, num_links, max_metric, seed, npar, ends.ctypes.data, m_uv.ctypes.data,
                               m_vu.ctypes.data)
    if rc != 0:
        raise ValueError(f"openr_topogen_wan({num_nodes}, {num_links}, {max_metric}) failed: {rc}")
    names = [f"wan{i}" for i in range(num_nodes)]
    return csr_from_links(names, ends.reshape(-1, 2).astype(np.int64), m_uv.astype(np.uint64),
                          m_vu.astype(np.uint64))


def grid_fast(n: int) -> CsrGraph:
    """Array-built grid with the benchmark per-row order (col+1, col-1, row-1, row+1)."""
    names = [str(i) for i in range(n * n)]
    adj: List[List[int]] = []
    for r in range(n):
        for c in range(n):
            lst = []
            if c + 1 < n:
                lst.append(r * n + c + 1)
            if c - 1 >= 0:
                lst.append(r * n + c - 1)
            if r - 1 >= 0:
                lst.append((r - 1) * n + c)
            if r + 1 < n:
                lst.append((r + 1) * n + c)
            adj.append(lst)
    return _csr_from_adjacency_lists(names, adj)


def from_adj_map(adj_map: Dict[int, Sequence], name_fmt: str = "{}") -> CsrGraph:
    """``getLinkState`` fixture builder (DecisionTestUtils.cpp:16-42).

    ``adj_map``: node -> [adj | (adj, weight)]; parallel adjacencies numbered k
    per neighbour; ifName "{node}/{adj}/{k}", otherIfName "{adj}/{node}/{k}".
    """
    dbs = []
    for node, lst in adj_map.items():
        num_par: Dict[int, int] = {}
        adjs = []
        for item in lst:
            adj, w = (item if isinstance(item, (tuple, list)) else (item, 1))
            k = num_par.get(adj, 0)
            num_par[adj] = k + 1
            adjs.append(Adjacency(name_fmt.format(adj), f"{node}/{adj}/{k}", f"{adj}/{node}/{k}", int(w), False,
                                  (node << 16) + adj))
        dbs.append(AdjacencyDatabase(name_fmt.format(node), adjs, False, node))
    return build_csr(dbs)
