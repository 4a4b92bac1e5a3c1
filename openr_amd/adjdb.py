"""Bulk AdjacencyDatabase input path: KvStore "adj:" values -> CSR mirror.

Python binding of include/openr_adjdb.h (built into libopenr_decision.so from
openr_amd/csrc/host/AdjDbCodec.cpp). It replaces, for a whole publication at once, the
per-key ``readThriftObjStr<thrift::AdjacencyDatabase>(value, CompactSerializer)`` of
Decision::processPublication (/root/reference/openr/decision/Decision.cpp:1755-1757)
and the ``LinkState::updateAdjacencyDatabase`` calls after it (:1773-1777), ending in
the ``openr_spf_graph`` CSR the SPF engine consumes. The decode is native C++ on host
threads; there is no Python fallback (the library must be built).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Sequence

import numpy as np

from .provenance import check_build_id
from .topology import CsrGraph

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libopenr_decision.so")


class AdjDbInfo(ctypes.Structure):
    _fields_ = [("n_dbs", ctypes.c_uint32), ("n_adjs", ctypes.c_uint64), ("n_strings", ctypes.c_uint64),
                ("string_bytes", ctypes.c_uint64), ("n_perf_events", ctypes.c_uint64)]


_COLUMNS = [
    ("str_pool", np.uint8), ("str_off", np.uint64),
    ("node_name", np.uint32), ("area", np.uint32), ("node_overloaded", np.uint8), ("node_label", np.int32),
    ("adj_begin", np.uint64),
    ("other_node", np.uint32), ("if_name", np.uint32), ("other_if_name", np.uint32), ("nh_v6", np.uint32),
    ("nh_v4", np.uint32), ("metric", np.int32), ("adj_label", np.int32), ("adj_overloaded", np.uint8),
    ("rtt", np.int32), ("timestamp", np.int64), ("weight", np.int64),
]


class AdjDbColumns(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n, _ in _COLUMNS]


class GraphInfo(ctypes.Structure):
    _fields_ = [("num_nodes", ctypes.c_uint32), ("num_dir_edges", ctypes.c_uint32), ("num_links", ctypes.c_uint32),
                ("name_bytes", ctypes.c_uint64)]


class RouteStats(ctypes.Structure):  # openr_routes_stats_t (include/openr_routes.h)
    _fields_ = [("unicast_routes", ctypes.c_uint64), ("mpls_routes", ctypes.c_uint64),
                ("nexthops", ctypes.c_uint64), ("weighted_nexthops", ctypes.c_uint64),
                ("checksum", ctypes.c_uint64), ("ms_build", ctypes.c_double), ("ms_policy", ctypes.c_double)]


ROUTES_LFA, ROUTES_V4, ROUTES_UCMP = 1, 2, 4

_lib = None


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build first (python -c 'import __graft_entry__ as g; g.build()')")
    l = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, P = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER
    l.openr_adjdb_last_error.restype = ctypes.c_char_p
    l.openr_adjdb_decode.argtypes = [vp, vp, u32, u32, P(vp)]
    l.openr_adjdb_free.argtypes = [vp]
    l.openr_adjdb_free.restype = None
    l.openr_adjdb_info.argtypes = [vp, P(AdjDbInfo)]
    l.openr_adjdb_export.argtypes = [vp, P(AdjDbColumns)]
    l.openr_adjdb_encode.argtypes = [vp, u32, vp, u64, P(u64)]
    l.openr_adjdb_batch_from_columns.argtypes = [P(AdjDbColumns), u32, P(vp)]
    l.openr_adjdb_encode_all.argtypes = [vp, vp, u64, vp, P(u64)]
    l.openr_adjdb_build_graph.argtypes = [vp, ctypes.c_char_p, P(vp)]
    l.openr_adjdb_graph_free.argtypes = [vp]
    l.openr_adjdb_graph_free.restype = None
    l.openr_adjdb_graph_info.argtypes = [vp, P(GraphInfo)]
    l.openr_adjdb_graph_export.argtypes = [vp] + [vp] * 9
    l.openr_topogen_wan.argtypes = [u32, u32, u32, u64, u32, vp, vp, vp]
    l.openr_routes_build.argtypes = [vp, vp, u32, u32, ctypes.c_int32, vp, P(RouteStats)]
    l.openr_routes_build.restype = ctypes.c_int
    l.openr_topogen_wan.restype = ctypes.c_int
    l.openr_decision_build_id.restype = ctypes.c_char_p
    check_build_id(l.openr_decision_build_id().decode(), LIB_PATH)
    _lib = l
    return l


class AdjDbError(RuntimeError):
    def __init__(self, code: int, msg: str) -> None:
        super().__init__(f"{msg} (code {code})")
        self.code = code


def _check(rc: int) -> None:
    if rc != 0:
        raise AdjDbError(rc, load_library().openr_adjdb_last_error().decode())


def pack_values(values: Sequence[bytes]):
    """Concatenate values into (data u8, offsets u64 [n+1])."""
    offsets = np.zeros(len(values) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(v) for v in values], dtype=np.uint64)
    data = np.frombuffer(b"".join(values), dtype=np.uint8) if values else np.zeros(1, dtype=np.uint8)
    return data, offsets


class AdjDbBatch:
    """Decoded AdjacencyDatabases (native). ``columns()`` exports them columnar."""

    def __init__(self, data: np.ndarray, offsets: np.ndarray, n_threads: int = 0) -> None:
        l = load_library()
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offsets) - 1
        h = ctypes.c_void_p()
        _check(l.openr_adjdb_decode(data.ctypes.data if data.size else None, offsets.ctypes.data, n, n_threads,
                                    ctypes.byref(h)))
        self._h = h

    @classmethod
    def from_values(cls, values: Sequence[bytes], n_threads: int = 0) -> "AdjDbBatch":
        return cls(*pack_values(values), n_threads=n_threads)

    @classmethod
    def from_columns(cls, cols: Dict[str, np.ndarray]) -> "AdjDbBatch":
        """Inverse of ``columns()`` (addresses as text)."""
        c = AdjDbColumns()
        keep = []
        for name, dt in _COLUMNS:
            a = np.ascontiguousarray(cols[name], dtype=dt)
            if a.size == 0:
                a = np.zeros(1, dtype=dt)
            keep.append(a)
            setattr(c, name, a.ctypes.data)
        self = cls.__new__(cls)
        h = ctypes.c_void_p()
        _check(load_library().openr_adjdb_batch_from_columns(ctypes.byref(c), len(cols["node_name"]), ctypes.byref(h)))
        self._h = h
        return self

    def encode_all(self):
        """All databases encoded back to back: (data u8, offsets u64 [n+1])."""
        l = load_library()
        total = ctypes.c_uint64()
        _check(l.openr_adjdb_encode_all(self._h, None, 0, None, ctypes.byref(total)))
        data = np.zeros(max(1, total.value), dtype=np.uint8)
        offsets = np.zeros(self.info().n_dbs + 1, dtype=np.uint64)
        _check(l.openr_adjdb_encode_all(self._h, data.ctypes.data, total.value, offsets.ctypes.data,
                                        ctypes.byref(total)))
        return data[: total.value], offsets

    def close(self) -> None:
        if self._h:
            load_library().openr_adjdb_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> AdjDbInfo:
        i = AdjDbInfo()
        _check(load_library().openr_adjdb_info(self._h, ctypes.byref(i)))
        return i

    def columns(self) -> Dict[str, np.ndarray]:
        i = self.info()
        sizes = {"str_pool": max(1, i.string_bytes), "str_off": i.n_strings + 1, "adj_begin": i.n_dbs + 1}
        per_db = {"node_name", "area", "node_overloaded", "node_label"}
        arrs = {}
        c = AdjDbColumns()
        for name, dt in _COLUMNS:
            n = sizes.get(name, i.n_dbs if name in per_db else i.n_adjs)
            a = np.zeros(max(1, n), dtype=dt)
            arrs[name] = a
            setattr(c, name, a.ctypes.data)
        _check(load_library().openr_adjdb_export(self._h, ctypes.byref(c)))
        for name in list(arrs):
            if name in per_db:
                arrs[name] = arrs[name][: i.n_dbs]
            elif name not in sizes:
                arrs[name] = arrs[name][: i.n_adjs]
        arrs["str_pool"] = arrs["str_pool"][: i.string_bytes]
        return arrs

    def encode(self, index: int) -> bytes:
        l = load_library()
        n = ctypes.c_uint64()
        _check(l.openr_adjdb_encode(self._h, index, None, 0, ctypes.byref(n)))
        buf = np.zeros(max(1, n.value), dtype=np.uint8)
        _check(l.openr_adjdb_encode(self._h, index, buf.ctypes.data, n.value, ctypes.byref(n)))
        return buf[: n.value].tobytes()

    def to_csr(self, area: str = "0") -> CsrGraph:
        """Apply every database to a fresh LinkState of ``area`` and export its CSR."""
        l = load_library()
        g = ctypes.c_void_p()
        _check(l.openr_adjdb_build_graph(self._h, area.encode(), ctypes.byref(g)))
        try:
            gi = GraphInfo()
            _check(l.openr_adjdb_graph_info(g, ctypes.byref(gi)))
            V, E = gi.num_nodes, gi.num_dir_edges
            row_ptr = np.zeros(V + 1, np.uint32)
            col = np.zeros(max(1, E), np.uint32)
            metric = np.zeros(max(1, E), np.uint64)
            link_id = np.zeros(max(1, E), np.uint32)
            up = np.zeros(max(1, E), np.uint8)
            ovl = np.zeros(max(1, V), np.uint8)
            rank = np.zeros(max(1, V), np.uint32)
            pool = np.zeros(max(1, gi.name_bytes), np.uint8)
            off = np.zeros(V + 1, np.uint64)
            _check(l.openr_adjdb_graph_export(g, *(a.ctypes.data for a in
                                                   (row_ptr, col, metric, link_id, up, ovl, rank, pool, off))))
        finally:
            l.openr_adjdb_graph_free(g)
        raw = pool.tobytes()
        names = [raw[off[k]:off[k + 1]].decode(errors="surrogateescape") for k in range(V)]
        return CsrGraph(names, row_ptr, col[:E], metric[:E], link_id[:E], up[:E], ovl[:V], rank[:V], gi.num_links,
                        index={n: k for k, n in enumerate(names)})


class RouteBuilder:
    """Batched SpfSolver route build (include/openr_routes.h) over the LinkState that
    ``batch``'s databases form: SPF on the GPU engine, routes + RibPolicy on the host."""

    def __init__(self, batch: "AdjDbBatch", area: str = "0") -> None:
        l = load_library()
        self._g = ctypes.c_void_p()
        _check(l.openr_adjdb_build_graph(batch._h, area.encode(), ctypes.byref(self._g)))
        gi = GraphInfo()
        _check(l.openr_adjdb_graph_info(self._g, ctypes.byref(gi)))
        self.num_nodes = gi.num_nodes

    def names(self) -> List[str]:
        """Graph node names by id (ids = name ranks)."""
        l = load_library()
        gi = GraphInfo()
        _check(l.openr_adjdb_graph_info(self._g, ctypes.byref(gi)))
        V, E = gi.num_nodes, max(1, gi.num_dir_edges)
        bufs = [np.zeros(V + 1, np.uint32), np.zeros(E, np.uint32), np.zeros(E, np.uint64), np.zeros(E, np.uint32),
                np.zeros(E, np.uint8), np.zeros(max(1, V), np.uint8), np.zeros(max(1, V), np.uint32),
                np.zeros(max(1, gi.name_bytes), np.uint8), np.zeros(V + 1, np.uint64)]
        _check(l.openr_adjdb_graph_export(self._g, *(a.ctypes.data for a in bufs)))
        raw, off = bufs[7].tobytes(), bufs[8]
        return [raw[off[k]:off[k + 1]].decode(errors="surrogateescape") for k in range(V)]

    def build(self, node_ids: Sequence[int], flags: int = 0, default_weight: int = 1,
              neighbor_weight: "np.ndarray | None" = None) -> RouteStats:
        ids = np.ascontiguousarray(node_ids, dtype=np.uint32)
        w = None if neighbor_weight is None else np.ascontiguousarray(neighbor_weight, dtype=np.int32)
        if w is not None and w.shape[0] != self.num_nodes:
            raise ValueError("neighbor_weight must have one entry per graph node")
        st = RouteStats()
        _check(load_library().openr_routes_build(self._g, ids.ctypes.data if ids.size else None, ids.shape[0], flags,
                                                 default_weight, None if w is None else w.ctypes.data,
                                                 ctypes.byref(st)))
        return st

    def close(self) -> None:
        if self._g:
            load_library().openr_adjdb_graph_free(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def wan_ucmp_weights(names: Sequence[str]) -> np.ndarray:
    """SURVEY.md §8d row 4 RibPolicy neighbour weights: node wan{i} weighs 1 + i % 4 when
    i % 3 == 0 (others: none, i.e. the default weight 1)."""
    w = np.zeros(len(names), np.int32)
    for k, nm in enumerate(names):
        if nm.startswith("wan"):
            i = int(nm[3:])
            if i % 3 == 0:
                w[k] = 1 + i % 4
    return w


def strings(cols: Dict[str, np.ndarray]) -> List[str]:
    """All strings of a columns() export, by string index."""
    raw = cols["str_pool"].tobytes()
    off = cols["str_off"]
    return [raw[off[k]:off[k + 1]].decode(errors="surrogateescape") for k in range(len(off) - 1)]


def columns_for_graph(g: CsrGraph, area: str = "0") -> Dict[str, np.ndarray]:
    """The AdjacencyDatabases a CSR topology's nodes would originate (one per node, one
    adjacency per directed edge in row order; LinkMonitor.cpp:586-620 fills the same
    fields): ifName ``if_<u>_<v>`` / otherIfName ``if_<v>_<u>`` (the benchmark naming,
    RoutingBenchmarkUtils.cpp:82-101), fe80::/10.x next hops, adjLabel 100001+v, rtt
    and timestamp as LinkMonitor sets them. Requires no parallel links (ifNames would
    collide)."""
    V, E = g.num_nodes, g.num_dir_edges
    pool: List[bytes] = []
    pos = [0]
    offs = [0]

    def put(s: str) -> int:
        b = s.encode()
        pool.append(b)
        pos[0] += len(b)
        offs.append(pos[0])
        return len(offs) - 2

    owner = g.edge_owner()
    cols: Dict[str, np.ndarray] = {
        "node_name": np.array([put(n) for n in g.names] or [0], np.uint32)[:V],
        "area": np.array([put(area) for _ in range(V)] or [0], np.uint32)[:V],
        "node_overloaded": np.asarray(g.node_overloaded, np.uint8),
        "node_label": np.arange(1, V + 1, dtype=np.int32),
        "adj_begin": np.asarray(g.row_ptr, np.uint64),
    }
    other, ifn, oifn, v6, v4 = [], [], [], [], []
    for e in range(E):
        u, v = int(owner[e]), int(g.col[e])
        other.append(put(g.names[v]))
        ifn.append(put(f"if_{g.names[u]}_{g.names[v]}"))
        oifn.append(put(f"if_{g.names[v]}_{g.names[u]}"))
        v6.append(put(f"fe80::{v >> 16:x}:{v & 0xffff:x}"))
        v4.append(put(f"10.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"))
    cols.update({
        "other_node": np.array(other, np.uint32), "if_name": np.array(ifn, np.uint32),
        "other_if_name": np.array(oifn, np.uint32), "nh_v6": np.array(v6, np.uint32),
        "nh_v4": np.array(v4, np.uint32),
        "metric": np.asarray(g.metric, np.uint64).astype(np.int64).astype(np.int32),
        "adj_label": (100001 + np.asarray(g.col, np.int64)).astype(np.int32),
        "adj_overloaded": (np.asarray(g.edge_up) == 0).astype(np.uint8),
        "rtt": np.full(E, 100, np.int32), "timestamp": np.full(E, 1_700_000_000, np.int64),
        "weight": np.ones(E, np.int64),
    })
    cols["str_pool"] = np.frombuffer(b"".join(pool), np.uint8) if pool else np.zeros(0, np.uint8)
    cols["str_off"] = np.array(offs, np.uint64)
    return cols
