"""ctypes wrapper over liboracle_spf.so — CPU ORACLE, test infrastructure only.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
use this module, and only as the checker / the timed CPU port. It restates
/root/reference/openr/decision/LinkState.cpp:762-882 (see spf_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_spf.so")
U64_MAX = 0xFFFFFFFFFFFFFFFF


class OracleGraph(ctypes.Structure):
    _fields_ = [
        ("num_nodes", ctypes.c_uint32),
        ("num_dir_edges", ctypes.c_uint32),
        ("num_links", ctypes.c_uint32),
        ("row_ptr", ctypes.POINTER(ctypes.c_uint32)),
        ("col", ctypes.POINTER(ctypes.c_uint32)),
        ("metric", ctypes.POINTER(ctypes.c_uint64)),
        ("link_id", ctypes.POINTER(ctypes.c_uint32)),
        ("edge_up", ctypes.POINTER(ctypes.c_uint8)),
        ("node_overloaded", ctypes.POINTER(ctypes.c_uint8)),
        ("name_rank", ctypes.POINTER(ctypes.c_uint32)),
    ]


_lib = None


def default_threads() -> int:
    """Host threads for the batch drivers: the process's CPU share, at most 16."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def build() -> None:
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        l = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        l.oracle_run_spf.restype = ctypes.c_int64
        l.oracle_run_spf.argtypes = [P(OracleGraph), ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
        l.oracle_kth_paths.restype = ctypes.c_int64
        l.oracle_kth_paths.argtypes = [P(OracleGraph), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        l.oracle_all_sources.restype = ctypes.c_int
        l.oracle_all_sources.argtypes = [P(OracleGraph), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        l.oracle_ksp2_batch.restype = ctypes.c_int
        l.oracle_ksp2_batch.argtypes = [P(OracleGraph), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        l.oracle_whatif.restype = ctypes.c_int
        l.oracle_whatif.argtypes = [P(OracleGraph), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        l.oracle_whatif_delta_digest.restype = ctypes.c_int
        l.oracle_whatif_delta_digest.argtypes = [P(OracleGraph), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                 ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_uint32, ctypes.c_int]
        l.faithful_all_sources.restype = ctypes.c_int
        l.faithful_all_sources.argtypes = [P(OracleGraph), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double)]
        l.oracle_num_distinct_neighbors.restype = ctypes.c_uint32
        l.oracle_num_distinct_neighbors.argtypes = [P(OracleGraph), ctypes.c_uint32]
        _lib = l
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class SpfRun:
    dist: np.ndarray  # u64 [V]
    nh: np.ndarray  # u8 [V, nh_bytes]
    order: np.ndarray  # settle order (u32)
    pl_ptr: np.ndarray
    pl_edge: np.ndarray

    def reachable(self) -> np.ndarray:
        return self.dist != np.uint64(U64_MAX)


class Oracle:
    """Reference-faithful SPF/KSP over a CSR mirror (topology.CsrGraph)."""

    def __init__(self, g) -> None:
        self.g = g
        self._s = g.ctypes_struct(OracleGraph)
        self.nh_bytes = g.nh_bytes()

    def run_spf(self, src: int, use_link_metric: bool = True,
                ignore_links: Optional[Sequence[int]] = None) -> SpfRun:
        g = self.g
        V, E = g.num_nodes, g.num_dir_edges
        ign = None
        if ignore_links:
            ign = np.zeros((g.num_links + 63) // 64 + 1, dtype=np.uint64)
            for l in ignore_links:
                ign[l >> 6] |= np.uint64(1 << (l & 63))
        dist = np.empty(V, dtype=np.uint64)
        nh = np.zeros((V, self.nh_bytes), dtype=np.uint8)
        order = np.zeros(V, dtype=np.uint32)
        pl_ptr = np.zeros(V + 1, dtype=np.uint32)
        pl_edge = np.zeros(max(E, 1), dtype=np.uint32)
        n = lib().oracle_run_spf(ctypes.byref(self._s), src, int(use_link_metric), _ptr(ign), _ptr(dist),
                                 _ptr(nh), self.nh_bytes, _ptr(order), _ptr(pl_ptr), _ptr(pl_edge))
        if n < 0:
            raise RuntimeError(f"oracle_run_spf failed ({n})")
        return SpfRun(dist, nh, order[:n].copy(), pl_ptr, pl_edge[: pl_ptr[V]].copy())

    def kth_paths(self, src: int, dest: int, k: int) -> List[List[int]]:
        g = self.g
        E = max(g.num_dir_edges, 1)
        pptr = np.zeros(E + 2, dtype=np.uint32)
        edges = np.zeros(E + 1, dtype=np.uint32)
        n = lib().oracle_kth_paths(ctypes.byref(self._s), src, dest, k, _ptr(pptr), E + 1, _ptr(edges), E + 1)
        if n < 0:
            raise RuntimeError("oracle_kth_paths failed")
        return [edges[pptr[i] : pptr[i + 1]].tolist() for i in range(n)]

    def all_sources(self, sources: Sequence[int], use_link_metric: bool = True, nthreads: int = 1,
                    want_dist: bool = True, want_nh: bool = True):
        g = self.g
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        n = src.shape[0]
        dist = np.empty((n, g.num_nodes), dtype=np.uint64) if want_dist else None
        nh = np.zeros((n, g.num_nodes, self.nh_bytes), dtype=np.uint8) if want_nh else None
        rc = lib().oracle_all_sources(ctypes.byref(self._s), _ptr(src), n, int(use_link_metric), _ptr(dist),
                                      _ptr(nh), self.nh_bytes, nthreads)
        if rc != 0:
            raise RuntimeError("oracle_all_sources failed")
        return dist, nh

    def faithful_all_sources(self, sources: Sequence[int], use_link_metric: bool = True, nthreads: int = 1,
                             want_dist: bool = False, want_nh: bool = False):
        """runSpf per source with the reference's data structures (spf_faithful.cpp: string
        keys, shared_ptr heap, unordered_set next hops): the faithful-cost CPU baseline.
        Returns (dist | None, nh | None, seconds of solving)."""
        g = self.g
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        n, V = src.shape[0], g.num_nodes
        raw = [nm.encode() for nm in g.names]
        pool = np.frombuffer(b"".join(raw) or b"\0", dtype=np.uint8)
        off = np.zeros(V + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in raw])
        dist = np.empty((n, V), dtype=np.uint64) if want_dist else None
        nh = np.zeros((n, V, self.nh_bytes), dtype=np.uint8) if want_nh else None
        secs = ctypes.c_double()
        rc = lib().faithful_all_sources(ctypes.byref(self._s), _ptr(pool), _ptr(off), _ptr(src), n,
                                        int(use_link_metric), nthreads, _ptr(dist), _ptr(nh), self.nh_bytes,
                                        ctypes.byref(secs))
        if rc != 0:
            raise RuntimeError("faithful_all_sources failed")
        return dist, nh, secs.value

    def ksp2_tokens(self, src: Sequence[int], dst: Sequence[int], tok_cap: int = 256, nthreads: int = 0):
        """getKthPaths(s, d, 1) and (.., 2) per pair as token rows [n, tok_cap] u32 (the
        openr_spf_ksp2 layout), on `nthreads` host threads (0 = up to 16)."""
        s_ = np.ascontiguousarray(src, dtype=np.uint32)
        d_ = np.ascontiguousarray(dst, dtype=np.uint32)
        n = int(s_.shape[0])
        t1 = np.zeros((n, tok_cap), dtype=np.uint32)
        t2 = np.zeros((n, tok_cap), dtype=np.uint32)
        rc = lib().oracle_ksp2_batch(ctypes.byref(self._s), _ptr(s_), _ptr(d_), n, tok_cap, _ptr(t1), _ptr(t2),
                                     nthreads or default_threads())
        if rc != 0:
            raise RuntimeError("oracle_ksp2_batch failed")
        return t1, t2

    def whatif(self, links: Sequence[int], sources: Sequence[int], use_link_metric: bool = True,
               nthreads: int = 0) -> np.ndarray:
        """changed[n_links, n_sources] u32: nodes whose dist or next-hop set differ between
        runSpf(s, {link}) and runSpf(s)."""
        lk = np.ascontiguousarray(links, dtype=np.uint32)
        sr = np.ascontiguousarray(sources, dtype=np.uint32)
        out = np.zeros((lk.shape[0], sr.shape[0]), dtype=np.uint32)
        rc = lib().oracle_whatif(ctypes.byref(self._s), _ptr(lk), lk.shape[0], _ptr(sr), sr.shape[0],
                                 int(use_link_metric), _ptr(out), nthreads or default_threads())
        if rc != 0:
            raise RuntimeError("oracle_whatif failed")
        return out

    def whatif_delta_digest(self, links: Sequence[int], sources: Sequence[int], nh_bytes: int,
                            use_link_metric: bool = True, nthreads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
        """(changed[n_links, n_sources] u32, digest[n_links, n_sources] u64): each unit's
        changed nodes hashed with their new distance and next-hop bytes (delta_digest()
        computes the same from a delta)."""
        lk = np.ascontiguousarray(links, dtype=np.uint32)
        sr = np.ascontiguousarray(sources, dtype=np.uint32)
        out = np.zeros((lk.shape[0], sr.shape[0]), dtype=np.uint32)
        dig = np.zeros((lk.shape[0], sr.shape[0]), dtype=np.uint64)
        rc = lib().oracle_whatif_delta_digest(ctypes.byref(self._s), _ptr(lk), lk.shape[0], _ptr(sr), sr.shape[0],
                                              int(use_link_metric), _ptr(out), _ptr(dig), nh_bytes,
                                              nthreads or default_threads())
        if rc != 0:
            raise RuntimeError("oracle_whatif_delta_digest failed")
        return out, dig

    # --- helpers mirroring the reference's SpfResult view -------------------
    def next_hop_names(self, src: int, run: SpfRun, v: int) -> Set[str]:
        nbrs = self.g.distinct_neighbors(src)
        out = set()
        for i, nb in enumerate(nbrs):
            if (run.nh[v, i >> 3] >> (i & 7)) & 1:
                out.add(self.g.names[nb])
        return out

    def spf_result(self, src: int, use_link_metric: bool = True,
                   ignore_links: Optional[Sequence[int]] = None) -> Dict[str, Dict]:
        """SpfResult-like dict: name -> {metric, nextHops, pathLinks[(link, prevName)]}."""
        run = self.run_spf(src, use_link_metric, ignore_links)
        owner = self.g.edge_owner()
        res = {}
        for v in np.nonzero(run.reachable())[0].tolist():
            pls = run.pl_edge[run.pl_ptr[v] : run.pl_ptr[v + 1]].tolist()
            res[self.g.names[v]] = {
                "metric": int(run.dist[v]),
                "nextHops": self.next_hop_names(src, run, v),
                "pathLinks": [(int(self.g.link_id[e]), self.g.names[int(owner[e])]) for e in pls],
            }
        return res


_M1, _M2, _G = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB), np.uint64(0x9E3779B97F4A7C15)


def _mix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + _G
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        return x ^ (x >> np.uint64(31))


def delta_digest(ptr: np.ndarray, node: np.ndarray, dist: np.ndarray, nh: np.ndarray) -> np.ndarray:
    """Per-unit digest of a CSR delta (openr_spf_whatif_delta's host form), as
    oracle_whatif_delta_digest computes it: sum mod 2^64 of the entries' hashes."""
    n, nb = nh.shape
    pad = np.zeros((n, (nb + 7) // 8 * 8), dtype=np.uint8)
    pad[:, :nb] = nh
    chunks = pad.view(np.uint64).reshape(n, -1)
    h = _mix64(node.astype(np.uint64) ^ np.uint64(0xD1B54A32D192ED03))
    h = _mix64(h ^ dist.astype(np.uint64))
    for k in range(chunks.shape[1]):
        h = _mix64(h ^ chunks[:, k])
    units = ptr.shape[0] - 1
    out = np.zeros(units, dtype=np.uint64)
    cnt = np.diff(ptr.astype(np.int64))
    nz = np.nonzero(cnt)[0]
    if len(nz):
        with np.errstate(over="ignore"):
            out[nz] = np.add.reduceat(h, ptr[:-1][nz].astype(np.int64))
    return out
