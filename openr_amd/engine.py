"""ctypes binding of the SPF engine's C-ABI (include/openr_spf.h).

``SpfEngine`` is a thin, typed wrapper: every call goes straight to
libopenr_spf.so and every failure raises ``SpfError`` with the library's
message. There is no Python or CPU implementation of the solve behind it.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

from .provenance import check_build_id

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libopenr_spf.so")

USE_LINK_METRIC = 1
EMIT_TIGHT = 2
EMIT_ORDER = 4
EMIT_LEVELS8 = 8
EMIT_LEVELS16 = 16
STATUS_LEVEL_OVERFLOW = 1

OK, EIO, ENOMEM, ENODEV, EINVAL, E2BIG, ENOTSUP = 0, -5, -12, -19, -22, -7, -95

# Exported symbols of include/openr_spf.h (checked by tests/test_capi_symbols.py).
EXPORTS = (
    "openr_spf_abi_version",
    "openr_spf_build_id",
    "openr_spf_last_error",
    "openr_spf_last_kernels",
    "openr_spf_limits",
    "openr_spf_create",
    "openr_spf_destroy",
    "openr_spf_set_graph",
    "openr_spf_nh_bytes",
    "openr_spf_neighbor_map",
    "openr_spf_solve",
    "openr_spf_solve_order",
    "openr_spf_solve_ignore",
    "openr_spf_solve_device",
    "openr_spf_whatif",
    "openr_spf_whatif_device",
    "openr_spf_whatif_delta",
    "openr_spf_whatif_delta_device",
    "openr_spf_ksp2",
    "openr_spf_ksp2_device",
    "openr_spf_host_alloc",
    "openr_spf_host_free",
    "openr_spf_patch_graph",
    "openr_spf_refresh",
    "openr_spf_refresh_device",
    "openr_spf_get_stats",
    "openr_spf_take_status",
)


class SpfError(RuntimeError):
    def __init__(self, code: int, msg: str) -> None:
        super().__init__(f"openr_spf error {code}: {msg}")
        self.code = code


class SpfGraph(ctypes.Structure):
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


class SpfPatch(ctypes.Structure):
    _fields_ = [
        ("n_edges", ctypes.c_uint32),
        ("edge_ids", ctypes.c_void_p),
        ("metric", ctypes.c_void_p),
        ("n_links", ctypes.c_uint32),
        ("link_ids", ctypes.c_void_p),
        ("link_up", ctypes.c_void_p),
        ("n_nodes", ctypes.c_uint32),
        ("node_ids", ctypes.c_void_p),
        ("node_overloaded", ctypes.c_void_p),
    ]


class WhatifDelta(ctypes.Structure):  # openr_spf_whatif_delta_t
    _fields_ = [
        ("ptr", ctypes.c_void_p),
        ("node", ctypes.c_void_p),
        ("dist", ctypes.c_void_p),
        ("nh", ctypes.c_void_p),
        ("cap", ctypes.c_uint64),
        ("nh_bytes", ctypes.c_uint32),
    ]


class SpfLimits(ctypes.Structure):
    _fields_ = [("max_nodes", ctypes.c_uint32), ("max_nh_bits", ctypes.c_uint32)]


class SpfStats(ctypes.Structure):
    _fields_ = [
        ("spf_runs", ctypes.c_uint64),
        ("batches", ctypes.c_uint64),
        ("last_batch_ms", ctypes.c_double),
        ("last_kernel_ms", ctypes.c_double),
    ]


_lib = None


def load_library():
    """Load libopenr_spf.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()')"
        )
    l = ctypes.CDLL(LIB_PATH)
    vp, u32, P = ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER
    l.openr_spf_abi_version.restype = ctypes.c_int
    l.openr_spf_build_id.restype = ctypes.c_char_p
    check_build_id(l.openr_spf_build_id().decode(), LIB_PATH)
    l.openr_spf_last_error.restype = ctypes.c_char_p
    l.openr_spf_last_kernels.restype = ctypes.c_char_p
    l.openr_spf_limits.argtypes = [P(SpfLimits)]
    l.openr_spf_limits.restype = None
    l.openr_spf_create.argtypes = [vp, ctypes.c_int, P(vp)]
    l.openr_spf_destroy.argtypes = [vp]
    l.openr_spf_destroy.restype = None
    l.openr_spf_set_graph.argtypes = [vp, P(SpfGraph)]
    l.openr_spf_nh_bytes.argtypes = [vp, P(u32)]
    l.openr_spf_neighbor_map.argtypes = [vp, u32, vp, u32, P(u32)]
    l.openr_spf_solve.argtypes = [vp, vp, u32, u32, vp, vp, u32, vp]
    l.openr_spf_solve_order.argtypes = [vp, vp, u32, u32, vp, vp, vp, vp, u32, vp, vp]
    l.openr_spf_solve_ignore.argtypes = [vp, vp, u32, u32, vp, vp, vp, vp, u32, vp]
    l.openr_spf_solve_device.argtypes = [vp, ctypes.c_int, vp, u32, u32, vp, vp, vp, vp, u32, vp, vp]
    l.openr_spf_whatif.argtypes = [vp, vp, u32, vp, u32, u32, vp, P(ctypes.c_uint64)]
    l.openr_spf_whatif_device.argtypes = [vp, ctypes.c_int, vp, u32, vp, u32, u32, vp, vp, P(ctypes.c_uint64)]
    l.openr_spf_whatif_delta.argtypes = [vp, vp, u32, vp, u32, u32, vp, P(WhatifDelta), P(ctypes.c_uint64)]
    l.openr_spf_whatif_delta_device.argtypes = [vp, ctypes.c_int, vp, u32, vp, u32, u32, vp, vp, vp, vp, vp,
                                                ctypes.c_uint64, u32, vp, P(ctypes.c_uint64), P(ctypes.c_uint64)]
    l.openr_spf_ksp2.argtypes = [vp, vp, vp, u32, u32, vp, vp]
    l.openr_spf_ksp2_device.argtypes = [vp, ctypes.c_int, vp, u32, vp, vp, u32, u32, vp, vp, vp]
    l.openr_spf_host_alloc.argtypes = [ctypes.c_size_t, P(vp)]
    l.openr_spf_host_free.argtypes = [vp]
    l.openr_spf_host_free.restype = None
    l.openr_spf_patch_graph.argtypes = [vp, P(SpfPatch)]
    l.openr_spf_refresh.argtypes = [vp, vp, u32, u32, vp, vp, u32, vp, P(u32)]
    l.openr_spf_refresh_device.argtypes = [vp, ctypes.c_int, vp, u32, u32, vp, vp, u32, vp, vp, P(u32)]
    l.openr_spf_get_stats.argtypes = [vp, P(SpfStats)]
    l.openr_spf_take_status.argtypes = [vp, ctypes.c_int, P(u32)]
    for name in EXPORTS:
        if name not in ("openr_spf_last_error", "openr_spf_last_kernels", "openr_spf_limits", "openr_spf_destroy",
                        "openr_spf_build_id", "openr_spf_host_free"):
            getattr(l, name).restype = ctypes.c_int
    _lib = l
    return l


def _check(rc: int) -> None:
    if rc != OK:
        msg = _lib.openr_spf_last_error()
        raise SpfError(rc, msg.decode() if msg else "")


def _p(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _ignore_arrays(ignore: Sequence[Sequence[int]], n: int) -> Tuple[np.ndarray, np.ndarray]:
    """Per-solve ignore sets -> (ignore_ptr[n+1], ignore_links) CSR arrays."""
    ptr = np.zeros(n + 1, dtype=np.uint32)
    ptr[1:] = np.cumsum([len(x) for x in ignore])
    links = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.uint32) for x in ignore])
                                 if ptr[-1] else np.zeros(1, dtype=np.uint32), dtype=np.uint32)
    return ptr, links


class SpfEngine:
    """One engine context (= one LinkState's device-side SPF backend)."""

    def __init__(self, device_ids: Optional[Sequence[int]] = None) -> None:
        self._lib = load_library()
        self._ctx = ctypes.c_void_p()
        if device_ids:
            ids = (ctypes.c_int * len(device_ids))(*device_ids)
            rc = self._lib.openr_spf_create(ctypes.cast(ids, ctypes.c_void_p), len(device_ids), ctypes.byref(self._ctx))
        else:
            rc = self._lib.openr_spf_create(None, 0, ctypes.byref(self._ctx))
        _check(rc)
        self.g = None
        self._gs = None
        self.nh_bytes = 1

    def close(self) -> None:
        if self._ctx:
            self._lib.openr_spf_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def set_graph(self, g) -> None:
        self._gs = g.ctypes_struct(SpfGraph)
        _check(self._lib.openr_spf_set_graph(self._ctx, ctypes.byref(self._gs)))
        self.g = g
        nb = ctypes.c_uint32()
        _check(self._lib.openr_spf_nh_bytes(self._ctx, ctypes.byref(nb)))
        self.nh_bytes = int(nb.value)

    def neighbor_map(self, src: int) -> np.ndarray:
        n = ctypes.c_uint32()
        _check(self._lib.openr_spf_neighbor_map(self._ctx, src, None, 0, ctypes.byref(n)))
        out = np.zeros(max(int(n.value), 1), dtype=np.uint32)
        _check(self._lib.openr_spf_neighbor_map(self._ctx, src, _p(out), out.shape[0], ctypes.byref(n)))
        return out[: int(n.value)]

    def solve(self, sources: Sequence[int], use_link_metric: bool = True, want_nh: bool = True,
              want_tight: bool = False, ignore: Optional[Sequence[Sequence[int]]] = None,
              nh_bytes: Optional[int] = None) -> Tuple[np.ndarray, Optional[np.ndarray], Optional[np.ndarray]]:
        """Batched SPF. Returns (dist[n,V] u64, nh[n,V,nh_bytes] u8 | None, tight[n,ceil(E/64)] u64 | None)."""
        g = self.g
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        n, V = int(src.shape[0]), g.num_nodes
        nb = self.nh_bytes if nh_bytes is None else nh_bytes
        dist = np.empty((n, V), dtype=np.uint64)
        nh = np.empty((n, V, nb), dtype=np.uint8) if want_nh else None
        tw = (g.num_dir_edges + 63) // 64
        tight = np.empty((n, max(tw, 1)), dtype=np.uint64) if want_tight else None
        flags = (USE_LINK_METRIC if use_link_metric else 0) | (EMIT_TIGHT if want_tight else 0)
        if ignore is None:
            rc = self._lib.openr_spf_solve(self._ctx, _p(src), n, flags, _p(dist), _p(nh), nb, _p(tight))
        else:
            ptr, links = _ignore_arrays(ignore, n)
            rc = self._lib.openr_spf_solve_ignore(self._ctx, _p(src), n, flags, _p(ptr), _p(links), _p(dist),
                                                  _p(nh), nb, _p(tight))
        _check(rc)
        return dist, nh, tight

    def solve_order(self, sources: Sequence[int], use_link_metric: bool = True, want_tight: bool = True,
                    ignore: Optional[Sequence[Sequence[int]]] = None
                    ) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray], np.ndarray]:
        """Exact-order solve: (dist, nh, tight | None, order[n,V] u32 pop index, UINT32_MAX unreached)."""
        g = self.g
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        n, V = int(src.shape[0]), g.num_nodes
        dist = np.empty((n, V), dtype=np.uint64)
        nh = np.empty((n, V, self.nh_bytes), dtype=np.uint8)
        tw = (g.num_dir_edges + 63) // 64
        tight = np.empty((n, max(tw, 1)), dtype=np.uint64) if want_tight else None
        order = np.empty((n, V), dtype=np.uint32)
        flags = (USE_LINK_METRIC if use_link_metric else 0) | (EMIT_TIGHT if want_tight else 0)
        ptr, links = _ignore_arrays(ignore, n) if ignore is not None else (None, None)
        _check(self._lib.openr_spf_solve_order(self._ctx, _p(src), n, flags, _p(ptr), _p(links), _p(dist), _p(nh),
                                               self.nh_bytes, _p(tight), _p(order)))
        return dist, nh, tight, order

    def solve_device(self, d_sources: int, n: int, d_dist: int, d_nh: int = 0, nh_bytes: int = 0,
                     use_link_metric: bool = True, stream: int = 0, device_index: int = 0,
                     d_ignore_ptr: int = 0, d_ignore_links: int = 0, d_tight: int = 0, level_bytes: int = 0) -> None:
        """Device-pointer form (ints are raw device addresses, e.g. torch data_ptr()).
        level_bytes = 1 / 2: d_dist receives u8 / u16 level rows instead of u64 distances
        (OPENR_SPF_EMIT_LEVELS8 / 16: uniform-cost graphs on the level BFS family)."""
        flags = (USE_LINK_METRIC if use_link_metric else 0) | (EMIT_TIGHT if d_tight else 0)
        if level_bytes:
            flags |= {1: EMIT_LEVELS8, 2: EMIT_LEVELS16}[level_bytes]
        vp = ctypes.c_void_p
        _check(self._lib.openr_spf_solve_device(self._ctx, device_index, vp(d_sources), n, flags,
                                                vp(d_ignore_ptr or None), vp(d_ignore_links or None), vp(d_dist),
                                                vp(d_nh or None), nh_bytes or self.nh_bytes, vp(d_tight or None),
                                                vp(stream or None)))

    def take_status(self, device_index: int = 0) -> int:
        """OPENR_SPF_STATUS_* bits raised by device-form calls since the last take (waits
        for the device)."""
        st = ctypes.c_uint32()
        _check(self._lib.openr_spf_take_status(self._ctx, device_index, ctypes.byref(st)))
        return int(st.value)

    def whatif(self, links: Sequence[int], sources: Sequence[int], use_link_metric: bool = True
               ) -> Tuple[np.ndarray, int]:
        """Per-link-failure sweep: (changed[n_links, n_sources] u32, SPFs run)."""
        lk = np.ascontiguousarray(links, dtype=np.uint32)
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        changed = np.zeros((lk.shape[0], src.shape[0]), dtype=np.uint32)
        solved = ctypes.c_uint64()
        flags = USE_LINK_METRIC if use_link_metric else 0
        _check(self._lib.openr_spf_whatif(self._ctx, _p(lk), lk.shape[0], _p(src), src.shape[0], flags,
                                          _p(changed), ctypes.byref(solved)))
        return changed, int(solved.value)

    def whatif_device(self, d_links: int, n_links: int, d_sources: int, n_sources: int, d_changed: int,
                      use_link_metric: bool = True, stream: int = 0, device_index: int = 0) -> int:
        """Device-pointer form; returns the number of SPFs run."""
        vp = ctypes.c_void_p
        solved = ctypes.c_uint64()
        flags = USE_LINK_METRIC if use_link_metric else 0
        _check(self._lib.openr_spf_whatif_device(self._ctx, device_index, vp(d_links), n_links, vp(d_sources),
                                                 n_sources, flags, vp(d_changed), vp(stream or None),
                                                 ctypes.byref(solved)))
        return int(solved.value)

    def whatif_delta(self, links: Sequence[int], sources: Sequence[int], use_link_metric: bool = True,
                     cap: Optional[int] = None, nh_bytes: Optional[int] = None):
        """Per-link-failure sweep with each unit's delta (openr_spf_whatif_delta):
        (changed[n_links, n_sources] u32, ptr[n_units + 1] u64, node u32, dist u64,
        nh[entries, nh_bytes] u8, SPFs run). Unit u = i * n_sources + j owns entries
        [ptr[u], ptr[u + 1]), node ids ascending. cap None: sized from a count-only pass."""
        lk = np.ascontiguousarray(links, dtype=np.uint32)
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        nb = nh_bytes if nh_bytes is not None else self.nh_bytes
        if cap is None:
            changed, _ = self.whatif(lk, src, use_link_metric)
            cap = int(changed.sum(dtype=np.uint64))
        changed = np.zeros((lk.shape[0], src.shape[0]), dtype=np.uint32)
        ptr = np.zeros(lk.shape[0] * src.shape[0] + 1, dtype=np.uint64)
        node = np.zeros(max(cap, 1), dtype=np.uint32)
        dist = np.zeros(max(cap, 1), dtype=np.uint64)
        nh = np.zeros((max(cap, 1), nb), dtype=np.uint8)
        d = WhatifDelta(_p(ptr), _p(node), _p(dist), _p(nh), cap, nb)
        solved = ctypes.c_uint64()
        flags = USE_LINK_METRIC if use_link_metric else 0
        _check(self._lib.openr_spf_whatif_delta(self._ctx, _p(lk), lk.shape[0], _p(src), src.shape[0], flags,
                                                _p(changed), ctypes.byref(d), ctypes.byref(solved)))
        n = int(ptr[-1])
        return changed, ptr, node[:n], dist[:n], nh[:n], int(solved.value)

    def whatif_delta_device(self, d_links: int, n_links: int, d_sources: int, n_sources: int, d_changed: int,
                            d_ptr: int, d_node: int, d_dist: int, d_nh: int, cap: int, nh_bytes: int,
                            use_link_metric: bool = True, stream: int = 0, device_index: int = 0,
                            allow_overflow: bool = False) -> Tuple[int, int]:
        """Device-pointer form: (total entries, SPFs run). d_ptr [n_units + 1] u64 CSR; unit
        u's entries are [ptr[u], ptr[u + 1]) in the repair's order."""
        vp = ctypes.c_void_p
        total = ctypes.c_uint64()
        solved = ctypes.c_uint64()
        flags = USE_LINK_METRIC if use_link_metric else 0
        rc = self._lib.openr_spf_whatif_delta_device(self._ctx, device_index, vp(d_links), n_links, vp(d_sources),
                                                     n_sources, flags, vp(d_changed), vp(d_ptr), vp(d_node or None),
                                                     vp(d_dist or None), vp(d_nh or None), cap, nh_bytes,
                                                     vp(stream or None), ctypes.byref(total), ctypes.byref(solved))
        if not (allow_overflow and rc == E2BIG):
            _check(rc)
        return int(total.value), int(solved.value)

    def ksp2_tokens(self, src: Sequence[int], dst: Sequence[int], tok_cap: int = 256,
                    allow_overflow: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        """getKthPaths(s, d, 1) and (.., 2) per pair as raw token rows [n, tok_cap] u32."""
        s_ = np.ascontiguousarray(src, dtype=np.uint32)
        d_ = np.ascontiguousarray(dst, dtype=np.uint32)
        n = int(s_.shape[0])
        t1 = np.zeros((n, tok_cap), dtype=np.uint32)
        t2 = np.zeros((n, tok_cap), dtype=np.uint32)
        rc = self._lib.openr_spf_ksp2(self._ctx, _p(s_), _p(d_), n, tok_cap, _p(t1), _p(t2))
        if not (allow_overflow and rc == E2BIG):
            _check(rc)
        return t1, t2

    def ksp2(self, src: Sequence[int], dst: Sequence[int], tok_cap: int = 256):
        """[(paths_k1, paths_k2)] per pair; a path = list of directed edge ids, src -> dest."""
        t1, t2 = self.ksp2_tokens(src, dst, tok_cap)
        return [(decode_paths(t1[i]), decode_paths(t2[i])) for i in range(t1.shape[0])]

    def ksp2_device(self, d_sources: int, n_sources: int, d_pair_row: int, d_pair_dst: int, n_pairs: int,
                    tok_cap: int, d_tok1: int, d_tok2: int, stream: int = 0, device_index: int = 0) -> None:
        vp = ctypes.c_void_p
        _check(self._lib.openr_spf_ksp2_device(self._ctx, device_index, vp(d_sources), n_sources, vp(d_pair_row),
                                               vp(d_pair_dst), n_pairs, tok_cap, vp(d_tok1), vp(d_tok2),
                                               vp(stream or None)))

    def patch(self, edges: Sequence[int] = (), metrics: Sequence[int] = (), links: Sequence[int] = (),
              link_up: Sequence[int] = (), nodes: Sequence[int] = (), node_overloaded: Sequence[int] = (),
              track: bool = True) -> None:
        """Attribute-only mirror update (openr_spf_patch_graph); with ``track`` also applies it
        to ``self.g`` (a patched copy of the host graph)."""
        e = np.ascontiguousarray(edges, dtype=np.uint32)
        m = np.ascontiguousarray(metrics, dtype=np.uint64)
        lk = np.ascontiguousarray(links, dtype=np.uint32)
        lu = np.ascontiguousarray(link_up, dtype=np.uint8)
        nd = np.ascontiguousarray(nodes, dtype=np.uint32)
        no = np.ascontiguousarray(node_overloaded, dtype=np.uint8)
        if e.shape != m.shape or lk.shape != lu.shape or nd.shape != no.shape:
            raise ValueError("patch id / value arrays differ in length")
        p = SpfPatch(int(e.shape[0]), _p(e), _p(m), int(lk.shape[0]), _p(lk), _p(lu), int(nd.shape[0]), _p(nd),
                     _p(no))
        _check(self._lib.openr_spf_patch_graph(self._ctx, ctypes.byref(p)))
        if track:
            self.g = self.g.patched(e, m, lk, lu, nd, no)

    def refresh(self, sources: Sequence[int], dist: np.ndarray, nh: Optional[np.ndarray] = None,
                tight: Optional[np.ndarray] = None, use_link_metric: bool = True) -> int:
        """Bring rows solved before the last patch up to date in place; returns rows re-solved."""
        src = np.ascontiguousarray(sources, dtype=np.uint32)
        for a in (dist, nh, tight):
            if a is not None and not a.flags.c_contiguous:
                raise ValueError("rows must be C-contiguous")
        nb = nh.shape[2] if nh is not None else self.nh_bytes
        flags = (USE_LINK_METRIC if use_link_metric else 0) | (EMIT_TIGHT if tight is not None else 0)
        out = ctypes.c_uint32()
        _check(self._lib.openr_spf_refresh(self._ctx, _p(src), int(src.shape[0]), flags, _p(dist), _p(nh), nb,
                                           _p(tight), ctypes.byref(out)))
        return int(out.value)

    def refresh_device(self, d_sources: int, n: int, d_dist: int, d_nh: int = 0, nh_bytes: int = 0,
                       use_link_metric: bool = True, stream: int = 0, device_index: int = 0,
                       d_tight: int = 0) -> int:
        vp = ctypes.c_void_p
        flags = (USE_LINK_METRIC if use_link_metric else 0) | (EMIT_TIGHT if d_tight else 0)
        out = ctypes.c_uint32()
        _check(self._lib.openr_spf_refresh_device(self._ctx, device_index, vp(d_sources), n, flags, vp(d_dist),
                                                  vp(d_nh or None), nh_bytes or self.nh_bytes, vp(d_tight or None),
                                                  vp(stream or None), ctypes.byref(out)))
        return int(out.value)

    def last_kernels(self) -> list:
        """Kernels this thread's last solve call enqueued (openr_spf_last_kernels)."""
        return [k for k in self._lib.openr_spf_last_kernels().decode().split(";") if k]

    def stats(self) -> SpfStats:
        s = SpfStats()
        _check(self._lib.openr_spf_get_stats(self._ctx, ctypes.byref(s)))
        return s


def decode_paths(tok: np.ndarray):
    """Token row [n_paths, len_0, e.., len_1, e.., ...] -> list of edge-id lists."""
    n = int(tok[0])
    if n == 0xFFFFFFFF:
        raise SpfError(E2BIG, "pair overflowed its token row")
    out, pos = [], 1
    for _ in range(n):
        ln = int(tok[pos])
        out.append(tok[pos + 1 : pos + 1 + ln].astype(np.int64).tolist())
        pos += 1 + ln
    return out


def limits() -> SpfLimits:
    l = load_library()
    s = SpfLimits()
    l.openr_spf_limits(ctypes.byref(s))
    return s
