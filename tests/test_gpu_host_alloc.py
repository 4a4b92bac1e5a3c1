"""openr_spf_host_alloc / openr_spf_host_free (include/openr_spf.h): page-locked host
buffers for the batch calls' host outputs (LinkState::prefetchKthPaths' token rows), and
an openr_spf_ksp2 call writing into them gives the same tokens as pageable buffers."""
import ctypes

import numpy as np
import pytest

from openr_amd import engine
from openr_amd import topology as T

pytestmark = pytest.mark.gpu


def test_host_alloc_roundtrip_and_errors():
    lib = engine.load_library()
    p = ctypes.c_void_p()
    assert lib.openr_spf_host_alloc(1 << 20, ctypes.byref(p)) == engine.OK and p.value
    buf = (ctypes.c_uint32 * (1 << 18)).from_address(p.value)
    buf[0], buf[(1 << 18) - 1] = 7, 9
    assert buf[0] == 7 and buf[(1 << 18) - 1] == 9
    lib.openr_spf_host_free(p)
    lib.openr_spf_host_free(None)  # no-op
    assert lib.openr_spf_host_alloc(16, None) == engine.EINVAL


def test_ksp2_tokens_into_pinned_buffers():
    lib = engine.load_library()
    eng = engine.SpfEngine([0])
    g = T.wan(300, 900, 10, seed=3)
    eng.set_graph(g)
    n, cap = 512, 256
    rng = np.random.default_rng(5)
    src = rng.integers(0, g.num_nodes, n).astype(np.uint32)
    dst = rng.integers(0, g.num_nodes, n).astype(np.uint32)
    ref1, ref2 = eng.ksp2_tokens(src, dst, cap)
    ptrs = []
    for _ in range(2):
        p = ctypes.c_void_p()
        assert lib.openr_spf_host_alloc(n * cap * 4, ctypes.byref(p)) == engine.OK
        ptrs.append(p)
    t1 = np.ctypeslib.as_array((ctypes.c_uint32 * (n * cap)).from_address(ptrs[0].value)).reshape(n, cap)
    t2 = np.ctypeslib.as_array((ctypes.c_uint32 * (n * cap)).from_address(ptrs[1].value)).reshape(n, cap)
    t1[:, 0] = t2[:, 0] = 0xFFFFFFFF
    rc = lib.openr_spf_ksp2(eng._ctx, src.ctypes.data, dst.ctypes.data, n, cap, ptrs[0], ptrs[1])
    assert rc in (engine.OK, engine.E2BIG)
    for i in range(n):
        for a, b in ((t1[i], ref1[i]), (t2[i], ref2[i])):
            if b[0] == 0xFFFFFFFF:
                continue
            m = 1
            for _ in range(int(b[0])):
                m += 1 + int(b[m])
            np.testing.assert_array_equal(a[:m], b[:m])
    for p in ptrs:
        lib.openr_spf_host_free(p)
    eng.close()
