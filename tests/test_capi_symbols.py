"""The C-ABI library builds, loads and exports every symbol include/openr_spf.h declares.

No compute call is made here (this container has no GPU); the one behavioural
check is that creating an engine without a device FAILS (no CPU fallback).
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from openr_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "openr_spf.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(openr_spf_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_binding_exports():
    assert declared_functions() == sorted(engine.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = engine.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (openr_spf_\w+)", out.stdout))
    for name in declared_functions():
        assert name in exported, name
        assert hasattr(lib, name)


def test_abi_version_and_limits():
    lib = engine.load_library()
    assert lib.openr_spf_abi_version() == 1
    lim = engine.limits()
    assert lim.max_nh_bits == 65535  # > 256 distinct neighbours: the exact-order kernel
    assert lim.max_nodes >= 10000  # G100 must fit the LDS-resident kernels


def test_library_targets_gfx950():
    data = open(engine.LIB_PATH, "rb").read()
    assert b"gfx950" in data  # offload bundle id of the embedded code object


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(engine.SpfError) as ei:
        engine.SpfEngine()
    assert ei.value.code == engine.ENODEV


def test_adjdb_library_exports_every_declared_symbol():
    """include/openr_adjdb.h (bulk AdjacencyDatabase decode) is exported by libopenr_decision.so."""
    from openr_amd import adjdb

    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "openr_adjdb.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(openr_adjdb_[a-z_0-9]+)\s*\(", text)))
    assert len(declared) >= 12
    lib = adjdb.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", adjdb.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (openr_adjdb_\w+)", out.stdout))
    for name in declared:
        assert name in exported, name
        assert hasattr(lib, name)


def test_topogen_library_exports_every_declared_symbol():
    """include/openr_topogen.h (seeded WAN generator, std::mt19937_64) is exported."""
    from openr_amd import adjdb

    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "openr_topogen.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(openr_topogen_[a-z_0-9]+)\s*\(", text)))
    assert declared == ["openr_topogen_wan"]
    lib = adjdb.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", adjdb.LIB_PATH], capture_output=True, text=True, check=True)
    for name in declared + ["openr_decision_build_id"]:
        assert re.search(r"\bT " + name + r"\b", out.stdout), name
        assert hasattr(lib, name)


def test_routes_library_exports_every_declared_symbol():
    """include/openr_routes.h (batched SpfSolver route build + RibPolicy) is exported."""
    from openr_amd import adjdb

    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "openr_routes.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(openr_routes_[a-z_0-9]+)\s*\(", text)))
    assert declared == ["openr_routes_build"]
    lib = adjdb.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", adjdb.LIB_PATH], capture_output=True, text=True, check=True)
    for name in declared:
        assert re.search(r"\bT " + name + r"\b", out.stdout), name
        assert hasattr(lib, name)


def test_binaries_built_from_this_tree():
    """Build provenance: the engine, the host library and the C++ test binaries embed the
    hash of the sources they were built from (Makefile build_id); it must match this tree
    (openr_amd/provenance.py), so no run can use a library built from other sources."""
    from openr_amd import adjdb
    from openr_amd.provenance import check_build_id

    ids = {
        "engine": engine.load_library().openr_spf_build_id().decode(),
        "host": adjdb.load_library().openr_decision_build_id().decode(),
    }
    for name, bid in ids.items():
        check_build_id(bid, name)
    files = ids["engine"].split()[1:]
    for f in re.findall(r"\$\(CSRC\)/(\w+\.hip)", open(os.path.join(ROOT, "Makefile")).read()):
        assert "openr_amd/csrc/" + f in files, f  # every engine source is covered by the hash
    for binary in ("linkstate_test", "decision_test"):
        p = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", binary), "build-id"], capture_output=True,
                           text=True, timeout=60)
        line = [l for l in p.stdout.splitlines() if l.startswith("build-id: ")]
        assert line, p.stdout + p.stderr
        check_build_id(line[0][len("build-id: "):], binary)


def test_wan_generator_is_deterministic():
    """the config-4 WAN comes from std::mt19937_64(seed)."""
    from openr_amd import topology as T

    a, b = T.wan(1000, 3000, 64, seed=1), T.wan(1000, 3000, 64, seed=1)
    assert a.num_links == 3000 and a.num_dir_edges == 6000 and a.num_nodes == 1000
    assert np.array_equal(a.col, b.col) and np.array_equal(a.metric, b.metric)
    assert int(a.metric.min()) >= 1 and int(a.metric.max()) <= 64
    # ring links first (i, i+1): every node has degree >= 2
    assert int(np.diff(a.row_ptr).min()) >= 2
    c = T.wan(1000, 3000, 64, seed=2)
    assert not np.array_equal(a.col, c.col)
    p = T.wan(256, 768, 64, seed=3, parallel_fraction=0.02)
    assert p.num_links == 768 + 15
