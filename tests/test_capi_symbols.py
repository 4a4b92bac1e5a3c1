"""The C-ABI library builds, loads and exports every symbol include/openr_spf.h declares.

No compute call is made here (this container has no GPU); the one behavioural
check is that creating an engine without a device FAILS (no CPU fallback).
"""
import ctypes
import os
import re
import subprocess

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
    assert lim.max_nh_bits == 256
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
