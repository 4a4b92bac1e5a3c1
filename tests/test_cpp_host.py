"""Runs the C++ host-mirror tests (tests/cpp/linkstate_test.cpp, decision_test.cpp).

cpu group: HoldableValue / Link / LinkState topology semantics and the CSR mirror
(LinkStateTest.cpp:22-242); gpu group: SPF, KSP, hop counts, spf_runs counters and
oracle parity through the C-ABI engine.
"""
import os
import subprocess

import pytest

from openr_amd.provenance import check_build_id

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "linkstate_test")
DEC_BIN = os.path.join(ROOT, "tests", "cpp", "build", "decision_test")


def run(group, binary=BIN):
    assert os.path.exists(binary), "build first: make"
    p = subprocess.run([binary, group], capture_output=True, text=True, timeout=600)
    print(p.stdout)
    print(p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    # provenance: the binary and the libraries it loaded were built from this tree
    for key in ("build-id: ", "engine-build-id: ", "host-build-id: "):
        line = [l for l in p.stdout.splitlines() if l.startswith(key)]
        assert line, key
        check_build_id(line[0][len(key):], f"{os.path.basename(binary)} {key.strip(': ')}")
    return p.stdout


def test_host_mirror_cpu():
    out = run("cpu")
    assert "0 failures" in out
    # pathLinks order among parallel links = linksFromNode order; the DecisionTest
    # adj12_2 expectation needs 2/2 before 2/1 on node 1.
    line = [l for l in out.splitlines() if "linksFromNode(1) order" in l][0]
    assert line.index("2/2") < line.index("2/1")


@pytest.mark.gpu
def test_host_mirror_gpu():
    out = run("gpu")
    assert "0 failures" in out


def test_decision_mirror_cpu():
    """SpfSolver / RibPolicy host logic without SPF (best-route selection, RibPolicy,
    unknown node)."""
    assert "0 failures" in run("cpu", DEC_BIN)


@pytest.mark.gpu
def test_decision_mirror_gpu():
    """Route builds transcribed from DecisionTest.cpp (ring SP / LFA / KSP2, MPLS label
    routes, grid route counts 2n^4 + 3n^2 - 4n) over engine SPF results."""
    assert "0 failures" in run("gpu", DEC_BIN)
