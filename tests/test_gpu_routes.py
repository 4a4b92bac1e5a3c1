"""BASELINE config 4's route half: UCMP-weighted route DBs of the WAN built through the
C-ABI (include/openr_routes.h): SPF on the GPU engine, SpfSolver route build and RibPolicy
set_weight on the host. Next-hop-for-next-hop parity against routes rebuilt from ORACLE
SPF runs is tests/cpp/decision_test.cpp WanUcmpRoutes_vs_Oracle_* (run by
test_cpp_host.py::test_decision_mirror_gpu); this checks the boundary and the policy."""
import numpy as np
import pytest

from openr_amd import adjdb
from openr_amd import topology as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wan_builder():
    g = T.wan(1000, 3000, 64, seed=1)
    batch = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g))
    rb = adjdb.RouteBuilder(batch, "0")
    yield g, rb
    rb.close()
    batch.close()


def test_wan_ucmp_route_build(wan_builder):
    g, rb = wan_builder
    names = rb.names()
    V = len(names)
    assert V == 1000
    w = adjdb.wan_ucmp_weights(names)
    ids = np.arange(0, V, 7)
    plain = rb.build(ids, 0)
    ucmp = rb.build(ids, adjdb.ROUTES_UCMP, 1, w)
    assert plain.unicast_routes == ucmp.unicast_routes == len(ids) * (V - 1)  # connected WAN
    assert plain.nexthops == ucmp.nexthops  # weights, never drops (all weights > 0)
    assert plain.weighted_nexthops == 0 and ucmp.weighted_nexthops > 0
    assert plain.checksum != ucmp.checksum
    again = rb.build(ids, adjdb.ROUTES_UCMP, 1, w)
    assert again.checksum == ucmp.checksum  # deterministic
    lfa = rb.build(ids[:20], adjdb.ROUTES_LFA | adjdb.ROUTES_UCMP, 1, w)
    sp = rb.build(ids[:20], adjdb.ROUTES_UCMP, 1, w)
    assert lfa.nexthops > sp.nexthops  # loop-free alternates on the WAN


def test_route_build_errors(wan_builder):
    _, rb = wan_builder
    with pytest.raises(adjdb.AdjDbError):
        rb.build([10**6])
    with pytest.raises(ValueError):
        rb.build([0], adjdb.ROUTES_UCMP, 1, np.zeros(3, np.int32))
    st = rb.build([])
    assert st.unicast_routes == 0
