// decision_test.cpp — tests of the C++ host mirror of openr::SpfSolver / RibPolicy
// (openr_amd/csrc/host/Decision.{h,cpp}).
//
// Transcribes route expectations of /root/reference/openr/decision/tests/DecisionTest.cpp
// (file:line per test) and RibPolicy / best-route-selection semantics. SPF results come
// from the engine, so route-building tests are in the gpu group.
//   decision_test cpu | gpu | all
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <cstdlib>
#include <thread>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/openr_topogen.h"
#include "../../openr_amd/csrc/host/Decision.h"
#include "../../openr_amd/csrc/host/HostParallel.h"
#include "../../oracle/spf_oracle.h"
#include "harness.h"

using namespace openr;
using thrift::MplsActionCode;

namespace {

const std::string kDefaultArea = "0";

// Util.cpp:756 createAdjacency(node, if, remoteIf, nhV6, nhV4, metric, adjLabel)
thrift::Adjacency createAdjacency(const std::string& node, const std::string& ifName, const std::string& otherIf,
                                  const std::string& nhV6, const std::string& nhV4, int32_t metric,
                                  int32_t adjLabel) {
  thrift::Adjacency a;
  a.otherNodeName = node;
  a.ifName = ifName;
  a.otherIfName = otherIf;
  a.nextHopV6.addr = nhV6;
  a.nextHopV4.addr = nhV4;
  a.metric = metric;
  a.adjLabel = adjLabel;
  a.rtt = metric * 100;
  return a;
}

thrift::AdjacencyDatabase createAdjDb(const std::string& node, const std::vector<thrift::Adjacency>& adjs,
                                      int32_t nodeLabel, bool overload = false) {
  thrift::AdjacencyDatabase db;
  db.thisNodeName = node;
  db.isOverloaded = overload;
  db.adjacencies = adjs;
  db.nodeLabel = nodeLabel;
  db.area = kDefaultArea;
  return db;
}

// DecisionTest.cpp:47-86
const auto adj12 = createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 100002);
const auto adj13 = createAdjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 100003);
const auto adj21 = createAdjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 100001);
const auto adj23 = createAdjacency("3", "2/3", "3/2", "fe80::3", "192.168.0.3", 10, 100003);
const auto adj24 = createAdjacency("4", "2/4", "4/2", "fe80::4", "192.168.0.4", 10, 100004);
const auto adj31 = createAdjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 100001);
const auto adj32 = createAdjacency("2", "3/2", "2/3", "fe80::2", "192.168.0.2", 10, 100002);
const auto adj34 = createAdjacency("4", "3/4", "4/3", "fe80::4", "192.168.0.4", 10, 100004);
const auto adj42 = createAdjacency("2", "4/2", "2/4", "fe80::2", "192.168.0.2", 10, 100002);
const auto adj43 = createAdjacency("3", "4/3", "3/4", "fe80::3", "192.168.0.3", 10, 100003);

thrift::IpPrefix pfx(const std::string& s) {
  const auto slash = s.find('/');
  return thrift::IpPrefix{s.substr(0, slash), (int16_t)std::atoi(s.c_str() + slash + 1)};
}

// DecisionTest.cpp:89-98
const auto addr1 = pfx("::ffff:10.1.1.1/128");
const auto addr2 = pfx("::ffff:10.2.2.2/128");
const auto addr3 = pfx("::ffff:10.3.3.3/128");
const auto addr4 = pfx("::ffff:10.4.4.4/128");
const auto addr1V4 = pfx("10.1.1.1/32");
const auto addr2V4 = pfx("10.2.2.2/32");
const auto addr3V4 = pfx("10.3.3.3/32");
const auto addr4V4 = pfx("10.4.4.4/32");

thrift::PrefixEntry createPrefixEntry(const thrift::IpPrefix& p, bool ksp2 = false) {
  thrift::PrefixEntry e;
  e.prefix = p;
  if (ksp2) {  // createPrefixDbWithKspfAlgo (DecisionTest.cpp:160-200)
    e.forwardingType = thrift::PrefixForwardingType::SR_MPLS;
    e.forwardingAlgorithm = thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
  }
  return e;
}

thrift::MplsAction mpls(MplsActionCode c, std::optional<int32_t> swap = std::nullopt,
                        std::optional<std::vector<int32_t>> push = std::nullopt) {
  return createMplsAction(c, swap, push);
}

// DecisionTest.cpp:203-215
thrift::NextHopThrift nhFromAdj(const thrift::Adjacency& adj, bool isV4, int32_t metric,
                                std::optional<thrift::MplsAction> act = std::nullopt) {
  return createNextHop(isV4 ? adj.nextHopV4 : adj.nextHopV6, adj.ifName, metric, std::move(act), kDefaultArea,
                       adj.otherNodeName);
}

using RouteMap = std::map<std::pair<std::string, std::string>, NextHopSet>;

// DecisionTest.cpp:249-290 fillRouteMap / getRouteMap (the batched form: one prefetch)
RouteMap getRouteMap(SpfSolver& solver, const std::vector<std::string>& nodes,
                     std::unordered_map<std::string, LinkState> const& als, PrefixState const& ps) {
  RouteMap m;
  auto dbs = solver.buildRouteDbs(nodes, als, ps);
  for (size_t i = 0; i < nodes.size(); ++i) {
    if (!dbs[i]) continue;
    for (auto const& [p, e] : dbs[i]->unicastRoutes)
      for (auto const& nh : e.nexthops) m[{nodes[i], p.toString()}].insert(nh);
    for (auto const& [l, e] : dbs[i]->mplsRoutes)
      for (auto const& nh : e.nexthops) m[{nodes[i], std::to_string(l)}].insert(nh);
  }
  return m;
}

const thrift::NextHopThrift labelPopNextHop = [] {
  thrift::NextHopThrift nh;
  nh.address.addr = "::";
  nh.mplsAction = mpls(MplsActionCode::POP_AND_LOOKUP);
  nh.area = kDefaultArea;
  return nh;
}();

// DecisionTest.cpp:343-363
void validateAdjLabelRoutes(RouteMap const& m, const std::string& node, const std::vector<thrift::Adjacency>& adjs) {
  for (auto const& adj : adjs) {
    auto it = m.find({node, std::to_string(adj.adjLabel)});
    EXPECT_TRUE(it != m.end());
    if (it != m.end()) EXPECT_EQ(it->second, NextHopSet({nhFromAdj(adj, false, adj.metric, mpls(MplsActionCode::PHP))}));
  }
}
void validatePopLabelRoute(RouteMap const& m, const std::string& node, int32_t label) {
  auto it = m.find({node, std::to_string(label)});
  EXPECT_TRUE(it != m.end());
  if (it != m.end()) EXPECT_EQ(it->second, NextHopSet({labelPopNextHop}));
}

NextHopSet at(RouteMap& m, const std::string& node, const thrift::IpPrefix& p) { return m[{node, p.toString()}]; }
NextHopSet at(RouteMap& m, const std::string& node, int32_t label) { return m[{node, std::to_string(label)}]; }

struct Ring {  // SimpleRingTopologyFixture::CustomSetUp (DecisionTest.cpp:1695-1780)
  std::unordered_map<std::string, LinkState> als;
  PrefixState ps;
  thrift::AdjacencyDatabase db1, db2, db3, db4;
  Ring(bool v4, bool ksp2) {
    db1 = createAdjDb("1", {adj12, adj13}, 1);
    db2 = createAdjDb("2", {adj21, adj24}, 2);
    db3 = createAdjDb("3", {adj31, adj34}, 3);
    db4 = createAdjDb("4", {adj42, adj43}, 4);
    als.emplace(kDefaultArea, LinkState(kDefaultArea));
    auto& ls = als.at(kDefaultArea);
    for (auto* db : {&db1, &db2, &db3, &db4}) ls.updateAdjacencyDatabase(*db);
    const thrift::IpPrefix p4[] = {addr1V4, addr2V4, addr3V4, addr4V4}, p6[] = {addr1, addr2, addr3, addr4};
    for (int i = 0; i < 4; ++i)
      ps.updatePrefix(std::to_string(i + 1), kDefaultArea, createPrefixEntry(v4 ? p4[i] : p6[i], ksp2));
  }
};

}  // namespace

// --- DecisionTest.cpp:404-529 ShortestPathTest.* ------------------------------
TEST_GPU(ShortestPathTest_UnreachableNodes) {  // :404-441
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  auto& ls = als.at(kDefaultArea);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("1", {}, 0)).topologyChanged);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("2", {}, 0)).topologyChanged);
  PrefixState ps;
  ps.updatePrefix("1", kDefaultArea, createPrefixEntry(addr1));
  ps.updatePrefix("2", kDefaultArea, createPrefixEntry(addr2));
  SpfSolver solver("1", false, false);
  for (auto node : {"1", "2"}) {
    auto db = solver.buildRouteDb(node, als, ps);
    EXPECT_TRUE(db.has_value());
    EXPECT_EQ(db->unicastRoutes.size(), 0u);
    EXPECT_EQ(db->mplsRoutes.size(), 0u);
  }
}

TEST_GPU(ShortestPathTest_MissingNeighborAdjacencyDb) {  // :444-473
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  EXPECT_FALSE(als.at(kDefaultArea).updateAdjacencyDatabase(createAdjDb("1", {adj12}, 0)).topologyChanged);
  PrefixState ps;
  ps.updatePrefix("1", kDefaultArea, createPrefixEntry(addr1));
  ps.updatePrefix("2", kDefaultArea, createPrefixEntry(addr2));
  SpfSolver solver("1", false, false);
  auto db = solver.buildRouteDb("1", als, ps);
  EXPECT_TRUE(db.has_value());
  EXPECT_EQ(db->unicastRoutes.size(), 0u);
  EXPECT_EQ(db->mplsRoutes.size(), 0u);
}

TEST_GPU(ShortestPathTest_EmptyNeighborAdjacencyDb) {  // :476-509
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  auto& ls = als.at(kDefaultArea);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("1", {adj12}, 0)).topologyChanged);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("2", {}, 0)).topologyChanged);
  PrefixState ps;
  ps.updatePrefix("1", kDefaultArea, createPrefixEntry(addr1));
  ps.updatePrefix("2", kDefaultArea, createPrefixEntry(addr2));
  SpfSolver solver("1", false, false);
  EXPECT_EQ(solver.buildRouteDb("1", als, ps)->unicastRoutes.size(), 0u);
  EXPECT_EQ(solver.buildRouteDb("2", als, ps)->unicastRoutes.size(), 0u);
}

TEST_CPU(ShortestPathTest_UnknownNode) {  // :512-526 (no SPF: the node is in no area)
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  PrefixState ps;
  SpfSolver solver("1", false, false);
  EXPECT_FALSE(solver.buildRouteDb("1", als, ps).has_value());
  EXPECT_FALSE(solver.buildRouteDb("2", als, ps).has_value());
}

TEST_GPU(MplsRoutes_BasicTest) {  // :670-712
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  auto& ls = als.at(kDefaultArea);
  auto db1 = createAdjDb("1", {adj12}, 1);
  auto db2 = createAdjDb("2", {adj23}, 0);  // no node label
  auto db3 = createAdjDb("3", {adj32}, 3);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db1) == LinkState::LinkStateChange(false, false, true));
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db1) == LinkState::LinkStateChange(false, false, false));
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db2) == LinkState::LinkStateChange(false, false, false));
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db3) == LinkState::LinkStateChange(true, false, true));
  PrefixState ps;
  SpfSolver solver("1", false, false);
  auto m = getRouteMap(solver, {"1", "2", "3"}, als, ps);
  EXPECT_EQ(m.size(), 5u);
  validatePopLabelRoute(m, "1", db1.nodeLabel);
  validateAdjLabelRoutes(m, "2", {adj23});
  validatePopLabelRoute(m, "3", db3.nodeLabel);
  validateAdjLabelRoutes(m, "3", {adj32});
}

// --- SimpleRingTopologyFixture (DecisionTest.cpp:1814-1944, 1999-2127) -----------
static void ringShortestPath(bool v4, bool lfa) {
  Ring r(v4, false);
  SpfCounters::get().reset();
  SpfSolver solver("1", v4, lfa);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 36u);  // 12 unicast + 16 node label + 8 adj label
  if (!lfa) EXPECT_EQ(SpfCounters::get().spfRuns(), 4u);
  auto P = [&](const thrift::IpPrefix& a6, const thrift::IpPrefix& a4) { return v4 ? a4 : a6; };
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  // router 1
  EXPECT_EQ(at(m, "1", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj12, v4, 20), nhFromAdj(adj13, v4, 20)}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(adj12, false, 20, swap(4)), nhFromAdj(adj13, false, 20, swap(4))}));
  EXPECT_EQ(at(m, "1", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj13, v4, 10)}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(adj13, false, 10, php)}));
  EXPECT_EQ(at(m, "1", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj12, v4, 10)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(adj12, false, 10, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  // router 2
  EXPECT_EQ(at(m, "2", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj24, v4, 10)}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(adj24, false, 10, php)}));
  EXPECT_EQ(at(m, "2", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj21, v4, 20), nhFromAdj(adj24, v4, 20)}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(adj21, false, 20, swap(3)), nhFromAdj(adj24, false, 20, swap(3))}));
  EXPECT_EQ(at(m, "2", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj21, v4, 10)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(adj21, false, 10, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  // router 3
  EXPECT_EQ(at(m, "3", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj34, v4, 10)}));
  EXPECT_EQ(at(m, "3", 4), NextHopSet({nhFromAdj(adj34, false, 10, php)}));
  EXPECT_EQ(at(m, "3", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj31, v4, 20), nhFromAdj(adj34, v4, 20)}));
  EXPECT_EQ(at(m, "3", 2), NextHopSet({nhFromAdj(adj31, false, 20, swap(2)), nhFromAdj(adj34, false, 20, swap(2))}));
  EXPECT_EQ(at(m, "3", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj31, v4, 10)}));
  EXPECT_EQ(at(m, "3", 1), NextHopSet({nhFromAdj(adj31, false, 10, php)}));
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);
  // router 4
  EXPECT_EQ(at(m, "4", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj43, v4, 10)}));
  EXPECT_EQ(at(m, "4", 3), NextHopSet({nhFromAdj(adj43, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj42, v4, 10)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(adj42, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj42, v4, 20), nhFromAdj(adj43, v4, 20)}));
  EXPECT_EQ(at(m, "4", 1), NextHopSet({nhFromAdj(adj42, false, 20, swap(1)), nhFromAdj(adj43, false, 20, swap(1))}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);
}

// DecisionRouteDb::calculateUpdate's MPLS half as verifyRouteInUpdateNoDelete uses it
// (DecisionTest.cpp:1785-1799): `label` is updated exactly once and nothing is withdrawn.
static DecisionRouteDb mplsUpdateNoDelete(SpfSolver& solver, Ring& r, const char* node, int32_t label,
                                          const DecisionRouteDb& comp) {
  auto db = solver.buildRouteDb(node, r.als, r.ps).value();
  int updates = 0;
  for (const auto& [l, e] : db.mplsRoutes) {
    auto it = comp.mplsRoutes.find(l);
    if (l == label && (it == comp.mplsRoutes.end() || !(it->second.nexthops == e.nexthops))) ++updates;
  }
  size_t deletes = 0;
  for (const auto& kv : comp.mplsRoutes) deletes += db.mplsRoutes.count(kv.first) ? 0 : 1;
  EXPECT_EQ(updates, 1);
  EXPECT_EQ(deletes, 0u);
  return db;
}

TEST_GPU(SimpleRing_DuplicateMplsRoutes) {  // DecisionTest.cpp:1946-1993
  Ring r(false, false);
  SpfSolver solver("1", false, false);
  const uint64_t dup0 = solver.counters().duplicate_node_label;
  r.db1.nodeLabel = 2;  // node 1 now shares node 2's label
  r.als.at(kDefaultArea).updateAdjacencyDatabase(r.db1);
  const DecisionRouteDb empty;
  for (auto node : {"1", "2", "3"}) mplsUpdateNoDelete(solver, r, node, 2, empty);
  EXPECT_EQ(dup0 + 3, solver.counters().duplicate_node_label);  // one collision noticed per build
  auto comp1 = solver.buildRouteDb("1", r.als, r.ps).value();
  auto comp2 = solver.buildRouteDb("2", r.als, r.ps).value();
  auto comp3 = solver.buildRouteDb("3", r.als, r.ps).value();
  EXPECT_EQ(dup0 + 6, solver.counters().duplicate_node_label);
  for (auto* db : {&comp1, &comp2, &comp3}) EXPECT_EQ(db->mplsRoutes.count(1), 0u);  // label 1 is unused
  r.db1.nodeLabel = 1;  // back to distinct labels: label 2 changes owner, nothing withdrawn
  r.als.at(kDefaultArea).updateAdjacencyDatabase(r.db1);
  mplsUpdateNoDelete(solver, r, "1", 2, comp1);
  mplsUpdateNoDelete(solver, r, "2", 2, comp2);
  mplsUpdateNoDelete(solver, r, "3", 2, comp3);
  EXPECT_EQ(dup0 + 6, solver.counters().duplicate_node_label);
}

TEST_GPU(SimpleRing_ShortestPathTest_v6) { ringShortestPath(false, false); }
TEST_GPU(SimpleRing_ShortestPathTest_v4) { ringShortestPath(true, false); }
TEST_GPU(SimpleRing_MultiPathTest_LFA_v6) { ringShortestPath(false, true); }
TEST_GPU(SimpleRing_MultiPathTest_LFA_v4) { ringShortestPath(true, true); }

// DecisionTest.cpp:2290-2476 (router 1 and 2 expectations, prefix type default)
static void ringKsp2(bool v4) {
  Ring r(v4, true);
  SpfCounters::get().reset();
  SpfSolver solver("1", v4, true);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 36u);
  // 4 memoized SPFs + one second SPF per (node, other node): 4 + 4 * 3
  EXPECT_EQ(SpfCounters::get().spfRuns(), 16u);
  auto push = [](std::vector<int32_t> l) { return mpls(MplsActionCode::PUSH, std::nullopt, l); };
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  auto P = [&](const thrift::IpPrefix& a6, const thrift::IpPrefix& a4) { return v4 ? a4 : a6; };
  EXPECT_EQ(at(m, "1", P(addr4, addr4V4)),
            NextHopSet({nhFromAdj(adj12, v4, 20, push({4})), nhFromAdj(adj13, v4, 20, push({4}))}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(adj12, false, 20, swap(4)), nhFromAdj(adj13, false, 20, swap(4))}));
  EXPECT_EQ(at(m, "1", P(addr3, addr3V4)),
            NextHopSet({nhFromAdj(adj13, v4, 10, std::nullopt), nhFromAdj(adj12, v4, 30, push({3, 4}))}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(adj13, false, 10, php)}));
  EXPECT_EQ(at(m, "1", P(addr2, addr2V4)),
            NextHopSet({nhFromAdj(adj12, v4, 10, std::nullopt), nhFromAdj(adj13, v4, 30, push({2, 4}))}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(adj12, false, 10, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", P(addr4, addr4V4)),
            NextHopSet({nhFromAdj(adj24, v4, 10, std::nullopt), nhFromAdj(adj21, v4, 30, push({4, 3}))}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(adj24, false, 10, php)}));
  EXPECT_EQ(at(m, "2", P(addr3, addr3V4)),
            NextHopSet({nhFromAdj(adj21, v4, 20, push({3})), nhFromAdj(adj24, v4, 20, push({3}))}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(adj21, false, 20, swap(3)), nhFromAdj(adj24, false, 20, swap(3))}));
  EXPECT_EQ(at(m, "2", P(addr1, addr1V4)),
            NextHopSet({nhFromAdj(adj21, v4, 10, std::nullopt), nhFromAdj(adj24, v4, 30, push({1, 3}))}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(adj21, false, 10, php)}));
}

TEST_GPU(SimpleRing_Ksp2EdEcmp_v6) { ringKsp2(false); }
TEST_GPU(SimpleRing_Ksp2EdEcmp_v4) { ringKsp2(true); }


// KSP2 corner case of traceEdgeDisjointPaths (DecisionTest.cpp:2455-2475): adj12 and
// node 3 overloaded -> from node 1 no route to 2 or 4, addr3 only over adj13
static void ringKsp2Overload(bool v4) {
  Ring r(v4, true);
  SpfSolver solver("1", v4, true);
  r.db1.adjacencies[0].isOverloaded = true;
  r.db3.isOverloaded = true;
  auto& ls = r.als.at(kDefaultArea);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db1).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db3).topologyChanged);
  auto m = getRouteMap(solver, {"1"}, r.als, r.ps);
  auto P = [&](const thrift::IpPrefix& a6, const thrift::IpPrefix& a4) { return v4 ? a4 : a6; };
  EXPECT_TRUE(m.find({"1", P(addr4, addr4V4).toString()}) == m.end());
  EXPECT_EQ(at(m, "1", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj13, v4, 10, std::nullopt)}));
  EXPECT_TRUE(m.find({"1", P(addr2, addr2V4).toString()}) == m.end());
}
// An anycast KSP2 prefix that the building node also advertises with a prepend label
// (ADVICE r5): the second-path loop of selectBestPathsKsp2 then reads getKthPaths(me, me,
// 2), which is empty in the reference (traceOnePath(me, me) is the empty path) and which
// the token rows of prefetchKthPaths do not stage. Routes and spf_runs with the device
// prefetch must equal the call-by-call path's.
TEST_GPU(SimpleRing_Ksp2EdEcmp_AnycastSelfPrependLabel) {
  const auto anycast = pfx("fd00::a/128");
  auto run = [&](const char* prefetch) {
    setenv("OPENR_KSP2_PREFETCH", prefetch, 1);
    Ring r(false, true);
    for (auto const& [node, label] : {std::pair<std::string, int32_t>{"1", 60001}, {"4", 60004}}) {
      auto e = createPrefixEntry(anycast, true);
      e.prependLabel = label;
      r.ps.updatePrefix(node, kDefaultArea, e);
    }
    SpfCounters::get().reset();
    SpfSolver solver("1", false, true);
    auto m = getRouteMap(solver, {"1", "2"}, r.als, r.ps);
    return std::make_pair(m, SpfCounters::get().spfRuns());
  };
  auto off = run("0");
  auto on = run("1");
  unsetenv("OPENR_KSP2_PREFETCH");
  EXPECT_TRUE(off.first == on.first);
  EXPECT_EQ(off.second, on.second);
  // node 1 reaches node 4's copy over both ring neighbours, under 4's prepend label
  const auto push = [](std::vector<int32_t> l) { return mpls(MplsActionCode::PUSH, std::nullopt, l); };
  EXPECT_EQ(at(on.first, "1", anycast),
            NextHopSet({nhFromAdj(adj12, false, 20, push({60004, 4})), nhFromAdj(adj13, false, 20, push({60004, 4}))}));
  EXPECT_EQ(at(on.first, "2", anycast).size(), at(off.first, "2", anycast).size());
}

TEST_GPU(SimpleRing_Ksp2EdEcmp_OverloadCorner_v6) { ringKsp2Overload(false); }
TEST_GPU(SimpleRing_Ksp2EdEcmp_OverloadCorner_v4) { ringKsp2Overload(true); }

// SimpleRingTopologyFixture.OverloadNodeTest (DecisionTest.cpp:2821-2930): nodes 2 and 3
// overloaded (reached, never transit), LFA on
static void ringOverloadNode(bool v4) {
  Ring r(v4, false);
  SpfSolver solver("1", v4, true);
  r.db2.isOverloaded = true;
  r.db3.isOverloaded = true;
  auto& ls = r.als.at(kDefaultArea);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db2).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db3).topologyChanged);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 32u);  // unicast 2+3+3+2, node labels 3+4+4+3, adj labels 4*2
  auto P = [&](const thrift::IpPrefix& a6, const thrift::IpPrefix& a4) { return v4 ? a4 : a6; };
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  EXPECT_EQ(at(m, "1", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj13, v4, 10)}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(adj13, false, 10, php)}));
  EXPECT_EQ(at(m, "1", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj12, v4, 10)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(adj12, false, 10, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj24, v4, 10)}));  // no LFA
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(adj24, false, 10, php)}));
  EXPECT_EQ(at(m, "2", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj21, v4, 20), nhFromAdj(adj24, v4, 20)}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(adj21, false, 20, swap(3)), nhFromAdj(adj24, false, 20, swap(3))}));
  EXPECT_EQ(at(m, "2", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj21, v4, 10)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(adj21, false, 10, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  EXPECT_EQ(at(m, "3", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj34, v4, 10)}));
  EXPECT_EQ(at(m, "3", 4), NextHopSet({nhFromAdj(adj34, false, 10, php)}));
  EXPECT_EQ(at(m, "3", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj31, v4, 20), nhFromAdj(adj34, v4, 20)}));
  EXPECT_EQ(at(m, "3", 2), NextHopSet({nhFromAdj(adj31, false, 20, swap(2)), nhFromAdj(adj34, false, 20, swap(2))}));
  EXPECT_EQ(at(m, "3", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj31, v4, 10)}));
  EXPECT_EQ(at(m, "3", 1), NextHopSet({nhFromAdj(adj31, false, 10, php)}));
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);
  EXPECT_EQ(at(m, "4", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj43, v4, 10)}));
  EXPECT_EQ(at(m, "4", 3), NextHopSet({nhFromAdj(adj43, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj42, v4, 10)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(adj42, false, 10, php)}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);
}
TEST_GPU(SimpleRing_OverloadNodeTest_v6) { ringOverloadNode(false); }
TEST_GPU(SimpleRing_OverloadNodeTest_v4) { ringOverloadNode(true); }

// SimpleRingTopologyFixture.OverloadLinkTest (DecisionTest.cpp:2936-3113): adj31, then also
// adj34, overloaded (Link::isUp false in both directions), LFA on
static void ringOverloadLink(bool v4) {
  Ring r(v4, false);
  SpfSolver solver("1", v4, true);
  r.db3.adjacencies[0].isOverloaded = true;  // adj31
  auto& ls = r.als.at(kDefaultArea);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db3).topologyChanged);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 36u);
  auto P = [&](const thrift::IpPrefix& a6, const thrift::IpPrefix& a4) { return v4 ? a4 : a6; };
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  EXPECT_EQ(at(m, "1", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj12, v4, 20)}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(adj12, false, 20, swap(4))}));
  EXPECT_EQ(at(m, "1", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj12, v4, 30)}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(adj12, false, 30, swap(3))}));
  EXPECT_EQ(at(m, "1", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj12, v4, 10)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(adj12, false, 10, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj24, v4, 10)}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(adj24, false, 10, php)}));
  EXPECT_EQ(at(m, "2", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj24, v4, 20)}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(adj24, false, 20, swap(3))}));
  EXPECT_EQ(at(m, "2", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj21, v4, 10)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(adj21, false, 10, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  EXPECT_EQ(at(m, "3", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj34, v4, 10)}));
  EXPECT_EQ(at(m, "3", 4), NextHopSet({nhFromAdj(adj34, false, 10, php)}));
  EXPECT_EQ(at(m, "3", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj34, v4, 20)}));
  EXPECT_EQ(at(m, "3", 2), NextHopSet({nhFromAdj(adj34, false, 20, swap(2))}));
  EXPECT_EQ(at(m, "3", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj34, v4, 30)}));
  EXPECT_EQ(at(m, "3", 1), NextHopSet({nhFromAdj(adj34, false, 30, swap(1))}));
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);  // adj label routes stay for a down link
  EXPECT_EQ(at(m, "4", P(addr3, addr3V4)), NextHopSet({nhFromAdj(adj43, v4, 10)}));
  EXPECT_EQ(at(m, "4", 3), NextHopSet({nhFromAdj(adj43, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj42, v4, 10)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(adj42, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj42, v4, 20)}));
  EXPECT_EQ(at(m, "4", 1), NextHopSet({nhFromAdj(adj42, false, 20, swap(1))}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);

  // adj34 overloaded too: node 3 is disconnected
  r.db3.adjacencies[1].isOverloaded = true;
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db3).topologyChanged);
  m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 24u);  // unicast 2+2+0+2, node labels 3*3+1, adj labels 4*2
  EXPECT_EQ(at(m, "1", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj12, v4, 20)}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(adj12, false, 20, swap(4))}));
  EXPECT_EQ(at(m, "1", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj12, v4, 10)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(adj12, false, 10, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", P(addr4, addr4V4)), NextHopSet({nhFromAdj(adj24, v4, 10)}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(adj24, false, 10, php)}));
  EXPECT_EQ(at(m, "2", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj21, v4, 10)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(adj21, false, 10, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);
  EXPECT_EQ(at(m, "4", P(addr2, addr2V4)), NextHopSet({nhFromAdj(adj42, v4, 10)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(adj42, false, 10, php)}));
  EXPECT_EQ(at(m, "4", P(addr1, addr1V4)), NextHopSet({nhFromAdj(adj42, v4, 20)}));
  EXPECT_EQ(at(m, "4", 1), NextHopSet({nhFromAdj(adj42, false, 20, swap(1))}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);
}
TEST_GPU(SimpleRing_OverloadLinkTest_v6) { ringOverloadLink(false); }
TEST_GPU(SimpleRing_OverloadLinkTest_v4) { ringOverloadLink(true); }

// --- ParallelAdjRingTopologyFixture (DecisionTest.cpp:3136-3705) ---------------------
namespace {
struct ParallelRing {  // CustomSetUp :3143-3222
  std::unordered_map<std::string, LinkState> als;
  PrefixState ps;
  thrift::Adjacency adj12_1 = createAdjacency("2", "2/1", "1/1", "fe80::2:1", "192.168.2.1", 11, 201),
                    adj12_2 = createAdjacency("2", "2/2", "1/2", "fe80::2:2", "192.168.2.2", 11, 202),
                    adj12_3 = createAdjacency("2", "2/3", "1/3", "fe80::2:3", "192.168.2.3", 20, 203),
                    adj13_1 = createAdjacency("3", "3/1", "1/1", "fe80::3:1", "192.168.3.1", 11, 301),
                    adj21_1 = createAdjacency("1", "1/1", "2/1", "fe80::1:1", "192.168.1.1", 11, 101),
                    adj21_2 = createAdjacency("1", "1/2", "2/2", "fe80::1:2", "192.168.1.2", 11, 102),
                    adj21_3 = createAdjacency("1", "1/3", "2/3", "fe80::1:3", "192.168.1.3", 20, 103),
                    adj24_1 = createAdjacency("4", "4/1", "2/1", "fe80::4:1", "192.168.4.1", 11, 401),
                    adj31_1 = createAdjacency("1", "1/1", "3/1", "fe80::1:1", "192.168.1.1", 11, 101),
                    adj34_1 = createAdjacency("4", "4/1", "3/1", "fe80::4:1", "192.168.4.1", 11, 401),
                    adj34_2 = createAdjacency("4", "4/2", "3/2", "fe80::4:2", "192.168.4.2", 20, 402),
                    adj34_3 = createAdjacency("4", "4/3", "3/3", "fe80::4:3", "192.168.4.3", 20, 403),
                    adj42_1 = createAdjacency("2", "2/1", "4/1", "fe80::2:1", "192.168.2.1", 11, 201),
                    adj43_1 = createAdjacency("3", "3/1", "4/1", "fe80::3:1", "192.168.3.1", 11, 301),
                    adj43_2 = createAdjacency("3", "3/2", "4/2", "fe80::3:2", "192.168.3.2", 20, 302),
                    adj43_3 = createAdjacency("3", "3/3", "4/3", "fe80::3:3", "192.168.3.3", 20, 303);
  thrift::AdjacencyDatabase db1, db2, db3, db4;
  explicit ParallelRing(bool ksp2) {
    db1 = createAdjDb("1", {adj12_1, adj12_2, adj12_3, adj13_1}, 1);
    db2 = createAdjDb("2", {adj21_1, adj21_2, adj21_3, adj24_1}, 2);
    db3 = createAdjDb("3", {adj31_1, adj34_1, adj34_2, adj34_3}, 3);
    db4 = createAdjDb("4", {adj42_1, adj43_1, adj43_2, adj43_3}, 4);
    als.emplace(kDefaultArea, LinkState(kDefaultArea));
    auto& ls = als.at(kDefaultArea);
    EXPECT_FALSE(ls.updateAdjacencyDatabase(db1).topologyChanged);
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db2).topologyChanged);
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db3).topologyChanged);
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db4).topologyChanged);
    const thrift::IpPrefix p6[] = {addr1, addr2, addr3, addr4};
    for (int i = 0; i < 4; ++i) ps.updatePrefix(std::to_string(i + 1), kDefaultArea, createPrefixEntry(p6[i], ksp2));
  }
};
}  // namespace

TEST_GPU(ParallelAdjRing_ShortestPathTest) {  // :3226-3335
  ParallelRing r(false);
  SpfSolver solver("1", false, false);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 44u);
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  EXPECT_EQ(at(m, "1", addr4), NextHopSet({nhFromAdj(r.adj12_2, false, 22), nhFromAdj(r.adj13_1, false, 22),
                                           nhFromAdj(r.adj12_1, false, 22)}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(r.adj12_2, false, 22, swap(4)), nhFromAdj(r.adj13_1, false, 22, swap(4)),
                                       nhFromAdj(r.adj12_1, false, 22, swap(4))}));
  EXPECT_EQ(at(m, "1", addr3), NextHopSet({nhFromAdj(r.adj13_1, false, 11)}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(r.adj13_1, false, 11, php)}));
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(r.adj12_2, false, 11), nhFromAdj(r.adj12_1, false, 11)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(r.adj12_2, false, 11, php), nhFromAdj(r.adj12_1, false, 11, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", addr4), NextHopSet({nhFromAdj(r.adj24_1, false, 11)}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(r.adj24_1, false, 11, php)}));
  EXPECT_EQ(at(m, "2", addr3), NextHopSet({nhFromAdj(r.adj21_2, false, 22), nhFromAdj(r.adj21_1, false, 22),
                                           nhFromAdj(r.adj24_1, false, 22)}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(r.adj21_2, false, 22, swap(3)), nhFromAdj(r.adj21_1, false, 22, swap(3)),
                                       nhFromAdj(r.adj24_1, false, 22, swap(3))}));
  EXPECT_EQ(at(m, "2", addr1), NextHopSet({nhFromAdj(r.adj21_2, false, 11), nhFromAdj(r.adj21_1, false, 11)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(r.adj21_2, false, 11, php), nhFromAdj(r.adj21_1, false, 11, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  EXPECT_EQ(at(m, "3", addr4), NextHopSet({nhFromAdj(r.adj34_1, false, 11)}));
  EXPECT_EQ(at(m, "3", 4), NextHopSet({nhFromAdj(r.adj34_1, false, 11, php)}));
  EXPECT_EQ(at(m, "3", addr2), NextHopSet({nhFromAdj(r.adj31_1, false, 22), nhFromAdj(r.adj34_1, false, 22)}));
  EXPECT_EQ(at(m, "3", 2), NextHopSet({nhFromAdj(r.adj31_1, false, 22, swap(2)), nhFromAdj(r.adj34_1, false, 22, swap(2))}));
  EXPECT_EQ(at(m, "3", addr1), NextHopSet({nhFromAdj(r.adj31_1, false, 11)}));
  EXPECT_EQ(at(m, "3", 1), NextHopSet({nhFromAdj(r.adj31_1, false, 11, php)}));
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);
  EXPECT_EQ(at(m, "4", addr3), NextHopSet({nhFromAdj(r.adj43_1, false, 11)}));
  EXPECT_EQ(at(m, "4", 3), NextHopSet({nhFromAdj(r.adj43_1, false, 11, php)}));
  EXPECT_EQ(at(m, "4", addr2), NextHopSet({nhFromAdj(r.adj42_1, false, 11)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(r.adj42_1, false, 11, php)}));
  EXPECT_EQ(at(m, "4", addr1), NextHopSet({nhFromAdj(r.adj42_1, false, 22), nhFromAdj(r.adj43_1, false, 22)}));
  EXPECT_EQ(at(m, "4", 1), NextHopSet({nhFromAdj(r.adj42_1, false, 22, swap(1)), nhFromAdj(r.adj43_1, false, 22, swap(1))}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);
}

TEST_GPU(ParallelAdjRing_MultiPathTest) {  // :3340-3512 (LFA: parallel links of larger metric too)
  ParallelRing r(false);
  SpfSolver solver("1", false, true);
  auto m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 44u);
  const auto swap = [](int l) { return mpls(MplsActionCode::SWAP, l); };
  const auto php = mpls(MplsActionCode::PHP);
  EXPECT_EQ(at(m, "1", addr4), NextHopSet({nhFromAdj(r.adj12_1, false, 22), nhFromAdj(r.adj12_2, false, 22),
                                           nhFromAdj(r.adj12_3, false, 31), nhFromAdj(r.adj13_1, false, 22)}));
  EXPECT_EQ(at(m, "1", 4), NextHopSet({nhFromAdj(r.adj12_1, false, 22, swap(4)), nhFromAdj(r.adj12_2, false, 22, swap(4)),
                                       nhFromAdj(r.adj12_3, false, 31, swap(4)), nhFromAdj(r.adj13_1, false, 22, swap(4))}));
  EXPECT_EQ(at(m, "1", addr3), NextHopSet({nhFromAdj(r.adj13_1, false, 11)}));
  EXPECT_EQ(at(m, "1", 3), NextHopSet({nhFromAdj(r.adj13_1, false, 11, php)}));
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(r.adj12_1, false, 11), nhFromAdj(r.adj12_2, false, 11),
                                           nhFromAdj(r.adj12_3, false, 20)}));
  EXPECT_EQ(at(m, "1", 2), NextHopSet({nhFromAdj(r.adj12_1, false, 11, php), nhFromAdj(r.adj12_2, false, 11, php),
                                       nhFromAdj(r.adj12_3, false, 20, php)}));
  validatePopLabelRoute(m, "1", 1);
  validateAdjLabelRoutes(m, "1", r.db1.adjacencies);
  EXPECT_EQ(at(m, "2", addr4), NextHopSet({nhFromAdj(r.adj24_1, false, 11)}));
  EXPECT_EQ(at(m, "2", 4), NextHopSet({nhFromAdj(r.adj24_1, false, 11, php)}));
  EXPECT_EQ(at(m, "2", addr3), NextHopSet({nhFromAdj(r.adj21_1, false, 22), nhFromAdj(r.adj21_2, false, 22),
                                           nhFromAdj(r.adj21_3, false, 31), nhFromAdj(r.adj24_1, false, 22)}));
  EXPECT_EQ(at(m, "2", 3), NextHopSet({nhFromAdj(r.adj21_1, false, 22, swap(3)), nhFromAdj(r.adj21_2, false, 22, swap(3)),
                                       nhFromAdj(r.adj21_3, false, 31, swap(3)), nhFromAdj(r.adj24_1, false, 22, swap(3))}));
  EXPECT_EQ(at(m, "2", addr1), NextHopSet({nhFromAdj(r.adj21_1, false, 11), nhFromAdj(r.adj21_2, false, 11),
                                           nhFromAdj(r.adj21_3, false, 20)}));
  EXPECT_EQ(at(m, "2", 1), NextHopSet({nhFromAdj(r.adj21_1, false, 11, php), nhFromAdj(r.adj21_2, false, 11, php),
                                       nhFromAdj(r.adj21_3, false, 20, php)}));
  validatePopLabelRoute(m, "2", 2);
  validateAdjLabelRoutes(m, "2", r.db2.adjacencies);
  EXPECT_EQ(at(m, "3", addr4), NextHopSet({nhFromAdj(r.adj34_1, false, 11), nhFromAdj(r.adj34_2, false, 20),
                                           nhFromAdj(r.adj34_3, false, 20)}));
  EXPECT_EQ(at(m, "3", 4), NextHopSet({nhFromAdj(r.adj34_1, false, 11, php), nhFromAdj(r.adj34_2, false, 20, php),
                                       nhFromAdj(r.adj34_3, false, 20, php)}));
  EXPECT_EQ(at(m, "3", addr2), NextHopSet({nhFromAdj(r.adj31_1, false, 22), nhFromAdj(r.adj34_1, false, 22),
                                           nhFromAdj(r.adj34_2, false, 31), nhFromAdj(r.adj34_3, false, 31)}));
  EXPECT_EQ(at(m, "3", 2), NextHopSet({nhFromAdj(r.adj31_1, false, 22, swap(2)), nhFromAdj(r.adj34_1, false, 22, swap(2)),
                                       nhFromAdj(r.adj34_2, false, 31, swap(2)), nhFromAdj(r.adj34_3, false, 31, swap(2))}));
  EXPECT_EQ(at(m, "3", addr1), NextHopSet({nhFromAdj(r.adj31_1, false, 11)}));
  EXPECT_EQ(at(m, "3", 1), NextHopSet({nhFromAdj(r.adj31_1, false, 11, php)}));
  validatePopLabelRoute(m, "3", 3);
  validateAdjLabelRoutes(m, "3", r.db3.adjacencies);
  EXPECT_EQ(at(m, "4", addr3), NextHopSet({nhFromAdj(r.adj43_1, false, 11), nhFromAdj(r.adj43_2, false, 20),
                                           nhFromAdj(r.adj43_3, false, 20)}));
  EXPECT_EQ(at(m, "4", 3), NextHopSet({nhFromAdj(r.adj43_1, false, 11, php), nhFromAdj(r.adj43_2, false, 20, php),
                                       nhFromAdj(r.adj43_3, false, 20, php)}));
  EXPECT_EQ(at(m, "4", addr2), NextHopSet({nhFromAdj(r.adj42_1, false, 11)}));
  EXPECT_EQ(at(m, "4", 2), NextHopSet({nhFromAdj(r.adj42_1, false, 11, php)}));
  EXPECT_EQ(at(m, "4", addr1), NextHopSet({nhFromAdj(r.adj42_1, false, 22), nhFromAdj(r.adj43_1, false, 22),
                                           nhFromAdj(r.adj43_2, false, 31), nhFromAdj(r.adj43_3, false, 31)}));
  EXPECT_EQ(at(m, "4", 1), NextHopSet({nhFromAdj(r.adj42_1, false, 22, swap(1)), nhFromAdj(r.adj43_1, false, 22, swap(1)),
                                       nhFromAdj(r.adj43_2, false, 31, swap(1)), nhFromAdj(r.adj43_3, false, 31, swap(1))}));
  validatePopLabelRoute(m, "4", 4);
  validateAdjLabelRoutes(m, "4", r.db4.adjacencies);
}

TEST_GPU(ParallelAdjRing_Ksp2EdEcmp) {  // :3517-3705 (prefix type unset)
  ParallelRing r(true);
  SpfSolver solver("1", false, true);
  auto push = [](std::vector<int32_t> l) { return mpls(MplsActionCode::PUSH, std::nullopt, l); };
  auto m = getRouteMap(solver, {"1"}, r.als, r.ps);
  // parallel links between node 1 and node 2
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(r.adj12_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj12_2, false, 11, std::nullopt),
                                           nhFromAdj(r.adj12_3, false, 20, std::nullopt)}));
  // minNexthop: an SR_MPLS / KSP2 loopback prefix of node 4 with threshold 4 is dropped,
  // with 2 it has the edge-disjoint pair adj12_2, adj13_1 (the adj12_2 choice is the
  // folly-hash linksFromNode order, :3596-3599)
  const auto bgpAddr1 = pfx("2401:1::10.1.1.1/32");
  thrift::PrefixEntry np;
  np.prefix = bgpAddr1;
  np.type = thrift::PrefixType::LOOPBACK;
  np.forwardingType = thrift::PrefixForwardingType::SR_MPLS;
  np.forwardingAlgorithm = thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
  np.minNexthop = 4;
  r.ps.updatePrefix("4", kDefaultArea, np);
  m = getRouteMap(solver, {"1"}, r.als, r.ps);
  EXPECT_TRUE(m.find({"1", bgpAddr1.toString()}) == m.end());
  np.minNexthop = 2;
  r.ps.updatePrefix("4", kDefaultArea, np);
  m = getRouteMap(solver, {"1"}, r.als, r.ps);
  EXPECT_EQ(at(m, "1", bgpAddr1), NextHopSet({nhFromAdj(r.adj12_2, false, 22, push({4})),
                                              nhFromAdj(r.adj13_1, false, 22, push({4}))}));
  // node 3 announces it too with threshold 4: the anycast threshold is 4, route dropped
  np.minNexthop = 4;
  r.ps.updatePrefix("3", kDefaultArea, np);
  m = getRouteMap(solver, {"1"}, r.als, r.ps);
  EXPECT_TRUE(m.find({"1", bgpAddr1.toString()}) == m.end());
  r.ps.deletePrefix("4", kDefaultArea, bgpAddr1);
  r.ps.deletePrefix("3", kDefaultArea, bgpAddr1);

  // adj12_2 and adj34_2 down
  r.db1.adjacencies.at(1).isOverloaded = true;
  r.db3.adjacencies.at(2).isOverloaded = true;
  auto& ls = r.als.at(kDefaultArea);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db1).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(r.db3).topologyChanged);
  m = getRouteMap(solver, {"1", "2", "3", "4"}, r.als, r.ps);
  EXPECT_EQ(m.size(), 44u);
  EXPECT_EQ(at(m, "1", addr4), NextHopSet({nhFromAdj(r.adj12_1, false, 22, push({4})),
                                           nhFromAdj(r.adj13_1, false, 22, push({4}))}));
  EXPECT_EQ(at(m, "1", addr3), NextHopSet({nhFromAdj(r.adj13_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj12_1, false, 33, push({3, 4}))}));
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(r.adj12_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj12_3, false, 20, std::nullopt)}));
  EXPECT_EQ(at(m, "2", addr4), NextHopSet({nhFromAdj(r.adj24_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj21_1, false, 33, push({4, 3}))}));
  EXPECT_EQ(at(m, "2", addr3), NextHopSet({nhFromAdj(r.adj21_1, false, 22, push({3})),
                                           nhFromAdj(r.adj24_1, false, 22, push({3}))}));
  EXPECT_EQ(at(m, "2", addr1), NextHopSet({nhFromAdj(r.adj21_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj21_3, false, 20, std::nullopt)}));
  EXPECT_EQ(at(m, "3", addr4), NextHopSet({nhFromAdj(r.adj34_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj34_3, false, 20, std::nullopt)}));
  EXPECT_EQ(at(m, "3", addr2), NextHopSet({nhFromAdj(r.adj31_1, false, 22, push({2})),
                                           nhFromAdj(r.adj34_1, false, 22, push({2}))}));
  EXPECT_EQ(at(m, "3", addr1), NextHopSet({nhFromAdj(r.adj31_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj34_1, false, 33, push({1, 2}))}));
  EXPECT_EQ(at(m, "4", addr3), NextHopSet({nhFromAdj(r.adj43_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj43_3, false, 20, std::nullopt)}));
  EXPECT_EQ(at(m, "4", addr2), NextHopSet({nhFromAdj(r.adj42_1, false, 11, std::nullopt),
                                           nhFromAdj(r.adj43_1, false, 33, push({2, 1}))}));
  EXPECT_EQ(at(m, "4", addr1), NextHopSet({nhFromAdj(r.adj42_1, false, 22, push({1})),
                                           nhFromAdj(r.adj43_1, false, 22, push({1}))}));
}

// --- DecisionTestFixture.LoopFreeAlternatePaths (DecisionTest.cpp:5702-5837) ----------
// Triangle 1-2 (10), 1-3 (8), 2-3 (9), LFA on: RFC 5286 alternates d(n,dst) < d(me,dst) +
// d(n,me) (Decision.cpp:1170-1204) with real alternates, then none after 1-2 goes to 100.
TEST_GPU(LoopFreeAlternatePaths) {
  auto a12 = createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 0);
  auto a13 = createAdjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 8, 0);
  auto a21 = createAdjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 0);
  auto a23 = createAdjacency("3", "2/3", "3/2", "fe80::3", "192.168.0.3", 9, 0);
  auto a31 = createAdjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 8, 0);
  auto a32 = createAdjacency("2", "3/2", "2/3", "fe80::2", "192.168.0.2", 9, 0);
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  auto& ls = als.at(kDefaultArea);
  ls.updateAdjacencyDatabase(createAdjDb("1", {a12, a13}, 0));
  ls.updateAdjacencyDatabase(createAdjDb("2", {a21, a23}, 0));
  ls.updateAdjacencyDatabase(createAdjDb("3", {a31, a32}, 0));
  PrefixState ps;
  ps.updatePrefix("1", kDefaultArea, createPrefixEntry(addr1));
  ps.updatePrefix("2", kDefaultArea, createPrefixEntry(addr2));
  ps.updatePrefix("3", kDefaultArea, createPrefixEntry(addr3));
  SpfSolver solver("1", false, true);
  auto m = getRouteMap(solver, {"1", "2", "3"}, als, ps);
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(a12, false, 10), nhFromAdj(a13, false, 17)}));
  EXPECT_EQ(at(m, "1", addr3), NextHopSet({nhFromAdj(a12, false, 19), nhFromAdj(a13, false, 8)}));
  EXPECT_EQ(at(m, "2", addr1), NextHopSet({nhFromAdj(a21, false, 10), nhFromAdj(a23, false, 17)}));
  EXPECT_EQ(at(m, "2", addr3), NextHopSet({nhFromAdj(a21, false, 18), nhFromAdj(a23, false, 9)}));
  EXPECT_EQ(at(m, "3", addr1), NextHopSet({nhFromAdj(a31, false, 8), nhFromAdj(a32, false, 19)}));
  EXPECT_EQ(at(m, "3", addr2), NextHopSet({nhFromAdj(a31, false, 18), nhFromAdj(a32, false, 9)}));
  // node1 -- node2 metric 100: node 3 loses its loop-free alternates
  a12.metric = 100;
  a21.metric = 100;
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("1", {a12, a13}, 0)).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("2", {a21, a23}, 0)).topologyChanged);
  m = getRouteMap(solver, {"1", "2", "3"}, als, ps);
  EXPECT_EQ(at(m, "1", addr2), NextHopSet({nhFromAdj(a12, false, 100), nhFromAdj(a13, false, 17)}));
  EXPECT_EQ(at(m, "1", addr3), NextHopSet({nhFromAdj(a12, false, 109), nhFromAdj(a13, false, 8)}));
  EXPECT_EQ(at(m, "2", addr1), NextHopSet({nhFromAdj(a21, false, 100), nhFromAdj(a23, false, 17)}));
  EXPECT_EQ(at(m, "2", addr3), NextHopSet({nhFromAdj(a21, false, 108), nhFromAdj(a23, false, 9)}));
  EXPECT_EQ(at(m, "3", addr1), NextHopSet({nhFromAdj(a31, false, 8)}));
  EXPECT_EQ(at(m, "3", addr2), NextHopSet({nhFromAdj(a32, false, 9)}));
}

// --- GridTopologyFixture.ShortestPathTest (DecisionTest.cpp:4206-4355) ------------
static int gridDistance(int a, int b, int n) { return std::abs(a % n - b % n) + std::abs(a / n - b / n); }

// createGrid (DecisionTest.cpp:4240-4265): n x n grid, unit metrics, adjacency labels
// 100001 + neighbour, node labels node + 1, one prefix per node
static void createGrid(LinkState& ls, PrefixState& ps, int n) {
  auto addAdj = [&](int i, int j, const std::string& ifName, std::vector<thrift::Adjacency>& adjs,
                    const std::string& otherIf) {  // :4208-4233
    if (i < 0 || i >= n || j < 0 || j >= n) return;
    const int nb = i * n + j;
    adjs.push_back(createAdjacency(std::to_string(nb), ifName, otherIf, "fe80::" + std::to_string(nb),
                                   "192.168." + std::to_string(nb / 256) + "." + std::to_string(nb % 256), 1,
                                   100001 + nb));
  };
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      const int node = i * n + j;
      std::vector<thrift::Adjacency> adjs;
      addAdj(i, j + 1, "0/1", adjs, "0/3");
      addAdj(i - 1, j, "0/2", adjs, "0/4");
      addAdj(i, j - 1, "0/3", adjs, "0/1");
      addAdj(i + 1, j, "0/4", adjs, "0/2");
      ls.updateAdjacencyDatabase(createAdjDb(std::to_string(node), adjs, node + 1));
      ps.updatePrefix(std::to_string(node), kDefaultArea, createPrefixEntry(pfx("fc00::" + std::to_string(node) + "/128")));
    }
}

// GridTopologyFixture over the reference's whole Range(2, 17, 2) (DecisionTest.cpp:4289-4290):
// the route count 2n^4 + 3n^2 - 4n, and — stronger than the reference's four sampled pairs —
// every (src, dst) unicast route: metric = grid distance, next hops = exactly the
// neighbours one hop closer to dst.
TEST_GPU(GridTopology_ShortestPathTest) {
  for (int n = 2; n <= 16; n += 2) {
    std::unordered_map<std::string, LinkState> als;
    als.emplace(kDefaultArea, LinkState(kDefaultArea));
    PrefixState ps;
    createGrid(als.at(kDefaultArea), ps, n);
    SpfSolver solver("1", false, false);
    std::vector<std::string> all;
    for (int i = 0; i < n * n; ++i) all.push_back(std::to_string(i));
    auto m = getRouteMap(solver, all, als, ps);
    EXPECT_EQ((long)m.size(), 2L * n * n * n * n + 3L * n * n - 4L * n);
    bool ok = true;
    for (int src = 0; src < n * n; ++src)
      for (int dst = 0; dst < n * n; ++dst) {
        if (src == dst) continue;
        auto const& nhs = m[{std::to_string(src), "fc00::" + std::to_string(dst) + "/128"}];
        std::set<std::string> got, want;
        for (auto const& nh : nhs) {
          ok &= nh.metric == gridDistance(src, dst, n);
          got.insert(nh.neighborNodeName.value_or(""));
        }
        const int si = src / n, sj = src % n;
        const int cand[4][2] = {{si, sj + 1}, {si - 1, sj}, {si, sj - 1}, {si + 1, sj}};
        for (auto const& c : cand)
          if (c[0] >= 0 && c[0] < n && c[1] >= 0 && c[1] < n &&
              gridDistance(c[0] * n + c[1], dst, n) == gridDistance(src, dst, n) - 1)
            want.insert(std::to_string(c[0] * n + c[1]));
        ok &= got == want;
      }
    EXPECT_TRUE(ok);
  }
}

// --- best route selection / RibPolicy (no SPF) -------------------------------------
TEST_CPU(SelectBestPrefixMetrics) {  // Util.h:548-578; UtilTest.cpp:990-1010
  PrefixEntries e;
  auto with = [](int pp, int sp, int d) {
    thrift::PrefixEntry x;
    x.metrics.path_preference = pp;
    x.metrics.source_preference = sp;
    x.metrics.distance = d;
    return x;
  };
  e[{"a", "0"}] = with(0, 0, 1);  // below the (0, 0, 0) start: never selected
  EXPECT_TRUE(selectBestPrefixMetrics(e).empty());
  e[{"b", "0"}] = with(100, 100, 10);
  e[{"c", "0"}] = with(100, 100, 5);
  e[{"d", "0"}] = with(100, 90, 1);
  EXPECT_EQ(selectBestPrefixMetrics(e), (std::set<NodeAndArea>{{"c", "0"}}));
  e[{"e", "0"}] = with(100, 100, 5);
  EXPECT_EQ(selectBestPrefixMetrics(e), (std::set<NodeAndArea>{{"c", "0"}, {"e", "0"}}));
  EXPECT_EQ(selectBestNodeArea({{"c", "0"}, {"e", "0"}}, "e"), NodeAndArea("e", "0"));
  EXPECT_EQ(selectBestNodeArea({{"c", "0"}, {"e", "0"}}, "x"), NodeAndArea("c", "0"));
}

TEST_CPU(RibPolicy_ApplyAction) {  // RibPolicy.cpp:61-111 (RibPolicyTest semantics)
  RibUnicastEntry route;
  route.prefix = addr1;
  auto mk = [](const std::string& nbr, const std::string& area) {
    thrift::NextHopThrift nh;
    nh.address.addr = "fe80::" + nbr;
    nh.neighborNodeName = nbr;
    nh.area = area;
    return nh;
  };
  route.nexthops = {mk("n1", "A"), mk("n2", "B"), mk("n3", "C")};
  RibPolicyStatement st;
  st.name = "s";
  st.prefixes = {addr1};
  st.defaultWeight = 1;
  st.areaToWeight = {{"B", 2}, {"C", 0}};
  st.neighborToWeight = {{"n2", 5}};
  RibPolicy policy({st});
  EXPECT_TRUE(policy.isActive());
  auto r = route;
  EXPECT_TRUE(policy.applyAction(r));
  std::map<std::string, int32_t> w;
  for (auto const& nh : r.nexthops) w[*nh.neighborNodeName] = nh.weight;
  EXPECT_EQ(w.size(), 2u);  // n3: area weight 0 drops it
  EXPECT_EQ(w["n1"], 1);    // default
  EXPECT_EQ(w["n2"], 5);    // neighbour beats area
  // a statement that drops every next-hop leaves the route unchanged
  RibPolicyStatement drop = st;
  drop.defaultWeight = 0;
  drop.areaToWeight.clear();
  drop.neighborToWeight.clear();
  auto r2 = route;
  EXPECT_FALSE(RibPolicy({drop}).applyAction(r2));
  EXPECT_EQ(r2.nexthops, route.nexthops);
  // no match
  auto r3 = route;
  r3.prefix = addr2;
  EXPECT_FALSE(policy.applyAction(r3));
  UnicastRoutes db{{addr1, route}, {addr2, r3}};
  EXPECT_EQ(policy.applyPolicy(db).size(), 1u);
  bool threw = false;
  try {
    RibPolicy({});
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  EXPECT_TRUE(threw);
  EXPECT_FALSE(RibPolicy({st}, 0).isActive());
}

// --- BASELINE config 4 routes: WAN + UCMP (RibPolicy set_weight), engine vs oracle ------
// The WAN of SURVEY.md §8d row 4 (openr_topogen_wan, std::mt19937_64) as AdjacencyDatabases;
// every node originates one prefix; SpfSolver builds the route DBs over ENGINE SPF results
// (one all-sources prefetch) and RibPolicy applies the UCMP weights (default 1, neighbour
// wan{i} weight 1 + i % 4 for i % 3 == 0). Expected routes are rebuilt here from ORACLE
// SPF runs (oracle/spf_oracle.c) with the reference's next-hop rules: shortest next-hop
// nodes of dst (Decision.cpp:1160-1166), LFA neighbours per RFC 5286 (:1170-1204), link
// expansion with the distOverLink == minMetric filter when LFA is off (:1224-1257), i32
// metric, and the RibPolicy weight precedence (RibPolicy.cpp:61-111).
namespace {
struct Wan {
  std::unordered_map<std::string, LinkState> als;
  PrefixState ps;
  std::vector<std::string> names;
  std::vector<thrift::IpPrefix> prefix;
  Wan(uint32_t n, uint32_t L, uint32_t par, uint64_t seed, bool nodeLabels = false, bool ksp2 = false) {
    std::vector<uint32_t> ends(2 * (L + par)), muv(L + par), mvu(L + par);
    EXPECT_EQ(openr_topogen_wan(n, L, 64, seed, par, ends.data(), muv.data(), mvu.data()), 0);
    std::vector<std::vector<thrift::Adjacency>> adjs(n);
    std::map<std::pair<uint32_t, uint32_t>, int> k;
    auto nm = [](uint32_t i) { return "wan" + std::to_string(i); };
    for (uint32_t l = 0; l < L + par; ++l) {
      const uint32_t u = ends[2 * l], v = ends[2 * l + 1];
      const int kk = k[{std::min(u, v), std::max(u, v)}]++;
      const std::string iu = "if_" + std::to_string(u) + "_" + std::to_string(v) + "_" + std::to_string(kk);
      const std::string iv = "if_" + std::to_string(v) + "_" + std::to_string(u) + "_" + std::to_string(kk);
      adjs[u].push_back(createAdjacency(nm(v), iu, iv, "fe80::" + std::to_string(v), "10.0.0." + std::to_string(v % 256),
                                        (int32_t)muv[l], 0));
      adjs[v].push_back(createAdjacency(nm(u), iv, iu, "fe80::" + std::to_string(u), "10.0.0." + std::to_string(u % 256),
                                        (int32_t)mvu[l], 0));
    }
    als.emplace(kDefaultArea, LinkState(kDefaultArea));
    for (uint32_t i = 0; i < n; ++i) {
      names.push_back(nm(i));
      als.at(kDefaultArea).updateAdjacencyDatabase(createAdjDb(nm(i), adjs[i], nodeLabels ? 100 + (int32_t)i : 0));
      prefix.push_back(pfx("fd00::" + std::to_string(i) + "/128"));
      ps.updatePrefix(nm(i), kDefaultArea, createPrefixEntry(prefix.back(), ksp2));
    }
  }
  RibPolicy policy() const {
    RibPolicyStatement st;
    st.name = "wan-ucmp";
    st.prefixes = std::set<thrift::IpPrefix>(prefix.begin(), prefix.end());
    st.defaultWeight = 1;
    for (uint32_t i = 0; i < names.size(); i += 3) st.neighborToWeight[names[i]] = 1 + (int32_t)(i % 4);
    return RibPolicy({st});
  }
};

// oracle SPF rows of the CSR mirror, memoized per source id
struct OracleRows {
  const LinkState::CsrMirror& m;
  oracle_graph og;
  std::map<uint32_t, std::pair<std::vector<uint64_t>, std::vector<uint8_t>>> rows;
  uint32_t nb;
  explicit OracleRows(const LinkState::CsrMirror& mm)
      : m(mm),
        og{(uint32_t)mm.names.size(), (uint32_t)mm.col.size(), (uint32_t)mm.links.size(), mm.rowPtr.data(),
           mm.col.data(), mm.metric.data(), mm.linkId.data(), mm.edgeUp.data(), mm.overloaded.data(),
           mm.nameRank.data()} {
    uint32_t mx = 1;
    for (uint32_t u = 0; u < og.num_nodes; ++u) mx = std::max(mx, oracle_num_distinct_neighbors(&og, u));
    nb = (mx + 7) / 8;
  }
  const std::pair<std::vector<uint64_t>, std::vector<uint8_t>>& of(uint32_t s) {
    auto it = rows.find(s);
    if (it != rows.end()) return it->second;
    std::vector<uint64_t> d(og.num_nodes);
    std::vector<uint8_t> h((size_t)og.num_nodes * nb);
    EXPECT_TRUE(oracle_run_spf(&og, s, 1, nullptr, d.data(), h.data(), nb, nullptr, nullptr, nullptr) >= 0);
    return rows.emplace(s, std::make_pair(std::move(d), std::move(h))).first->second;
  }
};

NextHopSet expectedRoute(OracleRows& o, uint32_t me, uint32_t dst, bool lfa, const RibPolicy& pol,
                         const thrift::IpPrefix& p) {
  const auto& m = o.m;
  const auto& [dm, hm] = o.of(me);
  NextHopSet out;
  if (dst == me || dm[dst] == UINT64_MAX) return out;
  std::vector<uint32_t> nbrs;  // distinct neighbours of me in row order (next-hop bit order)
  for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e)
    if (std::find(nbrs.begin(), nbrs.end(), m.col[e]) == nbrs.end()) nbrs.push_back(m.col[e]);
  std::map<uint32_t, uint64_t> nhNodes;  // next-hop node -> its distance to dst
  for (size_t i = 0; i < nbrs.size(); ++i)
    if ((hm[(size_t)dst * o.nb + i / 8] >> (i % 8)) & 1u) nhNodes[nbrs[i]] = dm[dst] - dm[nbrs[i]];
  if (lfa) {
    for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e) {
      if (!m.edgeUp[e]) continue;
      const uint32_t n = m.col[e];
      const auto& dn = o.of(n).first;
      if (dn[dst] == UINT64_MAX) continue;
      if (dn[dst] < dm[dst] + dn[me]) {
        auto it = nhNodes.find(n);
        if (it == nhNodes.end() || it->second > dn[dst]) nhNodes[n] = dn[dst];
      }
    }
  }
  for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e) {
    const uint32_t n = m.col[e];
    auto it = nhNodes.find(n);
    if (it == nhNodes.end() || !m.edgeUp[e]) continue;
    const uint64_t over = m.metric[e] + it->second;
    if (!lfa && over != dm[dst]) continue;
    const auto& link = m.links[m.linkId[e]];
    const auto& meName = m.names[me];
    out.insert(createNextHop(link->getNhV6FromNode(meName), link->getIfaceFromNode(meName), (int32_t)over,
                             std::nullopt, kDefaultArea, m.names[n]));
  }
  RibUnicastEntry r;
  r.prefix = p;
  r.nexthops = out;
  pol.applyAction(r);
  return r.nexthops;
}

void wanUcmpRoutes(Wan& w, const std::vector<uint32_t>& nodeIdx, bool lfa) {
  SpfSolver solver(w.names[0], false, lfa);
  const auto pol = w.policy();
  std::vector<std::string> nodes;
  for (auto i : nodeIdx) nodes.push_back(w.names[i]);
  auto dbs = solver.buildRouteDbs(nodes, w.als, w.ps);
  auto const& m = w.als.at(kDefaultArea).csrMirror();
  OracleRows o(m);
  std::map<std::string, uint32_t> prefixOwner;
  for (uint32_t i = 0; i < w.names.size(); ++i) prefixOwner[w.prefix[i].toString()] = m.id.at(w.names[i]);
  size_t routes = 0, weighted = 0, lfaExtra = 0;
  bool allSame = true;
  for (size_t k = 0; k < nodes.size(); ++k) {
    EXPECT_TRUE(dbs[k].has_value());
    if (!dbs[k]) continue;
    auto uni = dbs[k]->unicastRoutes;
    pol.applyPolicy(uni);
    const uint32_t me = m.id.at(nodes[k]);
    EXPECT_EQ(uni.size(), w.names.size() - 1);  // every other node's prefix (the WAN is connected)
    for (auto const& [p, route] : uni) {
      const uint32_t dst = prefixOwner.at(p.toString());
      const auto want = expectedRoute(o, me, dst, lfa, pol, p);
      allSame &= route.nexthops == want;
      ++routes;
      for (auto const& nh : route.nexthops) {
        weighted += nh.weight > 1;
        lfaExtra += nh.metric != route.nexthops.begin()->metric;
      }
    }
  }
  EXPECT_TRUE(allSame);
  EXPECT_TRUE(routes > 0 && weighted > 0);  // UCMP weights present
  if (lfa) EXPECT_TRUE(lfaExtra > 0);       // real loop-free alternates present
  std::printf("  wan routes: %zu, next hops with weight > 1: %zu, lfa: %d, alternates: %zu\n", routes, weighted,
              (int)lfa, lfaExtra);
}
}  // namespace

TEST_GPU(WanUcmpRoutes_vs_Oracle_256) {  // all nodes, parallel links
  Wan w(256, 768, 15, 3);
  std::vector<uint32_t> all(256);
  for (uint32_t i = 0; i < 256; ++i) all[i] = i;
  wanUcmpRoutes(w, all, false);
  wanUcmpRoutes(w, all, true);
}

TEST_GPU(WanUcmpRoutes_vs_Oracle_Config4) {  // the config-4 WAN (1000 nodes, 3000 links)
  Wan w(1000, 3000, 0, 1);
  std::vector<uint32_t> sample;
  for (uint32_t i = 0; i < 1000; i += 63) sample.push_back(i);
  wanUcmpRoutes(w, sample, false);
  wanUcmpRoutes(w, sample, true);
}

// GridTopology.StressTest (DecisionTest.cpp:4358-4372): 99 x 99 grid, LFA on, the route
// DB of node "523" — timed, and every unicast route checked against routes rebuilt from
// oracle SPF runs (shortest next hops + RFC 5286 alternates), plus the label routes.
TEST_GPU(GridTopology_StressTest) {
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  PrefixState ps;
  const auto t0 = std::chrono::steady_clock::now();
  createGrid(als.at(kDefaultArea), ps, 99);
  const auto t1 = std::chrono::steady_clock::now();
  SpfSolver solver("1", false, true);
  SpfCounters::get().reset();
  auto db = solver.buildRouteDb("523", als, ps);
  const auto t2 = std::chrono::steady_clock::now();
  EXPECT_TRUE(db.has_value());
  if (!db) return;
  EXPECT_EQ(99u * 99u - 1u, (unsigned)db->unicastRoutes.size());
  EXPECT_EQ(99u * 99u + 4u, (unsigned)db->mplsRoutes.size());  // node labels + 523's four adjacency labels
  EXPECT_EQ(5u, (unsigned)SpfCounters::get().spfRuns());       // 523 and its four LFA neighbours
  auto const& m = als.at(kDefaultArea).csrMirror();
  OracleRows o(m);
  RibPolicyStatement none;  // a policy that matches no route: applyAction leaves next hops as they are
  none.name = "none";
  none.prefixes = {pfx("fd99::1/128")};
  const RibPolicy pol({none});
  const uint32_t me = m.id.at("523");
  bool ok = true;
  size_t alternates = 0;
  for (auto const& [p, route] : db->unicastRoutes) {
    const std::string ps6 = p.toString();  // fc00::<node>/128
    const uint32_t dst = m.id.at(ps6.substr(6, ps6.size() - 10));
    ok &= route.nexthops == expectedRoute(o, me, dst, true, pol, p);
    for (auto const& nh : route.nexthops) alternates += nh.metric != route.nexthops.begin()->metric;
  }
  EXPECT_TRUE(ok);
  std::printf("  99x99 grid: createGrid %.1f ms, buildRouteDb(\"523\") with LFA %.1f ms, %zu routes, %zu alternates\n",
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count(), db->unicastRoutes.size(), alternates);
}

// buildRouteDbs on host worker threads (HostParallel.h) against the one-thread loop: the
// same route DBs (unicast + node-label MPLS routes, LFA on), counters and best-route
// cache; an unknown node and a repeated node in the list.
std::string flatten(const std::optional<DecisionRouteDb>& db) {
  if (!db) return "none";
  std::string s;
  auto nhs = [&](const NextHopSet& set) {
    for (auto const& nh : set)
      s += nh.address.addr + "%" + nh.address.ifName.value_or("") + "@" + nh.neighborNodeName.value_or("") + "#" +
           std::to_string(nh.metric) + "w" + std::to_string(nh.weight) +
           (nh.mplsAction ? "a" + std::to_string((int)nh.mplsAction->action) : "") +
           (nh.mplsAction && nh.mplsAction->swapLabel ? "s" + std::to_string(*nh.mplsAction->swapLabel) : "") +
           (nh.mplsAction && nh.mplsAction->pushLabels ? "p" + std::to_string(nh.mplsAction->pushLabels->size()) : "") +
           (nh.area ? "@" + *nh.area : "") + ";";
  };
  for (auto const& [p, r] : db->unicastRoutes) {
    s += p.toString() + "[" + r.bestArea + "]";
    nhs(r.nexthops);
    s += "\n";
  }
  for (auto const& [l, r] : db->mplsRoutes) {
    s += std::to_string(l) + ":";
    nhs(r.nexthops);
    s += "\n";
  }
  return s;
}

TEST_GPU(BuildRouteDbs_HostThreads_MatchSequential) {
  Wan w(300, 900, 10, 5, true);
  std::vector<std::string> nodes;
  for (uint32_t i = 0; i < 300; i += 2) nodes.push_back(w.names[i]);
  nodes.push_back("not-a-node");
  nodes.push_back(w.names[7]);
  nodes.push_back("not-a-node-either");  // last entry unknown: the cache is the last known node's
  auto run = [&](const char* threads) {
    setenv("OPENR_HOST_THREADS", threads, 1);
    Wan fresh(300, 900, 10, 5, true);  // cold SPF memo per run
    SpfSolver solver(fresh.names[0], false, true);
    auto dbs = solver.buildRouteDbs(nodes, fresh.als, fresh.ps);
    std::vector<std::string> flat;
    size_t mpls = 0;
    for (auto const& db : dbs) {
      flat.push_back(flatten(db));
      if (db) mpls += db->mplsRoutes.size();
    }
    std::string cache;
    for (auto const& [p, b] : solver.getBestRoutesCache()) {
      cache += p.toString() + (b.success ? "+" : "-") + b.bestNodeArea.first + ":";
      for (auto const& na : b.allNodeAreas) cache += na.first + ",";
    }
    auto const& c = solver.counters();
    std::vector<uint64_t> cnt{c.route_build_runs,     c.get_route_for_prefix, c.no_route_to_prefix,
                              c.skipped_unicast_route, c.skipped_mpls_route,   c.duplicate_node_label,
                              c.no_route_to_label,     c.incompatible_forwarding_type};
    return std::make_tuple(flat, cache, cnt, mpls);
  };
  const auto seq = run("1");
  const auto par = run("6");
  unsetenv("OPENR_HOST_THREADS");
  EXPECT_EQ(std::get<0>(seq).size(), nodes.size());
  EXPECT_TRUE(std::get<0>(seq) == std::get<0>(par));
  EXPECT_TRUE(std::get<0>(seq)[nodes.size() - 3] == "none");
  EXPECT_TRUE(!std::get<1>(seq).empty() && std::get<1>(seq) == std::get<1>(par));
  EXPECT_TRUE(std::get<2>(seq) == std::get<2>(par));
  EXPECT_EQ(std::get<2>(seq)[0], (uint64_t)nodes.size() - 2);
  EXPECT_TRUE(std::get<3>(seq) > 0);  // node-label routes present
}

// The id-based fast path of buildRouteDb (single-advertiser SP_ECMP prefixes and node-label
// MPLS routes on dense rows, Decision.h FastCtx) against the general path on the same
// memoised SPFs: identical unicast / MPLS routes, counters and best-route cache, LFA on and
// off, v4 on and off, with parallel links, asymmetric metrics, node labels, a v4 prefix, a
// prefix with two advertisers and one advertised by an unknown node.
TEST_GPU(RouteBuild_FastPath_MatchesGeneralPath) {
  Wan w(200, 600, 10, 11, true);
  w.ps.updatePrefix(w.names[5], kDefaultArea, createPrefixEntry(pfx("10.1.0.0/16")));
  w.ps.updatePrefix(w.names[7], kDefaultArea, createPrefixEntry(pfx("fd77::/64")));
  w.ps.updatePrefix(w.names[9], kDefaultArea, createPrefixEntry(pfx("fd77::/64")));
  w.ps.updatePrefix("ghost", kDefaultArea, createPrefixEntry(pfx("fd88::/64")));
  std::vector<std::string> nodes;
  for (uint32_t i = 0; i < 200; i += 9) nodes.push_back(w.names[i]);
  for (const bool lfa : {false, true})
    for (const bool v4 : {false, true}) {
      auto run = [&](bool fast) {
        SpfSolver solver(nodes[0], v4, lfa);
        solver.setFastPathForTesting(fast);
        std::vector<std::string> flat;
        for (auto const& n : nodes) flat.push_back(flatten(solver.buildRouteDb(n, w.als, w.ps)));
        std::string cache;
        for (auto const& [p, b] : solver.getBestRoutesCache()) {
          cache += p.toString() + (b.success ? "+" : "-") + b.bestNodeArea.first + ":";
          for (auto const& na : b.allNodeAreas) cache += na.first + ",";
        }
        auto const& c = solver.counters();
        std::vector<uint64_t> cnt{c.route_build_runs,     c.get_route_for_prefix, c.no_route_to_prefix,
                                  c.skipped_unicast_route, c.skipped_mpls_route,   c.duplicate_node_label,
                                  c.no_route_to_label,     c.incompatible_forwarding_type};
        return std::make_tuple(flat, cache, cnt);
      };
      const auto general = run(false), fast = run(true);
      EXPECT_TRUE(std::get<0>(general) == std::get<0>(fast));
      EXPECT_TRUE(std::get<1>(general) == std::get<1>(fast));
      EXPECT_TRUE(std::get<2>(general) == std::get<2>(fast));
      EXPECT_TRUE(std::get<0>(fast)[0].find(":fe80") != std::string::npos);  // label routes present
    }
}

// fastRoute's fallback: with LFA on, the fast path needs every
// neighbour's row on my mirror. A neighbour whose memo row was kept on a retired mirror
// snapshot (a new node nobody reciprocates rebuilds the mirror, not the memo) makes
// fastNextHopNodes return -1, and the rest of the build takes the general path. Routes,
// the best-route cache and the counters must equal an all-general build's.
TEST_GPU(FastRoute_FallbackOnRetiredNeighbourRow) {
  auto run = [&](bool fast, bool v4) {
    Ring r(v4, false);
    auto& ls = r.als.at(kDefaultArea);
    (void)ls.getSpfResult("2");  // neighbour 2's memo row, on the current mirror
    EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("5", {createAdjacency("1", "5/1", "1/5", "fe80::1", "192.168.0.1", 10, 0)}, 5))
                     .topologyChanged);
    SpfSolver solver("1", v4, true);  // LFA: the build reads the neighbours' rows
    solver.setFastPathForTesting(fast);
    std::vector<std::string> flat{flatten(solver.buildRouteDb("1", r.als, r.ps))};
    auto route = solver.createRouteForPrefix("1", r.als, r.ps, v4 ? addr4V4 : addr4);
    flat.push_back(route ? flatten(DecisionRouteDb{{{route->prefix, *route}}, {}}) : "none");
    std::string cache;
    for (auto const& [p, b] : solver.getBestRoutesCache()) {
      cache += p.toString() + (b.success ? "+" : "-") + b.bestNodeArea.first + ":";
      for (auto const& na : b.allNodeAreas) cache += na.first + ",";
    }
    auto const& c = solver.counters();
    std::vector<uint64_t> cnt{c.route_build_runs, c.get_route_for_prefix, c.no_route_to_prefix, c.skipped_unicast_route,
                              c.skipped_mpls_route, c.duplicate_node_label, c.no_route_to_label};
    return std::make_tuple(flat, cache, cnt, solver.fastFallbacksForTesting());
  };
  for (const bool v4 : {false, true}) {
    const auto general = run(false, v4), fast = run(true, v4);
    EXPECT_EQ(std::get<3>(general), 0u);
    EXPECT_EQ(std::get<3>(fast), 1u);  // the fallback was taken
    EXPECT_TRUE(std::get<0>(general) == std::get<0>(fast));
    EXPECT_TRUE(std::get<1>(general) == std::get<1>(fast));
    EXPECT_TRUE(std::get<2>(general) == std::get<2>(fast));
    EXPECT_TRUE(std::get<0>(fast)[1] != "none");
  }
}

// createRouteForPrefix outside buildRouteDb (Decision::rebuildRoutes on an
// incremental prefix update, DecisionTest-style) after LinkState updates must read the
// current SPF memo, not views a previous build cached: a new node with no up link (mirror
// rebuild) and a metric change (memo cleared, rows patched) between the two calls.
TEST_GPU(CreateRouteForPrefix_AfterLinkStateUpdate) {
  Ring r(false, false);
  auto& ls = r.als.at(kDefaultArea);
  SpfSolver solver("1", false, false);
  auto db = solver.buildRouteDb("1", r.als, r.ps);
  EXPECT_TRUE(db.has_value());
  EXPECT_EQ(db->unicastRoutes.at(addr4).nexthops, NextHopSet({nhFromAdj(adj12, false, 20), nhFromAdj(adj13, false, 20)}));
  // a new node whose adjacency nobody reciprocates, then 1 -> 2 gets metric 30
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("5", {createAdjacency("1", "5/1", "1/5", "fe80::1", "192.168.0.1", 10, 0)}, 5))
                   .topologyChanged);
  const auto adj12m = createAdjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 30, 100002);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("1", {adj12m, adj13}, 1)).topologyChanged);
  const uint64_t calls0 = solver.counters().get_route_for_prefix;
  auto route = solver.createRouteForPrefix("1", r.als, r.ps, addr4);
  EXPECT_TRUE(route.has_value());
  if (route) EXPECT_EQ(route->nexthops, NextHopSet({nhFromAdj(adj13, false, 20)}));
  EXPECT_EQ(calls0 + 1, solver.counters().get_route_for_prefix);
  auto r2 = solver.createRouteForPrefix("1", r.als, r.ps, addr2);  // 1 -> 2: via 3 and 4 (30) ties the direct link
  SpfSolver fresh("1", false, false);
  auto want = fresh.buildRouteDb("1", r.als, r.ps);
  EXPECT_TRUE(r2.has_value() && want.has_value());
  if (r2 && want) EXPECT_EQ(r2->nexthops, want->unicastRoutes.at(addr2).nexthops);
  if (route && want) EXPECT_EQ(route->nexthops, want->unicastRoutes.at(addr4).nexthops);
  // and a build after the calls still serves the same routes as a fresh solver
  auto again = solver.buildRouteDb("1", r.als, r.ps);
  EXPECT_TRUE(again.has_value() && want.has_value() && again->unicastRoutes.size() == want->unicastRoutes.size());
  if (again && want)
    for (auto const& [p, e] : want->unicastRoutes) EXPECT_EQ(again->unicastRoutes.at(p).nexthops, e.nexthops);
}

// KSP2 route DBs with the batched device prefetch (LinkState::prefetchKthPaths) against
// the call-by-call getKthPaths path: same routes (SR-MPLS push labels, parallel links),
// same decision.spf_runs, same memoised k-th paths afterwards.
TEST_GPU(Ksp2RouteBuild_Prefetch_MatchesCallByCall) {
  std::vector<uint32_t> picks{0, 17, 123, 250};
  auto run = [&](const char* prefetch) {
    setenv("OPENR_KSP2_PREFETCH", prefetch, 1);
    Wan w(300, 900, 10, 9, true, true);
    SpfSolver solver(w.names[0], false, false);
    std::vector<std::string> nodes;
    for (auto i : picks) nodes.push_back(w.names[i]);
    const uint64_t runs0 = SpfCounters::get().spfRuns();
    const auto t0 = std::chrono::steady_clock::now();
    auto dbs = solver.buildRouteDbs(nodes, w.als, w.ps);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const uint64_t runs = SpfCounters::get().spfRuns() - runs0;
    std::vector<std::string> flat;
    size_t routes = 0, pushes = 0;
    for (auto const& db : dbs) {
      flat.push_back(flatten(db));
      if (!db) continue;
      routes += db->unicastRoutes.size();
      for (auto const& [p, r] : db->unicastRoutes)
        for (auto const& nh : r.nexthops) pushes += nh.mplsAction && nh.mplsAction->pushLabels.has_value();
    }
    std::string memo;  // k-th paths memoised for a sample of pairs, as link strings
    auto const& ls = w.als.at(kDefaultArea);
    for (auto i : picks)
      for (uint32_t d = 1; d < 300; d += 37)
        for (size_t k = 1; k <= 2; ++k) {
          for (auto const& path : ls.getKthPaths(w.names[i], w.names[d], k)) {
            for (auto const& l : path) memo += l->toString() + ",";
            memo += "|";
          }
          memo += "\n";
        }
    std::printf("  prefetch=%s: %zu routes, %zu push next hops, spf_runs %llu, %.1f ms\n", prefetch, routes, pushes,
                (unsigned long long)runs, ms);
    return std::make_tuple(flat, runs, memo, routes, pushes);
  };
  const auto off = run("0");
  const auto on = run("1");
  unsetenv("OPENR_KSP2_PREFETCH");
  EXPECT_TRUE(std::get<0>(off) == std::get<0>(on));
  EXPECT_EQ(std::get<1>(off), std::get<1>(on));
  EXPECT_TRUE(std::get<2>(off) == std::get<2>(on));
  EXPECT_EQ(std::get<3>(on), picks.size() * 299);
  EXPECT_TRUE(std::get<4>(on) > 0);
}

// HostParallel.h: every item runs exactly once on some worker; an error reports the lowest
// failing index, as the one-thread loop would; OPENR_HOST_THREADS bounds the workers.
TEST_CPU(HostParallel_ParallelFor) {
  const size_t n = 10007;
  std::vector<std::atomic<int>> hits(n);
  for (auto& h : hits) h = 0;
  std::atomic<unsigned> maxWorker{0};
  parallelFor(n, 7, 6, [&](unsigned w, size_t i) {
    hits[i]++;
    unsigned m = maxWorker.load();
    while (w > m && !maxWorker.compare_exchange_weak(m, w)) {
    }
  });
  bool once = true;
  for (auto& h : hits) once &= h.load() == 1;
  EXPECT_TRUE(once);
  EXPECT_TRUE(maxWorker.load() < 6u);
  for (unsigned workers : {1u, 4u}) {
    std::string what;
    try {
      parallelFor(n, 3, workers, [&](unsigned, size_t i) {
        if (i == 777 || i == 5000) throw std::runtime_error("item " + std::to_string(i));
      });
    } catch (const std::runtime_error& e) {
      what = e.what();
    }
    EXPECT_TRUE(what == "item 777");
  }
  setenv("OPENR_HOST_THREADS", "3", 1);
  EXPECT_EQ(hostThreads(), 3u);
  EXPECT_EQ(parallelWorkers(100, 50), 2u);
  setenv("OPENR_HOST_THREADS", "1", 1);
  EXPECT_EQ(parallelWorkers(1000, 1), 1u);
  unsetenv("OPENR_HOST_THREADS");
  EXPECT_TRUE(hostThreads() >= 1u && hostThreads() <= 16u);
}

// --- RibPolicyTest.cpp:176-301 (RibPolicy.ApplyAction / ApplyPolicy) -----------------
namespace {
RibPolicyStatement policyStatement(std::vector<thrift::IpPrefix> prefixes, int32_t dflt,
                                   std::unordered_map<std::string, int32_t> area,
                                   std::unordered_map<std::string, int32_t> nbr = {}) {  // :23-37
  RibPolicyStatement p;
  p.name = "TestPolicyStatement";
  p.prefixes = std::set<thrift::IpPrefix>(prefixes.begin(), prefixes.end());
  p.defaultWeight = dflt;
  p.areaToWeight = std::move(area);
  p.neighborToWeight = std::move(nbr);
  return p;
}
thrift::BinaryAddress binAddr(const std::string& a) {
  thrift::BinaryAddress b;
  b.addr = a;
  return b;
}
}  // namespace

// UtilTest.cpp:911-972 MetricVectorUtilsTest.compareMetricVectors
TEST_CPU(MetricVectorUtils_compareMetricVectors) {
  using MetricVectorUtils::CompareResult;
  using MetricVectorUtils::compareMetricVectors;
  thrift::MetricVector l, r;
  EXPECT_TRUE(CompareResult::TIE == compareMetricVectors(l, r));
  l.version = 1;
  r.version = 2;
  EXPECT_TRUE(CompareResult::ERROR == compareMetricVectors(l, r));
  r.version = 1;
  const int64_t n = 5;
  l.metrics.resize(n);
  r.metrics.resize(n);
  for (int64_t i = 0; i < n; ++i)
    for (auto* v : {&l, &r}) v->metrics[i] = {i, i, thrift::CompareType::WIN_IF_PRESENT, false, {i}};
  EXPECT_TRUE(CompareResult::TIE == compareMetricVectors(l, r));
  r.metrics[n - 2].metric.front()--;
  EXPECT_TRUE(CompareResult::WINNER == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::LOOSER == compareMetricVectors(r, l));
  r.metrics[n - 2].isBestPathTieBreaker = true;
  EXPECT_TRUE(CompareResult::ERROR == compareMetricVectors(l, r));
  l.metrics[n - 2].isBestPathTieBreaker = true;
  EXPECT_TRUE(CompareResult::TIE_WINNER == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::TIE_LOOSER == compareMetricVectors(r, l));
  r.metrics.resize(n - 1);
  EXPECT_TRUE(CompareResult::WINNER == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::LOOSER == compareMetricVectors(r, l));
  l.metrics[0].type--;  // same priority, different type
  EXPECT_TRUE(CompareResult::ERROR == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::ERROR == compareMetricVectors(r, l));
  l.metrics[0].type++;
  l.metrics[n - 1].op = thrift::CompareType::WIN_IF_NOT_PRESENT;
  EXPECT_TRUE(CompareResult::LOOSER == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::WINNER == compareMetricVectors(r, l));
  l.metrics[n - 1].op = thrift::CompareType::IGNORE_IF_NOT_PRESENT;
  EXPECT_TRUE(CompareResult::TIE_WINNER == compareMetricVectors(l, r));
  EXPECT_TRUE(CompareResult::TIE_LOOSER == compareMetricVectors(r, l));
}

// DecisionTest.cpp:715-897 BGPRedistribution.BasicOperation: BGP routes by metric vector
TEST_GPU(BGPRedistribution_BasicOperation) {
  SpfSolver solver("1", false, false);
  std::unordered_map<std::string, LinkState> als;
  als.emplace(kDefaultArea, LinkState(kDefaultArea));
  auto& ls = als.at(kDefaultArea);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("1", {adj12, adj13}, 0)).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("2", {adj21}, 0)).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("3", {adj31}, 0)).topologyChanged);
  PrefixState ps;
  ps.updatePrefix("1", kDefaultArea, createPrefixEntry(addr1));
  ps.updatePrefix("2", kDefaultArea, createPrefixEntry(addr2));
  thrift::MetricVector mv1, mv2;
  for (int64_t i = 0; i < 5; ++i) {
    mv1.metrics.push_back({i, i, thrift::CompareType::WIN_IF_PRESENT, false, {i}});
    mv2.metrics.push_back({i, i, thrift::CompareType::WIN_IF_PRESENT, false, {i}});
  }
  auto bgp = [](const thrift::MetricVector& mv, const std::string& data) {
    auto e = createPrefixEntry(addr3);
    e.type = thrift::PrefixType::BGP;
    e.data = data;
    e.mv = mv;
    return e;
  };
  auto routeTo = [&](const std::string& node) -> std::optional<RibUnicastEntry> {
    auto db = solver.buildRouteDb(node, als, ps);
    auto it = db->unicastRoutes.find(addr3);
    if (it == db->unicastRoutes.end()) return std::nullopt;
    return it->second;
  };
  auto routes = [&](const std::string& node) { return solver.buildRouteDb(node, als, ps)->unicastRoutes.size(); };
  // only node 1 advertises the BGP prefix: it is the best path
  ps.updatePrefix("1", kDefaultArea, bgp(mv1, "data1"));
  EXPECT_EQ(2u, routes("2"));
  auto r = routeTo("2");
  EXPECT_TRUE(r.has_value());
  if (r) {
    EXPECT_EQ(r->nexthops, NextHopSet({nhFromAdj(adj21, false, adj21.metric)}));
    EXPECT_TRUE(r->bestPrefixEntry.type == thrift::PrefixType::BGP && r->bestPrefixEntry.data == "data1");
    EXPECT_FALSE(r->doNotInstall);
  }
  // node 2 with the same metric vector: no best path, the route goes; the tie is logged,
  // not counted (Decision.cpp:830-837, createRouteForPrefix :503-505)
  ps.updatePrefix("2", kDefaultArea, bgp(mv2, "data2"));
  const uint64_t skipped0 = solver.counters().skipped_unicast_route;
  EXPECT_EQ(1u, routes("1"));
  EXPECT_EQ(skipped0, solver.counters().skipped_unicast_route);
  // node 2's last metric lower: node 1 again
  mv2.metrics[4].metric.front()--;
  ps.updatePrefix("2", kDefaultArea, bgp(mv2, "data2"));
  EXPECT_EQ(2u, routes("2"));
  r = routeTo("2");
  EXPECT_TRUE(r && r->bestPrefixEntry.data == "data1" && r->nexthops == NextHopSet({nhFromAdj(adj21, false, 10)}));
  // node 2 better
  mv2.metrics[4].metric.front() += 2;
  ps.updatePrefix("2", kDefaultArea, bgp(mv2, "data2"));
  EXPECT_EQ(2u, routes("1"));
  r = routeTo("1");
  EXPECT_TRUE(r && r->bestPrefixEntry.data == "data2" && r->nexthops == NextHopSet({nhFromAdj(adj12, false, 10)}));
  // the last entity a tie breaker: multipath over both advertisers
  mv1.metrics[4].isBestPathTieBreaker = true;
  mv2.metrics[4].isBestPathTieBreaker = true;
  ps.updatePrefix("1", kDefaultArea, bgp(mv1, "data1"));
  ps.updatePrefix("2", kDefaultArea, bgp(mv2, "data2"));
  EXPECT_EQ(1u, routes("1"));  // 1 and 2 advertise it themselves: no route
  EXPECT_EQ(3u, routes("3"));
  r = routeTo("3");
  EXPECT_TRUE(r && r->bestPrefixEntry.data == "data2" && r->nexthops == NextHopSet({nhFromAdj(adj31, false, 10)}));
  // disconnected: each node considers its own BGP route best and programs nothing
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("1", {}, 0)).topologyChanged);
  EXPECT_FALSE(routeTo("1").has_value());
  EXPECT_FALSE(routeTo("2").has_value());
  // a BGP advertiser without a metric vector: the route is skipped
  auto noMv = bgp(mv1, "data1");
  noMv.mv.reset();
  ps.updatePrefix("1", kDefaultArea, noMv);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(createAdjDb("1", {adj12, adj13}, 0)).topologyChanged);
  EXPECT_FALSE(routeTo("3").has_value());
}

// The route containers (sorted vectors with the reference's map / set semantics): keys
// kept unique and ordered whatever the insertion order, insert_or_assign overwriting,
// emplace not, lookups and erasure.
TEST_CPU(RouteContainers_MapAndSetSemantics) {
  MplsRoutes m;
  for (int32_t k : {30, 10, 20, 40, 10}) m.emplace(k, RibMplsEntry{k, {}});
  EXPECT_EQ(m.size(), 4u);
  std::vector<int32_t> keys;
  for (auto const& [k, e] : m) keys.push_back(k);
  EXPECT_TRUE((keys == std::vector<int32_t>{10, 20, 30, 40}));
  m.insert_or_assign(20, RibMplsEntry{99, {}});
  EXPECT_EQ(m.at(20).label, 99);
  m.emplace(20, RibMplsEntry{7, {}});  // present: unchanged
  EXPECT_EQ(m.at(20).label, 99);
  m.insert_or_assign(25, RibMplsEntry{25, {}});
  EXPECT_EQ(std::next(m.begin(), 2)->first, 25);
  EXPECT_EQ(m.count(25), 1u);
  EXPECT_EQ(m.erase(25), 1u);
  EXPECT_EQ(m.erase(25), 0u);
  EXPECT_TRUE(m.find(25) == m.end());
  EXPECT_THROW(m.at(25));
  EXPECT_EQ(m[50].label, 0);  // default-constructed on first access
  EXPECT_EQ(m.size(), 5u);

  thrift::NextHopThrift a, b, c;
  a.address.addr = "a";
  b.address.addr = "b";
  c.address.addr = "c";
  NextHopSet s{c, a, b, a};
  EXPECT_EQ(s.size(), 3u);
  EXPECT_TRUE(s.begin()->address.addr == "a" && std::prev(s.end())->address.addr == "c");
  EXPECT_FALSE(s.insert(b).second);
  thrift::NextHopThrift b5 = b;
  b5.metric = 5;  // a different next hop
  EXPECT_TRUE(s.emplace(b5).second);
  EXPECT_EQ(s.size(), 4u);
  EXPECT_EQ(s.count(b5), 1u);
  EXPECT_EQ(s.erase(b5), 1u);
  EXPECT_TRUE((s == NextHopSet{b, c, a}));
}

TEST_CPU(RibPolicyTest_ApplyAction) {  // :180-236 only the first matching statement applies
  const auto stmt1 = policyStatement({pfx("fc01::/64")}, 1, {{"area1", 99}});
  const auto stmt2 = policyStatement({pfx("fc00::/64"), pfx("fc02::/64")}, 1, {{"area2", 99}});
  RibPolicy policy({stmt1, stmt2}, 1);
  const auto nh1 = createNextHop(binAddr("fe80::1"), std::string("iface1"), 0, std::nullopt, std::string("area1"));
  const auto nh2 = createNextHop(binAddr("fe80::1"), std::string("iface2"), 0, std::nullopt, std::string("area2"));
  {
    RibUnicastEntry e;
    e.prefix = pfx("fc01::/64");
    e.nexthops = {nh1, nh2};
    EXPECT_TRUE(policy.applyAction(e));
    auto x1 = nh1, x2 = nh2;
    x1.weight = 99;
    x2.weight = 1;
    EXPECT_EQ(e.nexthops, NextHopSet({x1, x2}));
  }
  {
    RibUnicastEntry e;
    e.prefix = pfx("fc02::/64");
    e.nexthops = {nh1, nh2};
    EXPECT_TRUE(policy.applyAction(e));
    auto x1 = nh1, x2 = nh2;
    x1.weight = 1;
    x2.weight = 99;
    EXPECT_EQ(e.nexthops, NextHopSet({x1, x2}));
  }
  {
    RibUnicastEntry e;
    e.prefix = pfx("fc03::/64");
    e.nexthops = {nh1, nh2};
    const auto before = e.nexthops;
    EXPECT_FALSE(policy.applyAction(e));
    EXPECT_EQ(e.nexthops, before);
  }
}

TEST_CPU(RibPolicyTest_ApplyPolicy) {  // :238-301 neighbour > area > default, all-dropped kept, TTL
  const auto stmt1 = policyStatement({pfx("fc01::/64")}, 1, {{"area1", 99}}, {{"nbr3", 98}});
  const auto stmt2 = policyStatement({pfx("fc00::/64"), pfx("fc02::/64")}, 1, {{"area2", 0}});
  RibPolicy policy({stmt1, stmt2}, 1);
  const auto nh1 = createNextHop(binAddr("fe80::1"), std::string("iface1"), 0, std::nullopt, std::string("area1"),
                                 std::string("nbr1"));
  const auto nh2 = createNextHop(binAddr("fe80::1"), std::string("iface2"), 0, std::nullopt, std::string("area2"),
                                 std::string("nbr2"));
  const auto nh3 = createNextHop(binAddr("fe80::1"), std::string("iface3"), 0, std::nullopt, std::string("area1"),
                                 std::string("nbr3"));
  RibUnicastEntry e1, e2;
  e1.prefix = pfx("fc01::/64");
  e1.nexthops = {nh1, nh2, nh3};
  e2.prefix = pfx("fc02::/64");
  e2.nexthops = {nh2};
  {
    UnicastRoutes entries{{e1.prefix, e1}, {e2.prefix, e2}};
    const uint64_t inv0 = RibPolicyCounters::get().invalidatedRoutes;
    const auto updated = policy.applyPolicy(entries);
    EXPECT_EQ(updated, std::vector<thrift::IpPrefix>({e1.prefix}));
    EXPECT_EQ(RibPolicyCounters::get().invalidatedRoutes - inv0, 1u);  // fc02: every next-hop weight 0
    EXPECT_EQ(entries.size(), 2u);
    auto x1 = nh1, x2 = nh2, x3 = nh3;
    x1.weight = 99;
    x2.weight = 1;
    x3.weight = 98;
    EXPECT_EQ(entries.at(e1.prefix).nexthops, NextHopSet({x1, x2, x3}));
    EXPECT_EQ(entries.at(e2.prefix).nexthops, e2.nexthops);
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(1100));  // the policy expires
  EXPECT_FALSE(policy.isActive());
  {
    UnicastRoutes entries{{e1.prefix, e1}, {e2.prefix, e2}};
    EXPECT_TRUE(policy.applyPolicy(entries).empty());
    EXPECT_EQ(entries.at(e1.prefix).nexthops, e1.nexthops);
  }
}

int main(int argc, char** argv) { return run_tests(argc, argv); }
