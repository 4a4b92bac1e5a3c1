// linkstate_test.cpp — tests of the C++ host mirror of openr::LinkState.
//
// Transcribes /root/reference/openr/decision/tests/LinkStateTest.cpp and the
// LinkState-level expectations of DecisionTest.cpp (file:line per test), plus
// oracle cross-checks (the oracle is linked here as the checker only).
//   linkstate_test cpu   -> host-only tests (no GPU needed)
//   linkstate_test gpu   -> tests that run SPF on the engine
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../oracle/spf_oracle.h"
#include "harness.h"
#include "../../openr_amd/csrc/host/LinkState.h"
#include "../../openr_amd/csrc/host/AdjDbCodec.h"

using namespace openr;

static const std::string kArea = "0";

static thrift::Adjacency createAdjacency(const std::string& otherNode, const std::string& ifName,
                                         const std::string& otherIfName, int32_t metric, int32_t adjLabel = 0) {
  thrift::Adjacency a;
  a.otherNodeName = otherNode;
  a.ifName = ifName;
  a.otherIfName = otherIfName;
  a.metric = metric;
  a.adjLabel = adjLabel;
  a.nextHopV6.addr = "fe80::" + otherNode;
  a.nextHopV4.addr = "10.0.0." + otherNode;
  return a;
}

static thrift::AdjacencyDatabase createAdjDb(const std::string& node, std::vector<thrift::Adjacency> adjs,
                                             int32_t nodeLabel) {
  thrift::AdjacencyDatabase db;
  db.thisNodeName = node;
  db.adjacencies = std::move(adjs);
  db.nodeLabel = nodeLabel;
  db.area = kArea;
  return db;
}

// getLinkState fixture builder (DecisionTestUtils.cpp:16-42)
static LinkState getLinkState(const std::vector<std::pair<int, std::vector<std::pair<int, int>>>>& adjMap) {
  LinkState ls(kArea);
  for (auto const& [node, adjList] : adjMap) {
    std::vector<thrift::Adjacency> adjs;
    std::map<int, int> numParallel;
    for (auto const& [adj, weight] : adjList) {
      const int k = numParallel[adj]++;
      adjs.push_back(createAdjacency(std::to_string(adj), std::to_string(node) + "/" + std::to_string(adj) + "/" +
                                                             std::to_string(k),
                                     std::to_string(adj) + "/" + std::to_string(node) + "/" + std::to_string(k),
                                     weight, (node << 16) + adj));
    }
    ls.updateAdjacencyDatabase(createAdjDb(std::to_string(node), adjs, node), 0, 0);
  }
  return ls;
}

static std::vector<std::pair<int, std::vector<std::pair<int, int>>>> unit(
    const std::vector<std::pair<int, std::vector<int>>>& m) {
  std::vector<std::pair<int, std::vector<std::pair<int, int>>>> r;
  for (auto const& [n, adjs] : m) {
    std::vector<std::pair<int, int>> w;
    for (int a : adjs) w.emplace_back(a, 1);
    r.emplace_back(n, w);
  }
  return r;
}

// ---------------------------------------------------------------------------
// LinkStateTest.cpp:22-83
TEST_CPU(HoldableValueTest_BasicOperation) {
  HoldableValue<bool> hv{true};
  EXPECT_TRUE(hv.value());
  EXPECT_FALSE(hv.hasHold());
  EXPECT_FALSE(hv.decrementTtl());
  const LinkStateMetric holdUpTtl = 10, holdDownTtl = 5;
  EXPECT_FALSE(hv.updateValue(false, holdUpTtl, holdDownTtl));
  for (LinkStateMetric i = 0; i < holdUpTtl - 1; ++i) {
    EXPECT_TRUE(hv.hasHold());
    EXPECT_TRUE(hv.value());
    EXPECT_FALSE(hv.decrementTtl());
  }
  EXPECT_TRUE(hv.decrementTtl());
  EXPECT_FALSE(hv.hasHold());
  EXPECT_FALSE(hv.value());
  EXPECT_FALSE(hv.updateValue(false, holdUpTtl, holdDownTtl));
  EXPECT_FALSE(hv.hasHold());
  EXPECT_FALSE(hv.value());
  EXPECT_FALSE(hv.updateValue(true, holdUpTtl, holdDownTtl));
  for (LinkStateMetric i = 0; i < holdDownTtl - 1; ++i) {
    EXPECT_TRUE(hv.hasHold());
    EXPECT_FALSE(hv.value());
    EXPECT_FALSE(hv.decrementTtl());
  }
  EXPECT_TRUE(hv.decrementTtl());
  EXPECT_FALSE(hv.hasHold());
  EXPECT_TRUE(hv.value());
  EXPECT_FALSE(hv.updateValue(false, holdUpTtl, holdDownTtl));
  EXPECT_TRUE(hv.hasHold());
  EXPECT_TRUE(hv.value());
  EXPECT_FALSE(hv.decrementTtl());
  EXPECT_TRUE(hv.updateValue(true, holdUpTtl, holdDownTtl));
  EXPECT_FALSE(hv.hasHold());
  EXPECT_TRUE(hv.value());

  HoldableValue<LinkStateMetric> hvLsm{10};
  EXPECT_EQ(10u, hvLsm.value());
  EXPECT_FALSE(hvLsm.hasHold());
  EXPECT_FALSE(hvLsm.decrementTtl());
  EXPECT_FALSE(hvLsm.updateValue(5, holdUpTtl, holdDownTtl));
  for (LinkStateMetric i = 0; i < holdUpTtl - 1; ++i) {
    EXPECT_TRUE(hvLsm.hasHold());
    EXPECT_EQ(10u, hvLsm.value());
    EXPECT_FALSE(hvLsm.decrementTtl());
  }
  EXPECT_TRUE(hvLsm.decrementTtl());
  EXPECT_FALSE(hvLsm.hasHold());
  EXPECT_EQ(5u, hvLsm.value());
}

// LinkStateTest.cpp:85-137
TEST_CPU(LinkTest_BasicOperation) {
  std::string n1 = "node1";
  auto adj1 = createAdjacency(n1, "if1", "if2", 1, 1);
  std::string n2 = "node2";
  auto adj2 = createAdjacency(n2, "if2", "if1", 1, 2);
  Link l1(kArea, n1, adj1, n2, adj2);
  EXPECT_EQ(kArea, l1.getArea());
  EXPECT_EQ(n2, l1.getOtherNodeName(n1));
  EXPECT_EQ(n1, l1.getOtherNodeName(n2));
  EXPECT_THROW(l1.getOtherNodeName("node3"));
  EXPECT_EQ(adj1.ifName, l1.getIfaceFromNode(n1));
  EXPECT_EQ(adj2.ifName, l1.getIfaceFromNode(n2));
  EXPECT_THROW(l1.getIfaceFromNode("node3"));
  EXPECT_EQ((LinkStateMetric)adj1.metric, l1.getMetricFromNode(n1));
  EXPECT_EQ((LinkStateMetric)adj2.metric, l1.getMetricFromNode(n2));
  EXPECT_THROW(l1.getMetricFromNode("node3"));
  EXPECT_EQ(adj1.adjLabel, l1.getAdjLabelFromNode(n1));
  EXPECT_EQ(adj2.adjLabel, l1.getAdjLabelFromNode(n2));
  EXPECT_THROW(l1.getAdjLabelFromNode("node3"));
  EXPECT_FALSE(l1.getOverloadFromNode(n1));
  EXPECT_FALSE(l1.getOverloadFromNode(n2));
  EXPECT_TRUE(l1.isUp());
  EXPECT_TRUE(l1.setMetricFromNode(n1, 2, 0, 0));
  EXPECT_EQ(2u, l1.getMetricFromNode(n1));
  EXPECT_TRUE(l1.setOverloadFromNode(n2, true, 0, 0));
  EXPECT_FALSE(l1.getOverloadFromNode(n1));
  EXPECT_TRUE(l1.getOverloadFromNode(n2));
  EXPECT_FALSE(l1.isUp());
  Link l2(kArea, n2, adj2, n1, adj1);
  EXPECT_TRUE(l1 == l2);
  EXPECT_FALSE(l1 < l2);
  EXPECT_FALSE(l2 < l1);
  std::string n3 = "node3";
  auto adj3 = createAdjacency(n2, "if3", "if2", 1, 1);
  Link l3(kArea, n1, adj1, n3, adj3);
  EXPECT_FALSE(l1 == l3);
  EXPECT_TRUE(l1 < l3 || l3 < l1);
}

static bool sameLinks(const LinkState::LinkSet& set, std::vector<Link> want) {
  if (set.size() != want.size()) return false;
  for (auto const& w : want) {
    bool found = false;
    for (auto const& l : set) found |= (*l == w);
    if (!found) return false;
  }
  return true;
}

// LinkStateTest.cpp:139-200
TEST_CPU(LinkStateTest_BasicOperation) {
  std::string n1 = "node1", n2 = "node2", n3 = "node3";
  auto adj12 = createAdjacency(n2, "if2", "if1", 1, 1);
  auto adj13 = createAdjacency(n3, "if3", "if1", 1, 1);
  auto adj21 = createAdjacency(n1, "if1", "if2", 1, 1);
  auto adj23 = createAdjacency(n3, "if3", "if2", 1, 1);
  auto adj31 = createAdjacency(n1, "if1", "if3", 1, 1);
  auto adj32 = createAdjacency(n2, "if2", "if3", 1, 1);
  Link l1(kArea, n1, adj12, n2, adj21);
  Link l2(kArea, n2, adj23, n3, adj32);
  Link l3(kArea, n3, adj31, n1, adj13);
  auto adjDb1 = createAdjDb(n1, {adj12, adj13}, 1);
  auto adjDb2 = createAdjDb(n2, {adj21, adj23}, 2);
  auto adjDb3 = createAdjDb(n3, {adj31, adj32}, 3);
  LinkState state{kArea};
  EXPECT_EQ(kArea, state.getArea());
  EXPECT_FALSE(state.updateAdjacencyDatabase(adjDb1, 0, 0).topologyChanged);
  EXPECT_TRUE(state.updateAdjacencyDatabase(adjDb2, 0, 0).topologyChanged);
  EXPECT_TRUE(state.updateAdjacencyDatabase(adjDb3, 0, 0).topologyChanged);
  EXPECT_TRUE(sameLinks(state.linksFromNode(n1), {l1, l3}));
  EXPECT_TRUE(sameLinks(state.linksFromNode(n2), {l1, l2}));
  EXPECT_TRUE(sameLinks(state.linksFromNode(n3), {l2, l3}));
  EXPECT_TRUE(state.linksFromNode("node4").empty());
  EXPECT_FALSE(state.isNodeOverloaded(n1));
  adjDb1.isOverloaded = true;
  EXPECT_TRUE(state.updateAdjacencyDatabase(adjDb1, 0, 0).topologyChanged);
  EXPECT_TRUE(state.isNodeOverloaded(n1));
  EXPECT_FALSE(state.updateAdjacencyDatabase(adjDb1, 0, 0).topologyChanged);
  adjDb1.isOverloaded = false;
  EXPECT_TRUE(state.updateAdjacencyDatabase(adjDb1, 0, 0).topologyChanged);
  EXPECT_FALSE(state.isNodeOverloaded(n1));
  adjDb1 = createAdjDb(n1, {adj13}, 1);
  EXPECT_TRUE(state.updateAdjacencyDatabase(adjDb1, 0, 0).topologyChanged);
  EXPECT_TRUE(sameLinks(state.linksFromNode(n1), {l3}));
  EXPECT_TRUE(sameLinks(state.linksFromNode(n2), {l2}));
  EXPECT_TRUE(sameLinks(state.linksFromNode(n3), {l2, l3}));
  EXPECT_TRUE(state.deleteAdjacencyDatabase(n1).topologyChanged);
  EXPECT_TRUE(state.linksFromNode(n1).empty());
  EXPECT_TRUE(sameLinks(state.linksFromNode(n2), {l2}));
  EXPECT_TRUE(sameLinks(state.linksFromNode(n3), {l2}));
}

// Bulk adjacency publication (Decision.cpp:1737-1782 through AdjDbCodec): encoded
// "adj:" values applied in one call give the same LinkState and CSR mirror as direct
// updateAdjacencyDatabase calls; other keys are ignored; a key/node mismatch throws.
TEST_CPU(AdjDbCodec_PublicationMatchesDirectUpdates) {
  std::string n1 = "node1", n2 = "node2", n3 = "node3";
  auto db1 = createAdjDb(n1, {createAdjacency(n2, "if2", "if1", 3, 1), createAdjacency(n3, "if3", "if1", 1, 1)}, 1);
  auto db2 = createAdjDb(n2, {createAdjacency(n1, "if1", "if2", 5, 1), createAdjacency(n3, "if3", "if2", 1, 1)}, 2);
  auto db3 = createAdjDb(n3, {createAdjacency(n1, "if1", "if3", 1, 1), createAdjacency(n2, "if2", "if3", 7, 1)}, 3);
  db2.isOverloaded = true;
  db3.adjacencies[1].isOverloaded = true;
  db1.perfEvents = thrift::PerfEvents{{{n1, "ADJ_DB_UPDATED", 42}}};
  LinkState direct{kArea};
  for (auto const* db : {&db1, &db2, &db3}) direct.updateAdjacencyDatabase(*db, 0, 0);

  std::vector<std::pair<std::string, std::string>> kv;
  for (auto db : {db1, db2, db3}) {
    db.area = "stale";  // Decision stamps the area of the LinkState (Decision.cpp:1762)
    kv.emplace_back("adj:" + db.thisNodeName, serializer::writeAdjacencyDatabase(db));
  }
  kv.emplace_back("prefix:node1:0:[10.0.0.0/8]", "not an adjacency db");
  LinkState bulk{kArea};
  auto res = applyAdjacencyPublication(bulk, kv, 2);
  EXPECT_EQ(res.adjDbsApplied, 3u);
  EXPECT_TRUE(res.topologyChanged);
  EXPECT_EQ(bulk.numLinks(), direct.numLinks());
  EXPECT_EQ(bulk.getAdjacencyDatabases().at(n3).area, kArea);
  auto const& a = direct.csrMirror();
  auto const& b = bulk.csrMirror();
  EXPECT_TRUE(a.names == b.names);
  EXPECT_TRUE(a.rowPtr == b.rowPtr);
  EXPECT_TRUE(a.col == b.col);
  EXPECT_TRUE(a.metric == b.metric);
  EXPECT_TRUE(a.edgeUp == b.edgeUp);
  EXPECT_TRUE(a.overloaded == b.overloaded);
  // a re-advertisement moved in (bulk path) reports and applies the same change as a copy
  auto db1b = db1;
  db1b.adjacencies[0].metric = 9;
  db1b.nodeLabel = 77;
  const auto cd = direct.updateAdjacencyDatabase(db1b, 0, 0);
  const auto cb = bulk.updateAdjacencyDatabase(thrift::AdjacencyDatabase(db1b), 0, 0);
  EXPECT_TRUE(cd.topologyChanged && cb.topologyChanged);
  EXPECT_TRUE(cd.nodeLabelChanged && cb.nodeLabelChanged);
  EXPECT_TRUE(direct.csrMirror().metric == bulk.csrMirror().metric);
  EXPECT_EQ(bulk.getAdjacencyDatabases().at(n1).nodeLabel, 77);
  // decoded struct equals the original, perf events included
  auto rt = serializer::readAdjacencyDatabase(serializer::writeAdjacencyDatabase(db1));
  EXPECT_TRUE(rt.perfEvents.has_value() && rt.perfEvents->events.size() == 1 &&
              rt.perfEvents->events[0].unixTs == 42);
  EXPECT_EQ(rt.adjacencies[0].nextHopV6.addr, db1.adjacencies[0].nextHopV6.addr);
  // key/node mismatch: CHECK_EQ in the reference
  std::vector<std::pair<std::string, std::string>> wrong{{"adj:node9", serializer::writeAdjacencyDatabase(db1)}};
  LinkState other{kArea};
  EXPECT_THROW(applyAdjacencyPublication(other, wrong));
  // a malformed value names its index
  std::vector<std::pair<std::string, std::string>> broken{kv[0], {"adj:node2", kv[1].second.substr(0, 9)}};
  bool named = false;
  try {
    applyAdjacencyPublication(other, broken);
  } catch (const CompactProtocolError& e) {
    named = std::string(e.what()).rfind("value 1:", 0) == 0;
  }
  EXPECT_TRUE(named);
}

// LinkStateTest.cpp:202-242
TEST_CPU(LinkStateTest_pathAInPathB) {
  auto l1 = std::make_shared<Link>(kArea, "1", "1/2", "2", "2/1");
  auto l2 = std::make_shared<Link>(kArea, "2", "2/3", "3", "3/2");
  auto l3 = std::make_shared<Link>(kArea, "1", "1/3", "3", "3/1");
  LinkState::Path p1, p2;
  EXPECT_TRUE(LinkState::pathAInPathB(p1, p2));
  EXPECT_TRUE(LinkState::pathAInPathB(p2, p1));
  p1.push_back(l1);
  EXPECT_FALSE(LinkState::pathAInPathB(p1, p2));
  EXPECT_TRUE(LinkState::pathAInPathB(p2, p1));
  p2.push_back(l1);
  EXPECT_TRUE(LinkState::pathAInPathB(p1, p2));
  EXPECT_TRUE(LinkState::pathAInPathB(p2, p1));
  p1.push_back(l2);
  EXPECT_FALSE(LinkState::pathAInPathB(p1, p2));
  EXPECT_TRUE(LinkState::pathAInPathB(p2, p1));
  p1.push_back(l3);
  p2.push_back(l2);
  EXPECT_FALSE(LinkState::pathAInPathB(p1, p2));
  EXPECT_TRUE(LinkState::pathAInPathB(p2, p1));
  p1.clear();
  p2.clear();
  p1.push_back(l3);
  p1.push_back(l2);
  p2.push_back(l1);
  EXPECT_FALSE(LinkState::pathAInPathB(p1, p2));
  EXPECT_FALSE(LinkState::pathAInPathB(p2, p1));
}

// Hold-down: a link added with holdUpTtl stays down until the hold expires.
TEST_CPU(LinkStateTest_HoldUpAndMirror) {
  LinkState ls(kArea);
  ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 1), 0, 0);
  auto ch = ls.updateAdjacencyDatabase(createAdjDb("b", {createAdjacency("a", "b/a", "a/b", 4)}, 2), 2, 0);
  EXPECT_FALSE(ch.topologyChanged);  // held up
  EXPECT_TRUE(ls.hasHolds());
  auto const& m = ls.csrMirror();
  EXPECT_EQ(2u, (unsigned)m.names.size());
  EXPECT_EQ(2u, (unsigned)m.col.size());
  EXPECT_EQ(0, (int)m.edgeUp[0]);
  EXPECT_FALSE(ls.decrementHolds().topologyChanged);
  EXPECT_TRUE(ls.decrementHolds().topologyChanged);
  auto const& m2 = ls.csrMirror();
  EXPECT_EQ(1, (int)m2.edgeUp[0]);
  EXPECT_EQ(3u, m2.metric[m2.rowPtr[m2.id.at("a")]]);
  EXPECT_EQ(4u, m2.metric[m2.rowPtr[m2.id.at("b")]]);
}

// The mirror (and so the device graph) is rebuilt only when the link structure changes: a
// re-advertised database, or one that changes only adjacency labels, keeps it;
// a metric change patches it in place (round 3: same generation, new metric); a new node
// rebuilds it.
TEST_CPU(LinkStateTest_MirrorRebuiltOnlyOnTopologyChange) {
  LinkState ls(kArea);
  ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 1), 0, 0);
  ls.updateAdjacencyDatabase(createAdjDb("b", {createAdjacency("a", "b/a", "a/b", 4)}, 2), 0, 0);
  ls.csrMirror();
  const uint64_t g0 = ls.mirrorGeneration();
  auto ch = ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 1), 0, 0);
  EXPECT_FALSE(ch.topologyChanged);
  ls.csrMirror();
  EXPECT_EQ(g0, ls.mirrorGeneration());
  auto relabel = createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 1);
  relabel.adjacencies[0].adjLabel = 777;
  ch = ls.updateAdjacencyDatabase(relabel, 0, 0);
  EXPECT_FALSE(ch.topologyChanged);
  EXPECT_TRUE(ch.linkAttributesChanged);
  ls.csrMirror();
  EXPECT_EQ(g0, ls.mirrorGeneration());
  ch = ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 9)}, 1), 0, 0);
  EXPECT_TRUE(ch.topologyChanged);
  auto const& m = ls.csrMirror();
  EXPECT_EQ(g0, ls.mirrorGeneration());  // patched in place
  EXPECT_EQ(9u, m.metric[m.rowPtr[m.id.at("a")]]);
  EXPECT_EQ(4u, m.metric[m.rowPtr[m.id.at("b")]]);
  const uint64_t g1 = ls.mirrorGeneration();
  ls.updateAdjacencyDatabase(createAdjDb("c", {}, 3), 0, 0);  // isolated new node
  auto const& m2 = ls.csrMirror();
  EXPECT_TRUE(ls.mirrorGeneration() != g1);
  EXPECT_EQ(3u, (unsigned)m2.names.size());
}

// labeledNodeCount() follows every add, relabel, unlabel and delete (the route build skips
// its node-label pass, and its SPF prefetch when no prefix needs one, on a count of 0)
TEST_CPU(LinkStateTest_LabeledNodeCount) {
  LinkState ls(kArea);
  EXPECT_EQ(0u, (unsigned)ls.labeledNodeCount());
  ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 0), 0, 0);
  EXPECT_EQ(0u, (unsigned)ls.labeledNodeCount());
  ls.updateAdjacencyDatabase(createAdjDb("b", {createAdjacency("a", "b/a", "a/b", 4)}, 7), 0, 0);
  EXPECT_EQ(1u, (unsigned)ls.labeledNodeCount());
  ls.updateAdjacencyDatabase(createAdjDb("b", {createAdjacency("a", "b/a", "a/b", 4)}, 8), 0, 0);  // relabel
  EXPECT_EQ(1u, (unsigned)ls.labeledNodeCount());
  ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 5), 0, 0);  // label a
  EXPECT_EQ(2u, (unsigned)ls.labeledNodeCount());
  ls.updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 0), 0, 0);  // unlabel a
  EXPECT_EQ(1u, (unsigned)ls.labeledNodeCount());
  ls.deleteAdjacencyDatabase("b");
  EXPECT_EQ(0u, (unsigned)ls.labeledNodeCount());
  ls.deleteAdjacencyDatabase("b");  // unknown: no change
  EXPECT_EQ(0u, (unsigned)ls.labeledNodeCount());
}

// A copy of a LinkState reads its own databases' names in labeledNodes(), not the
// source's (the cached list holds pointers into adjacencyDatabases_)
TEST_CPU(LinkStateTest_LabeledNodesSurviveCopy) {
  std::unique_ptr<LinkState> src(new LinkState(kArea));
  src->updateAdjacencyDatabase(createAdjDb("a", {createAdjacency("b", "a/b", "b/a", 3)}, 5), 0, 0);
  src->updateAdjacencyDatabase(createAdjDb("b", {createAdjacency("a", "b/a", "a/b", 4)}, 7), 0, 0);
  EXPECT_EQ(2u, (unsigned)src->labeledNodes().size());  // the source's cache is filled
  LinkState copy(*src);
  LinkState copy2(copy);  // a copy of a copy whose cache is filled too
  (void)copy.labeledNodes();
  src.reset();  // the source's databases (and the names its cache pointed at) are gone
  for (LinkState* ls : {&copy, &copy2}) {
    auto const& l = ls->labeledNodes();
    EXPECT_EQ(2u, (unsigned)l.size());
    std::set<std::pair<std::string, int32_t>> got;
    for (auto const& n : l) {
      EXPECT_TRUE(n.name == &ls->getAdjacencyDatabases().at(*n.name).thisNodeName);
      got.emplace(*n.name, n.label);
    }
    EXPECT_TRUE(got == (std::set<std::pair<std::string, int32_t>>{{"a", 5}, {"b", 7}}));
  }
}

// ParallelAdjRingTopologyFixture adjacencies (DecisionTest.cpp:3146-3203)
static LinkState parallelRing() {
  LinkState ls(kArea);
  auto db1 = createAdjDb("1",
                         {createAdjacency("2", "2/1", "1/1", 11), createAdjacency("2", "2/2", "1/2", 11),
                          createAdjacency("2", "2/3", "1/3", 20), createAdjacency("3", "3/1", "1/1", 11)},
                         1);
  auto db2 = createAdjDb("2",
                         {createAdjacency("1", "1/1", "2/1", 11), createAdjacency("1", "1/2", "2/2", 11),
                          createAdjacency("1", "1/3", "2/3", 20), createAdjacency("4", "4/1", "2/1", 11)},
                         2);
  auto db3 = createAdjDb("3",
                         {createAdjacency("1", "1/1", "3/1", 11), createAdjacency("4", "4/1", "3/1", 11),
                          createAdjacency("4", "4/2", "3/2", 20), createAdjacency("4", "4/3", "3/3", 20)},
                         3);
  auto db4 = createAdjDb("4",
                         {createAdjacency("2", "2/1", "4/1", 11), createAdjacency("3", "3/1", "4/1", 11),
                          createAdjacency("3", "3/2", "4/2", 20), createAdjacency("3", "3/3", "4/3", 20)},
                         4);
  EXPECT_FALSE(ls.updateAdjacencyDatabase(db1).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db2).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db3).topologyChanged);
  EXPECT_TRUE(ls.updateAdjacencyDatabase(db4).topologyChanged);
  return ls;
}

TEST_CPU(LinkStateTest_LinksFromNodeOrder) {
  // The pathLinks order among parallel links follows linksFromNode() iteration;
  // with folly's pair hash on libstdc++ node 1 iterates its 1-2 links as 2/2 before 2/1
  // (what DecisionTest.cpp:3596-3599 relies on). Printed for the record.
  auto ls = parallelRing();
  std::string order;
  for (auto const& l : ls.linksFromNode("1")) order += l->getIfaceFromNode("1") + " ";
  std::printf("    linksFromNode(1) order: %s\n", order.c_str());
  size_t p22 = order.find("2/2"), p21 = order.find("2/1");
  EXPECT_TRUE(p22 != std::string::npos && p21 != std::string::npos);
}

// ---------------------------------------------------------------------------
// GPU tests
// LinkStateTest.cpp:244-284
TEST_GPU(LinkStateTest_getKthPaths_box) {
  auto linkState = getLinkState({{1, {{2, 10}, {3, 5}}},
                                 {2, {{1, 10}, {4, 15}, {4, 35}}},
                                 {3, {{1, 5}, {4, 20}}},
                                 {4, {{2, 15}, {3, 20}, {2, 35}}}});
  auto firstPaths = linkState.getKthPaths("2", "4", 1);
  EXPECT_EQ(1u, firstPaths.size());
  EXPECT_EQ(1u, firstPaths.at(0).size());
  EXPECT_EQ(15u, firstPaths.at(0).at(0)->getMetricFromNode("2"));
  auto secondPaths = linkState.getKthPaths("2", "4", 2);
  EXPECT_EQ(2u, secondPaths.size());
  std::multiset<size_t> sizes;
  for (auto const& path : secondPaths) {
    sizes.insert(path.size());
    std::string next = "2";
    LinkStateMetric dist = 0;
    for (auto const& link : path) {
      dist += link->getMetricFromNode(next);
      next = link->getOtherNodeName(next);
    }
    EXPECT_EQ(35u, dist);
  }
  EXPECT_TRUE((sizes == std::multiset<size_t>{1, 3}));
}

// LinkStateTest.cpp:286-315
TEST_GPU(LinkStateTest_getKthPaths_mesh) {
  auto linkState = getLinkState(
      unit({{1, {2, 2, 3, 3, 4, 4}}, {2, {1, 1, 3, 3, 4, 4}}, {3, {1, 1, 2, 2, 4, 4}}, {4, {1, 1, 2, 2, 3, 3}}}));
  auto firstPaths = linkState.getKthPaths("2", "4", 1);
  EXPECT_EQ(2u, firstPaths.size());
  for (auto const& p : firstPaths) EXPECT_EQ(1u, p.size());
  auto secondPaths = linkState.getKthPaths("2", "4", 2);
  EXPECT_EQ(4u, secondPaths.size());
  for (auto const& p : secondPaths) EXPECT_EQ(2u, p.size());
  LinkState::LinkSet set;
  auto all = firstPaths;
  all.insert(all.end(), secondPaths.begin(), secondPaths.end());
  for (auto const& path : all)
    for (auto const& link : path) EXPECT_TRUE(set.insert(link).second);
}

// LinkStateTest.cpp:318-377
TEST_GPU(LinkStateTest_getHopCounts) {
  {
    auto ls = getLinkState(unit({{1, {2, 3}}, {2, {1, 4}}, {3, {1, 4}}, {4, {2, 3}}}));
    EXPECT_TRUE(ls.getHopsFromAToB("1", "2") == 1u);
    EXPECT_TRUE(ls.getHopsFromAToB("1", "4") == 2u);
    EXPECT_EQ(2u, ls.getMaxHopsToNode("1"));
  }
  {
    auto ls = getLinkState(unit({{1, {2}}, {2, {1, 3}}, {3, {2, 4}}, {4, {3, 5}}, {5, {4}}}));
    EXPECT_TRUE(ls.getHopsFromAToB("1", "2") == 1u);
    EXPECT_TRUE(ls.getHopsFromAToB("1", "4") == 3u);
    EXPECT_TRUE(ls.getHopsFromAToB("2", "3") == 1u);
    EXPECT_EQ(4u, ls.getMaxHopsToNode("1"));
    EXPECT_EQ(3u, ls.getMaxHopsToNode("2"));
    EXPECT_EQ(2u, ls.getMaxHopsToNode("3"));
  }
  {
    auto ls = getLinkState(unit({{1, {2}}, {2, {1, 3}}, {3, {2, 4}}, {4, {3}}, {5, {}}}));
    EXPECT_FALSE(ls.getHopsFromAToB("1", "5").has_value());
    EXPECT_TRUE(ls.getHopsFromAToB("2", "3") == 1u);
    EXPECT_EQ(3u, ls.getMaxHopsToNode("1"));
    EXPECT_EQ(0u, ls.getMaxHopsToNode("5"));
  }
}

// DecisionTest.cpp:3536-3599 (KSP2 on the parallel-adjacency ring): k=1 paths from 1
// to 4 leave node 1 over adj12_2 (ifName 2/2) and adj13_1 (ifName 3/1); k=2 is empty.
TEST_GPU(DecisionTest_ParallelAdjRing_Ksp2FirstHops) {
  auto ls = parallelRing();
  auto const& k1 = ls.getKthPaths("1", "4", 1);
  EXPECT_EQ(2u, k1.size());
  std::set<std::string> firstIfs;
  for (auto const& p : k1) firstIfs.insert(p.front()->getIfaceFromNode("1"));
  EXPECT_TRUE((firstIfs == std::set<std::string>{"2/2", "3/1"}));
  EXPECT_TRUE(ls.getKthPaths("1", "4", 2).empty());
  auto const& r = ls.getSpfResult("1");
  EXPECT_EQ(22u, r.at("4").metric());
  EXPECT_TRUE((r.at("4").nextHops() == std::unordered_set<std::string>{"2", "3"}));
}

// SimpleRingTopologyFixture counters (DecisionTest.cpp:1826-1827, 2306-2309):
// 4 base SPFs for 4 sources, then 12 KSP2 second SPFs.
TEST_GPU(DecisionTest_SimpleRing_SpfRunCounts) {
  LinkState ls(kArea);
  ls.updateAdjacencyDatabase(
      createAdjDb("1", {createAdjacency("2", "1/2", "2/1", 10), createAdjacency("3", "1/3", "3/1", 10)}, 1));
  ls.updateAdjacencyDatabase(
      createAdjDb("2", {createAdjacency("1", "2/1", "1/2", 10), createAdjacency("4", "2/4", "4/2", 10)}, 2));
  ls.updateAdjacencyDatabase(
      createAdjDb("3", {createAdjacency("1", "3/1", "1/3", 10), createAdjacency("4", "3/4", "4/3", 10)}, 3));
  ls.updateAdjacencyDatabase(
      createAdjDb("4", {createAdjacency("2", "4/2", "2/4", 10), createAdjacency("3", "4/3", "3/4", 10)}, 4));
  SpfCounters::get().reset();
  const std::vector<std::string> nodes{"1", "2", "3", "4"};
  for (auto const& n : nodes) ls.getSpfResult(n);
  EXPECT_EQ(4u, SpfCounters::get().spfRuns());
  for (auto const& s : nodes)
    for (auto const& d : nodes)
      if (s != d) {
        ls.getKthPaths(s, d, 1);
        ls.getKthPaths(s, d, 2);
      }
  EXPECT_EQ(16u, SpfCounters::get().spfRuns());
  auto const& r1 = ls.getSpfResult("1");
  EXPECT_EQ(20u, r1.at("4").metric());
  EXPECT_TRUE((r1.at("4").nextHops() == std::unordered_set<std::string>{"2", "3"}));
}

// DecisionTest.cpp:4207-4355 grid, all sources via one batched prefetch
TEST_GPU(DecisionTest_Grid_ShortestPath) {
  for (int n : {2, 4, 10, 16}) {
    LinkState ls(kArea);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        std::vector<thrift::Adjacency> adjs;
        auto add = [&](int ii, int jj, const char* ifn, const char* oifn) {
          if (ii < 0 || ii >= n || jj < 0 || jj >= n) return;
          adjs.push_back(createAdjacency(std::to_string(ii * n + jj), ifn, oifn, 1));
        };
        add(i, j + 1, "0/1", "0/3");
        add(i - 1, j, "0/2", "0/4");
        add(i, j - 1, "0/3", "0/1");
        add(i + 1, j, "0/4", "0/2");
        ls.updateAdjacencyDatabase(createAdjDb(std::to_string(i * n + j), adjs, i * n + j + 1));
      }
    std::vector<std::string> all;
    for (int v = 0; v < n * n; ++v) all.push_back(std::to_string(v));
    SpfCounters::get().reset();
    ls.prefetchSpfResults(all);
    EXPECT_EQ(0u, SpfCounters::get().spfRuns());  // prefetched runs count when first read
    bool ok = true;
    for (int a = 0; a < n * n; ++a)
      for (int b = 0; b < n * n; ++b) {
        auto m = ls.getMetricFromAToB(std::to_string(a), std::to_string(b));
        const int want = std::abs(a % n - b % n) + std::abs(a / n - b / n);
        ok &= m.has_value() && *m == (LinkStateMetric)want;
      }
    EXPECT_TRUE(ok);
    EXPECT_EQ((uint64_t)(n * n), SpfCounters::get().spfRuns());  // all served by the memo
  }
}

// The memo under LinkState::MemoFreeze (SpfSolver::buildRouteDbs' worker threads): reads
// the prefetch covered are served, a miss throws instead of solving concurrently; prefetched
// results count as SPF runs when first read (the reference's memo-miss accounting).
TEST_GPU(LinkState_FrozenMemoMissThrows) {
  LinkState ls(kArea);
  ls.updateAdjacencyDatabase(
      createAdjDb("1", {createAdjacency("2", "1/2", "2/1", 10), createAdjacency("3", "1/3", "3/1", 10)}, 1));
  ls.updateAdjacencyDatabase(createAdjDb("2", {createAdjacency("1", "2/1", "1/2", 10)}, 2));
  ls.updateAdjacencyDatabase(createAdjDb("3", {createAdjacency("1", "3/1", "1/3", 10)}, 3));
  SpfCounters::get().reset();
  ls.prefetchSpfResults({"1", "2"});
  EXPECT_EQ(0u, SpfCounters::get().spfRuns());
  {
    LinkState::MemoFreeze freeze(ls);
    EXPECT_EQ(10u, ls.getSpfResult("1").at("2").metric());
    EXPECT_EQ(1u, SpfCounters::get().spfRuns());
    ls.getSpfResult("1");  // a memo hit: no new run
    EXPECT_EQ(1u, SpfCounters::get().spfRuns());
    EXPECT_THROW(ls.getSpfResult("3"));
    EXPECT_THROW(ls.getSpfResult("1", false));
    EXPECT_THROW(ls.getKthPaths("1", "3", 1));
    EXPECT_THROW(ls.prefetchSpfResults({"3"}));
  }
  EXPECT_EQ(20u, ls.getSpfResult("3").at("2").metric());  // unfrozen: a miss solves again
  EXPECT_EQ(2u, SpfCounters::get().spfRuns());
  ls.getSpfResult("2");
  EXPECT_EQ(3u, SpfCounters::get().spfRuns());
}

// Random topologies through the full adjacency-database path: every getSpfResult and
// getKthPaths equals the oracle run on the same CSR mirror (pathLinks order included).
// metric(rng) draws every directed metric of a trial
template <typename MetricFn>
static void randomOracleParity(uint64_t seed, MetricFn metric) {
  std::mt19937_64 rng(seed);
  for (int trial = 0; trial < 6; ++trial) {
    const int V = 12 + trial * 9;
    LinkState ls(kArea);
    std::vector<std::vector<thrift::Adjacency>> adjs(V);
    int ifc = 0;
    auto link = [&](int a, int b, int wa, int wb, bool ovl) {
      const std::string ia = "if" + std::to_string(ifc++), ib = "if" + std::to_string(ifc++);
      auto x = createAdjacency(std::to_string(b), ia, ib, wa);
      x.isOverloaded = ovl;
      adjs[a].push_back(x);
      adjs[b].push_back(createAdjacency(std::to_string(a), ib, ia, wb));
    };
    for (int v = 1; v < V; ++v) link((int)(rng() % v), v, metric(rng), metric(rng), false);
    for (int k = 0; k < V; ++k) {
      int a = rng() % V, b = rng() % V;
      if (a != b) link(a, b, metric(rng), metric(rng), rng() % 10 == 0);
    }
    for (int k = 0; k < V / 4; ++k) {  // parallel links
      int a = rng() % V;
      if (!adjs[a].empty()) {
        int b = std::stoi(adjs[a][0].otherNodeName);
        link(a, b, metric(rng), metric(rng), false);
      }
    }
    for (int v = 0; v < V; ++v) {
      auto db = createAdjDb(std::to_string(v), adjs[v], v + 1);
      db.isOverloaded = rng() % 8 == 0;
      ls.updateAdjacencyDatabase(db);
    }
    auto const& m = ls.csrMirror();
    oracle_graph og{(uint32_t)m.names.size(), (uint32_t)m.col.size(), (uint32_t)m.links.size(), m.rowPtr.data(),
                    m.col.data(), m.metric.data(), m.linkId.data(), m.edgeUp.data(), m.overloaded.data(),
                    m.nameRank.data()};
    const uint32_t NV = og.num_nodes, NE = og.num_dir_edges;
    std::vector<uint64_t> dist(NV);
    std::vector<uint32_t> plp(NV + 1), ple(NE + 1), order(NV);
    std::vector<uint8_t> reached(NV);
    for (uint32_t s = 0; s < NV; ++s) {
      for (int useMetric = 0; useMetric < 2; ++useMetric) {
        auto const& res = ls.getSpfResult(m.names[s], useMetric != 0);
        int64_t cnt = oracle_run_spf(&og, s, useMetric, nullptr, dist.data(), nullptr, 0, order.data(), plp.data(),
                                     ple.data());
        EXPECT_EQ((size_t)cnt, res.size());
        std::fill(reached.begin(), reached.end(), 0);
        for (int64_t i = 0; i < cnt; ++i) reached[order[i]] = 1;  // a wrapped dist may equal UINT64_MAX
        for (uint32_t v = 0; v < NV; ++v) {
          auto it = res.find(m.names[v]);
          if (!reached[v]) {
            EXPECT_TRUE(it == res.end());
            continue;
          }
          if (it == res.end()) {
            EXPECT_TRUE(false);
            continue;
          }
          EXPECT_EQ(dist[v], it->second.metric());
          auto const& pls = it->second.pathLinks();
          bool same = pls.size() == plp[v + 1] - plp[v];
          for (uint32_t i = 0; same && i < pls.size(); ++i) {
            const uint32_t e = ple[plp[v] + i];
            same = pls[i].link.get() == m.links[m.linkId[e]].get() && pls[i].prevNode == m.names[m.edgeOwner[e]];
          }
          EXPECT_TRUE(same);
        }
      }
      for (uint32_t d = 0; d < NV; d += 3) {
        for (uint32_t k = 1; k <= 2; ++k) {
          auto const& paths = ls.getKthPaths(m.names[s], m.names[d], k);
          std::vector<uint32_t> pptr(NE + 2), pe(NE + 2);
          int64_t np = oracle_kth_paths(&og, s, d, k, pptr.data(), NE + 1, pe.data(), NE + 1);
          EXPECT_EQ((size_t)np, paths.size());
          bool same = (size_t)np == paths.size();
          for (int64_t i = 0; same && i < np; ++i) {
            same = paths[i].size() == pptr[i + 1] - pptr[i];
            for (uint32_t j = 0; same && j < paths[i].size(); ++j)
              same = paths[i][j].get() == m.links[m.linkId[pe[pptr[i] + j]]].get();
          }
          EXPECT_TRUE(same);
        }
      }
    }
  }
}

TEST_GPU(LinkState_RandomOracleParity) {
  randomOracleParity(7, [](std::mt19937_64& r) { return (int)(1 + r() % 6); });
}

// Zero and negative i32 metrics (LinkState.cpp:151-152 stores them as u64, sums wrap):
// the mirror routes these graphs to the exact-order kernel and rebuilds pathLinks from
// its pop order (openr_spf_solve_order); results still equal the oracle's.
TEST_GPU(LinkState_ZeroAndNegativeMetricOracleParity) {
  randomOracleParity(11, [](std::mt19937_64& r) {
    static const int kPool[] = {0, 0, 1, 2, 3, -1, -7};
    return kPool[r() % 7];
  });
}

// A hub with 300 distinct neighbours (next-hop sets wider than 256 bits): served by the
// exact-order kernel; getSpfResult from the hub and from a leaf equals the oracle.
TEST_GPU(LinkState_WideHubOracleParity) {
  LinkState ls(kArea);
  const int leaves = 300;
  std::vector<thrift::Adjacency> hub;
  for (int i = 1; i <= leaves; ++i) {
    const std::string leaf = std::to_string(i), other = std::to_string(i % leaves + 1);
    hub.push_back(createAdjacency(leaf, "h" + leaf, "u" + leaf, 1 + i % 3));
    std::vector<thrift::Adjacency> adjs{createAdjacency("0", "u" + leaf, "h" + leaf, 2),
                                        createAdjacency(other, "r" + leaf, "l" + other, 5)};
    const std::string prev = std::to_string((i + leaves - 2) % leaves + 1);
    adjs.push_back(createAdjacency(prev, "l" + leaf, "r" + prev, 5));
    ls.updateAdjacencyDatabase(createAdjDb(leaf, adjs, i + 1));
  }
  ls.updateAdjacencyDatabase(createAdjDb("0", hub, 1));
  auto const& m = ls.csrMirror();
  oracle_graph og{(uint32_t)m.names.size(), (uint32_t)m.col.size(), (uint32_t)m.links.size(), m.rowPtr.data(),
                  m.col.data(), m.metric.data(), m.linkId.data(), m.edgeUp.data(), m.overloaded.data(),
                  m.nameRank.data()};
  const uint32_t NV = og.num_nodes, NE = og.num_dir_edges;
  std::vector<uint64_t> dist(NV);
  std::vector<uint32_t> plp(NV + 1), ple(NE + 1);
  for (const char* src : {"0", "1", "150"}) {
    const uint32_t s = m.id.at(src);
    auto const& res = ls.getSpfResult(src, true);
    const int64_t cnt = oracle_run_spf(&og, s, 1, nullptr, dist.data(), nullptr, 0, nullptr, plp.data(), ple.data());
    EXPECT_EQ((size_t)cnt, res.size());
    bool same = true;
    for (uint32_t v = 0; v < NV; ++v) {
      auto it = res.find(m.names[v]);
      same &= it != res.end() && it->second.metric() == dist[v] && it->second.pathLinks().size() == plp[v + 1] - plp[v];
    }
    EXPECT_TRUE(same);
  }
  auto const& r0 = ls.getSpfResult("0", true);
  EXPECT_EQ(1u, r0.at("3").nextHops().size());  // direct neighbour 3 of the 300-wide hub
}

// getSpfResult(names[s], useMetric) of every source in `srcs` equals the oracle run on the
// current CSR mirror: reached set, metrics, next-hop names and pathLinks (link and previous
// node, in order).
static bool spfMatchesOracle(const LinkState& ls, const std::vector<uint32_t>& srcs, bool useMetric) {
  auto const& m = ls.csrMirror();
  oracle_graph og{(uint32_t)m.names.size(), (uint32_t)m.col.size(), (uint32_t)m.links.size(), m.rowPtr.data(),
                  m.col.data(), m.metric.data(), m.linkId.data(), m.edgeUp.data(), m.overloaded.data(),
                  m.nameRank.data()};
  const uint32_t NV = og.num_nodes, NE = og.num_dir_edges;
  std::vector<uint64_t> dist(NV);
  std::vector<uint32_t> plp(NV + 1), ple(NE + 1);
  bool ok = true;
  for (uint32_t s : srcs) {
    const uint32_t nb = (oracle_num_distinct_neighbors(&og, s) + 7) / 8 + 1;
    std::vector<uint8_t> nh((size_t)NV * nb);
    std::vector<uint32_t> nbr;  // distinct neighbours of s in row order = next-hop bit order
    for (uint32_t e = m.rowPtr[s]; e < m.rowPtr[s + 1]; ++e)
      if (std::find(nbr.begin(), nbr.end(), m.col[e]) == nbr.end()) nbr.push_back(m.col[e]);
    auto const& res = ls.getSpfResult(m.names[s], useMetric);
    const int64_t cnt = oracle_run_spf(&og, s, useMetric, nullptr, dist.data(), nh.data(), nb, nullptr, plp.data(),
                                       ple.data());
    ok &= (size_t)cnt == res.size();
    for (uint32_t v = 0; v < NV && ok; ++v) {
      auto it = res.find(m.names[v]);
      if (dist[v] == UINT64_MAX) {
        ok &= it == res.end();
        continue;
      }
      if (it == res.end()) {
        ok = false;
        break;
      }
      ok &= dist[v] == it->second.metric();
      std::unordered_set<std::string> want;
      for (uint32_t i = 0; i < nbr.size(); ++i)
        if ((nh[(size_t)v * nb + (i >> 3)] >> (i & 7)) & 1u) want.insert(m.names[nbr[i]]);
      ok &= want == it->second.nextHops();
      auto const& pls = it->second.pathLinks();
      ok &= pls.size() == plp[v + 1] - plp[v];
      for (uint32_t i = 0; ok && i < pls.size(); ++i) {
        const uint32_t e = ple[plp[v] + i];
        ok &= pls[i].link.get() == m.links[m.linkId[e]].get() && pls[i].prevNode == m.names[m.edgeOwner[e]];
      }
    }
    if (!ok) std::printf("    oracle mismatch: source %s (useMetric %d)\n", m.names[s].c_str(), (int)useMetric);
  }
  return ok;
}

// getKthPaths(names[s], names[d], k) for k = 1, 2 equals oracle_kth_paths on the current
// mirror (link for link, in order) for every (s, d) of srcs x dsts.
static bool kthMatchesOracle(const LinkState& ls, const std::vector<uint32_t>& srcs, const std::vector<uint32_t>& dsts) {
  auto const& m = ls.csrMirror();
  oracle_graph og{(uint32_t)m.names.size(), (uint32_t)m.col.size(), (uint32_t)m.links.size(), m.rowPtr.data(),
                  m.col.data(), m.metric.data(), m.linkId.data(), m.edgeUp.data(), m.overloaded.data(),
                  m.nameRank.data()};
  const uint32_t NE = og.num_dir_edges;
  std::vector<uint32_t> pptr(NE + 2), pe(NE + 2);
  bool ok = true;
  for (uint32_t s : srcs)
    for (uint32_t d : dsts)
      for (uint32_t k = 1; k <= 2; ++k) {
        auto const& paths = ls.getKthPaths(m.names[s], m.names[d], k);
        const int64_t np = oracle_kth_paths(&og, s, d, k, pptr.data(), NE + 1, pe.data(), NE + 1);
        bool same = np >= 0 && (size_t)np == paths.size();
        for (int64_t i = 0; same && i < np; ++i) {
          same = paths[i].size() == pptr[i + 1] - pptr[i];
          for (uint32_t j = 0; same && j < paths[i].size(); ++j)
            same = paths[i][j].get() == m.links[m.linkId[pe[pptr[i] + j]]].get();
        }
        if (!same) std::printf("    kth-path mismatch: %s -> %s k=%u\n", m.names[s].c_str(), m.names[d].c_str(), k);
        ok &= same;
      }
  return ok;
}

// n x n grid adjacency databases (DecisionTest.cpp:4207-4355 names / ifnames), metric w(i, j)
template <typename W>
static thrift::AdjacencyDatabase gridDb(int n, int i, int j, W w, bool overloaded = false) {
  std::vector<thrift::Adjacency> adjs;
  auto add = [&](int ii, int jj, const char* ifn, const char* oifn) {
    if (ii < 0 || ii >= n || jj < 0 || jj >= n) return;
    adjs.push_back(createAdjacency(std::to_string(ii * n + jj), ifn, oifn, w(i, j, ii, jj)));
  };
  add(i, j + 1, "0/1", "0/3");
  add(i - 1, j, "0/2", "0/4");
  add(i, j - 1, "0/3", "0/1");
  add(i + 1, j, "0/4", "0/2");
  auto db = createAdjDb(std::to_string(i * n + j), adjs, i * n + j + 1);
  db.isOverloaded = overloaded;
  return db;
}

// attribute-only updates — a node overload toggle (the BM_DecisionGrid /
// BM_DecisionFabric update, RoutingBenchmarkUtils.cpp:407-479), a metric change, an
// adjacency overload (Link::isUp), and held values released by decrementHolds — patch the
// engine's resident graph instead of re-uploading it, keep the memo's dense rows and
// refresh only the rows the change can affect; every result equals the oracle on the
// updated graph, and decision.spf_runs counts each source read again as the reference's
// cleared memo would (LinkState.cpp:714-717).
TEST_GPU(LinkState_AttributeUpdatesPatchAndRefresh) {
  const int n = 12;
  for (int weighted = 0; weighted < 2; ++weighted) {
    auto w = [weighted](int i, int j, int ii, int jj) { return weighted ? 1 + (i * 7 + j * 3 + ii + jj * 5) % 9 : 1; };
    LinkState ls(kArea);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) ls.updateAdjacencyDatabase(gridDb(n, i, j, w));
    std::vector<std::string> all;
    std::vector<uint32_t> ids;
    for (int v = 0; v < n * n; ++v) all.push_back(std::to_string(v));
    ls.prefetchSpfResults(all);
    ls.prefetchSpfResults(all, false);
    auto const& m0 = ls.csrMirror();
    for (auto const& a : all) ids.push_back(m0.id.at(a));
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    EXPECT_TRUE(spfMatchesOracle(ls, ids, false));
    const uint64_t gen = ls.mirrorGeneration(), uploads = ls.updateStats().graphUploads;
    EXPECT_EQ((size_t)(n * n), ls.denseRows(true));
    // 1) node overload on, then off (the benchmark's toggle)
    const int x = 5 * n + 6, xi = x / n, xj = x % n;
    for (int on = 1; on >= 0; --on) {
      auto ch = ls.updateAdjacencyDatabase(gridDb(n, xi, xj, w, on != 0));
      EXPECT_TRUE(ch.topologyChanged);
      SpfCounters::get().reset();
      ls.prefetchSpfResults(all);
      EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
      EXPECT_EQ((uint64_t)(n * n), SpfCounters::get().spfRuns());  // every source read once, counted once
      EXPECT_TRUE(spfMatchesOracle(ls, ids, false));
    }
    // getKthPaths after the patches: its k = 1 paths trace pathLinks re-derived from the
    // refreshed rows' distances, its k = 2 paths an ignore-set solve on the patched graph
    {
      auto on = ls.updateAdjacencyDatabase(gridDb(n, xi, xj, w, true));
      EXPECT_TRUE(on.topologyChanged);
      EXPECT_TRUE(kthMatchesOracle(ls, {0u, (uint32_t)(x - 1), (uint32_t)(n * n - 1)},
                                   {(uint32_t)(x + 1), (uint32_t)(x + n), (uint32_t)(n * n / 2), 3u}));
      EXPECT_TRUE(ls.updateAdjacencyDatabase(gridDb(n, xi, xj, w, false)).topologyChanged);
      EXPECT_TRUE(kthMatchesOracle(ls, {0u, (uint32_t)(x - 1), (uint32_t)(n * n - 1)},
                                   {(uint32_t)(x + 1), (uint32_t)(x + n), (uint32_t)(n * n / 2), 3u}));
    }
    EXPECT_EQ(gen, ls.mirrorGeneration());
    EXPECT_EQ(uploads, ls.updateStats().graphUploads);  // patched, never re-uploaded
    EXPECT_EQ(4u, (unsigned)ls.updateStats().patches);
    // incremental: the refreshes re-solved fewer rows than they kept
    EXPECT_TRUE(ls.updateStats().rowsRefreshed < ls.updateStats().rowsKept);
    // 2) metric change of one adjacency, 3) adjacency overload (link down), then back up
    auto w2 = [&](int i, int j, int ii, int jj) { return (i == 3 && j == 3 && jj == 4) ? 40 : w(i, j, ii, jj); };
    ls.updateAdjacencyDatabase(gridDb(n, 3, 3, w2));
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    auto db = gridDb(n, 7, 2, w);
    db.adjacencies[0].isOverloaded = true;
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db).topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    EXPECT_TRUE(spfMatchesOracle(ls, ids, false));
    db.adjacencies[0].isOverloaded = false;
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db).topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    // 4) a metric rise held down for two decrementHolds ticks (HoldableValue), released there
    auto w3 = [&](int i, int j, int ii, int jj) { return (i == 9 && j == 9) ? 30 : w2(i, j, ii, jj); };
    EXPECT_FALSE(ls.updateAdjacencyDatabase(gridDb(n, 9, 9, w3), 0, 2).topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    EXPECT_FALSE(ls.decrementHolds().topologyChanged);
    EXPECT_TRUE(ls.decrementHolds().topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    EXPECT_TRUE(spfMatchesOracle(ls, ids, false));
    EXPECT_EQ(gen, ls.mirrorGeneration());
    EXPECT_EQ(uploads, ls.updateStats().graphUploads);
    // a structural change (a new link) rebuilds the mirror and uploads it
    ls.updateAdjacencyDatabase(createAdjDb("extra", {createAdjacency("0", "x/0", "0/x", 1)}, 999));
    auto db0 = gridDb(n, 0, 0, w);
    db0.adjacencies.push_back(createAdjacency("extra", "0/x", "x/0", 1));
    EXPECT_TRUE(ls.updateAdjacencyDatabase(db0).topologyChanged);
    ids.clear();
    auto const& m1 = ls.csrMirror();
    for (uint32_t v = 0; v < m1.names.size(); ++v) ids.push_back(v);
    EXPECT_TRUE(spfMatchesOracle(ls, ids, true));
    EXPECT_TRUE(gen != ls.mirrorGeneration());
    EXPECT_EQ(uploads + 1, ls.updateStats().graphUploads);
    std::printf("    weighted=%d patches=%llu refreshes=%llu rows kept=%llu re-solved=%llu\n", weighted,
                (unsigned long long)ls.updateStats().patches, (unsigned long long)ls.updateStats().refreshes,
                (unsigned long long)ls.updateStats().rowsKept, (unsigned long long)ls.updateStats().rowsRefreshed);
  }
}

// changes that rebuild the mirror without being topology changes keep
// the reference's memo (LinkState.cpp:714-717 clears it only on topologyChanged): a new
// node's first adjacency database that forms no link, and a link that forms while held
// down (holdUpTtl > 0). The memo entries keep reading the rows of the mirror they were
// solved on (a retired snapshot), rows solved after the rebuild use the new ids, and every
// read equals the oracle on the current graph with no SPF re-run.
TEST_GPU(LinkState_MemoSurvivesNonTopologyRebuild) {
  const int n = 7;
  auto w = [](int i, int j, int ii, int jj) { return 1 + (i * 5 + j + ii * 3 + jj) % 4; };
  LinkState ls(kArea);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) ls.updateAdjacencyDatabase(gridDb(n, i, j, w));
  std::vector<std::string> all;
  for (int v = 0; v < n * n; ++v) all.push_back(std::to_string(v));
  ls.prefetchSpfResults(all);
  ls.prefetchSpfResults(all, false);
  auto oldIds = [&]() {
    std::vector<uint32_t> ids;
    for (auto const& a : all) ids.push_back(ls.csrMirror().id.at(a));
    return ids;
  };
  EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), true));
  EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), false));
  auto viewMatches = [&](bool um) {
    bool ok = true;
    for (auto const& s : all) {
      auto const v = ls.getSpfView(s, um);
      auto const& r = ls.getSpfResult(s, um);
      for (auto const& d : ls.csrMirror().names) {
        auto it = r.find(d);
        ok &= v.reached(d) == (it != r.end());
        if (it == r.end()) continue;
        ok &= v.metric(d) == it->second.metric();
        auto nh = v.nextHops(d);
        ok &= std::unordered_set<std::string>(nh.begin(), nh.end()) == it->second.nextHops();
      }
    }
    return ok;
  };
  // 1) "zz" (sorts after every grid name) and "!a" (sorts before: every old id shifts by
  //    one in the rebuilt mirror) advertise adjacencies that are not reciprocated
  for (const char* nn : {"zz", "!a"}) {
    auto ch = ls.updateAdjacencyDatabase(createAdjDb(nn, {createAdjacency("0", "y/0", "0/y", 1)}, 900));
    EXPECT_FALSE(ch.topologyChanged);
  }
  SpfCounters::get().reset();
  EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), true));
  EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), false));
  EXPECT_TRUE(viewMatches(true));
  EXPECT_TRUE(viewMatches(false));
  EXPECT_EQ(0u, (unsigned)SpfCounters::get().spfRuns());  // memo hits: nothing re-run
  // rows solved on the rebuilt mirror beside the retired ones
  EXPECT_TRUE(spfMatchesOracle(ls, {ls.csrMirror().id.at("zz"), ls.csrMirror().id.at("!a")}, true));
  // 2) a link between 0 and 1 formed while held down: not a topology change either
  {
    auto db0 = gridDb(n, 0, 0, w);
    db0.adjacencies.push_back(createAdjacency("1", "0/h", "1/h", 1));
    auto db1 = gridDb(n, 0, 1, w);
    db1.adjacencies.push_back(createAdjacency("0", "1/h", "0/h", 1));
    EXPECT_FALSE(ls.updateAdjacencyDatabase(db0, 2, 0).topologyChanged);
    EXPECT_FALSE(ls.updateAdjacencyDatabase(db1, 2, 0).topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), true));
    EXPECT_TRUE(viewMatches(true));
    EXPECT_TRUE(spfMatchesOracle(ls, {ls.csrMirror().id.at("zz")}, true));
    EXPECT_EQ(2u, (unsigned)SpfCounters::get().spfRuns());  // only zz and !a ran
    // the hold expires: a topology change, the memo is cleared and results follow the link
    EXPECT_FALSE(ls.decrementHolds().topologyChanged);
    EXPECT_TRUE(ls.decrementHolds().topologyChanged);
    EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), true));
    EXPECT_TRUE(spfMatchesOracle(ls, oldIds(), false));
    EXPECT_TRUE(viewMatches(true));
  }
}

// a mirror rebuild (a new node) keeps only the dense rows live memo entries
// still reference. After an attribute change clears the memo, a build reads a few sources
// again; the rebuild then retires those rows alone, not every row of the set.
TEST_GPU(LinkState_RetireKeepsOnlyLiveRows) {
  const int n = 7;
  auto w = [](int i, int j, int ii, int jj) { return 1 + (i * 3 + j + ii + 2 * jj) % 4; };
  LinkState ls(kArea);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) ls.updateAdjacencyDatabase(gridDb(n, i, j, w));
  std::vector<std::string> all;
  for (int v = 0; v < n * n; ++v) all.push_back(std::to_string(v));
  ls.prefetchSpfResults(all);
  EXPECT_EQ((size_t)(n * n), ls.denseRows(true));
  // overload toggle: the memo is cleared, the rows stay (refreshed on the next read)
  ls.updateAdjacencyDatabase(gridDb(n, 3, 3, w, true));
  const std::vector<std::string> reread{"5", "30"};
  for (auto const& s : reread) ls.getSpfResult(s);
  const uint64_t retired0 = ls.updateStats().rowsRetired;
  // "zz" advertises an adjacency nobody reciprocates: a new node, not a topology change
  EXPECT_FALSE(ls.updateAdjacencyDatabase(createAdjDb("zz", {createAdjacency("0", "y/0", "0/y", 1)}, 900))
                   .topologyChanged);
  ls.csrMirror();  // rebuild
  EXPECT_EQ(retired0 + reread.size(), ls.updateStats().rowsRetired);
  SpfCounters::get().reset();
  std::vector<uint32_t> ids;
  for (auto const& s : reread) ids.push_back(ls.csrMirror().id.at(s));
  EXPECT_TRUE(spfMatchesOracle(ls, ids, true));  // served from the retired rows
  for (auto const& s : reread) {
    auto const v = ls.getSpfView(s);
    auto const& r = ls.getSpfResult(s);
    bool ok = true;
    for (auto const& d : ls.csrMirror().names) {
      auto it = r.find(d);
      ok &= v.reached(d) == (it != r.end());
      if (it != r.end()) ok &= v.metric(d) == it->second.metric();
    }
    EXPECT_TRUE(ok);
  }
  EXPECT_EQ(0u, (unsigned)SpfCounters::get().spfRuns());  // memo hits
}

// SpfView (the route build's dense read path) serves what getSpfResult does.
TEST_GPU(LinkState_SpfViewMatchesSpfResult) {
  const int n = 9;
  LinkState ls(kArea);
  auto w = [](int i, int j, int ii, int jj) { return 1 + (i + 2 * j + ii * jj) % 5; };
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) ls.updateAdjacencyDatabase(gridDb(n, i, j, w, i * n + j == 40));
  bool ok = true;
  for (int useMetric = 0; useMetric < 2; ++useMetric)
    for (int s = 0; s < n * n; s += 4) {
      auto const v = ls.getSpfView(std::to_string(s), useMetric != 0);
      auto const& r = ls.getSpfResult(std::to_string(s), useMetric != 0);
      for (int d = 0; d < n * n; ++d) {
        const std::string dn = std::to_string(d);
        auto it = r.find(dn);
        ok &= v.reached(dn) == (it != r.end());
        if (it == r.end()) continue;
        ok &= v.metric(dn) == it->second.metric();
        auto nh = v.nextHops(dn);
        ok &= std::unordered_set<std::string>(nh.begin(), nh.end()) == it->second.nextHops();
      }
    }
  EXPECT_TRUE(ok);
  auto const u = ls.getSpfView("no-such-node");
  EXPECT_TRUE(u.reached("no-such-node"));
  EXPECT_FALSE(u.reached("0"));
}

// Dense memo rows hold distances as u32 while every finite one fits and widen to u64 when
// one does not (round 4): a chain whose far end lies past 2^32 with metrics of 2^31 - 1,
// read first from a source whose rows fit (u32 rows), then from sources past 2^32 (every
// row widens), then after a metric change (the refresh path on u64 rows); every result
// against the oracle.
TEST_GPU(LinkState_DenseRowsWidenPastU32) {
  const int n = 8;
  const int32_t big = 2147483647;
  auto build = [&](int32_t farMetric) {
    std::vector<std::pair<int, std::vector<std::pair<int, int>>>> adj;
    for (int i = 0; i < n; ++i) {
      std::vector<std::pair<int, int>> a;
      if (i > 0) a.emplace_back(i - 1, i >= n - 3 ? farMetric : 1);
      if (i + 1 < n) a.emplace_back(i + 1, i + 1 >= n - 3 ? farMetric : 1);
      adj.emplace_back(i, a);
    }
    return adj;
  };
  LinkState ls = getLinkState(build(big));
  auto const& m = ls.csrMirror();
  auto id = [&](int i) { return m.id.at(std::to_string(i)); };
  // node 0 reaches node 7 over 1 + 1 + 1 + 1 + 3 x (2^31 - 1) > 2^32
  EXPECT_TRUE(spfMatchesOracle(ls, {id(3)}, false));  // hop counts: u32 rows
  EXPECT_TRUE(spfMatchesOracle(ls, {id(0), id(7)}, true));
  const auto v = ls.getSpfView("0");
  EXPECT_EQ(v.metric("7"), (uint64_t)4 + 3ull * (uint64_t)big);
  EXPECT_TRUE(spfMatchesOracle(ls, {id(1), id(5), id(2)}, true));
  // a metric change on the far links: attribute patch + refresh of the (now u64) rows
  for (auto const& [node, adjs] : build(big - 5))
    if (node >= n - 4) {
      std::vector<thrift::Adjacency> as;
      for (auto const& [o, w] : adjs)
        as.push_back(createAdjacency(std::to_string(o), std::to_string(node) + "/" + std::to_string(o) + "/0",
                                     std::to_string(o) + "/" + std::to_string(node) + "/0", w,
                                     (node << 16) + o));
      ls.updateAdjacencyDatabase(createAdjDb(std::to_string(node), as, node), 0, 0);
    }
  EXPECT_TRUE(spfMatchesOracle(ls, {id(0), id(7), id(1), id(5), id(2)}, true));
  EXPECT_EQ(ls.getSpfView("0").metric("7"), (uint64_t)4 + 3ull * (uint64_t)(big - 5));
}

int main(int argc, char** argv) { return run_tests(argc, argv); }
