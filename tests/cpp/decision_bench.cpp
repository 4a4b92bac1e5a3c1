// decision_bench.cpp — DecisionBenchmark through the drop-in (benchmark / test
// infrastructure: it links the oracle as the checker and as the faithful-cost CPU
// baseline; the timed path is the product only).
//
// Restates BM_DecisionGrid / BM_DecisionFabric
// (/root/reference/openr/decision/tests/DecisionBenchmark.cpp:12-29, RoutingBenchmarkUtils.cpp):
//   * topology: createGrid (:203-240: n x n grid, unit metrics, adjacency labels 100001 + id,
//     node label 0, numPrefixes = 1 prefix per node fc00:<id hi>::<id lo>/128 with the
//     benchmark's forwarding algorithm, SR_MPLS for KSP2_ED_ECMP) or createFabric
//     (:242-400: SSW 1-plane-i, FSW 2-pod-plane, RSW 3-pod-i; each SSW keeps only its pod-0
//     adjacency because of the `emplace` at :267-271; no prefixes);
//   * Decision runs with computeLfaPaths = true (RoutingBenchmarkUtils.h:77-85) and my node
//     "1" (grid) or "2-0-0" (fabric, :571);
//   * one iteration (updateRandomGridAdjs :453-479 / updateRandomFabricAdjs :406-447 +
//     sendRecvUpdate :52-79): a node's adjacency database is re-advertised with its
//     overload bit set (a random node) or cleared (the node of the previous iteration), and
//     Decision rebuilds its own route DB.
// Timed per iteration, through the drop-in only: LinkState::updateAdjacencyDatabase +
// SpfSolver::buildRouteDb(my node) (SPF on the GPU engine: patched device graph, memo rows
// refreshed, LFA neighbours and KSP2 paths prefetched in batches).
//
// After the timed loop (not timed):
//   --check     the last route DB against routes rebuilt from oracle SPF runs on the same
//               mirror (SP_ECMP: shortest next hops + RFC 5286 alternates, Decision.cpp:
//               1160-1257; KSP2_ED_ECMP: every destination's k = 1, 2 paths against
//               oracle_kth_paths, link for link, and the route DB against a call-by-call
//               build on a fresh LinkState);
//   --cpu-iters the reference's cost of the same iteration on this host: the SPF runs its
//               cleared memo re-runs (decision.spf_runs per iteration, counted by the
//               drop-in exactly where the reference counts them) timed on the
//               faithful-cost restatement of runSpf (oracle/spf_faithful.cpp, reference
//               data structures; KSP2's ignore-set runs are priced as plain runs from a
//               sample of sources), plus the route construction itself (the same
//               buildRouteDb with every SPF memoised: the host code is a restatement of
//               the reference's).
// Prints one JSON line.
//   decision_bench --topology grid|fabric --size N --algo sp|ksp2 [--iters K] [--warmup W]
//                  [--check] [--cpu-iters C] [--cpu-threads T (faithful runs timed on T threads;
//                  priced serial, as Decision runs them)] [--seed S]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../openr_amd/csrc/host/Decision.h"
#include "../../oracle/spf_oracle.h"

using namespace openr;

extern "C" int faithful_all_sources(const oracle_graph* g, const char* name_pool, const uint64_t* name_off,
                                    const uint32_t* sources, uint32_t n, int use_link_metric, int nthreads,
                                    uint64_t* dist, uint8_t* nh, uint32_t nh_bytes, double* out_seconds);

namespace {

const std::string kArea = "0";
using clk = std::chrono::steady_clock;
double msSince(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

std::string hex2(uint32_t x) {  // folly::sformat("{:02x}", num)
  char b[16];
  std::snprintf(b, sizeof(b), "%02x", x);
  return b;
}

thrift::Adjacency adjacency(const std::string& other, const std::string& ifName, const std::string& nhV6,
                            const std::string& nhV4, int32_t label, const std::string& otherIf) {
  thrift::Adjacency a;  // createThriftAdjacency(..., metric 1, label, false, rtt 100, ts 10000, weight 1, otherIf)
  a.otherNodeName = other;
  a.ifName = ifName;
  a.nextHopV6.addr = nhV6;
  a.nextHopV4.addr = nhV4;
  a.metric = 1;
  a.adjLabel = label;
  a.isOverloaded = false;
  a.rtt = 100;
  a.timestamp = 10000;
  a.weight = 1;
  a.otherIfName = otherIf;
  return a;
}

thrift::AdjacencyDatabase adjDb(const std::string& node, std::vector<thrift::Adjacency> adjs, bool overload) {
  thrift::AdjacencyDatabase db;  // createAdjDb(nodeId, adjs, 0 /* node label */, overloadBit)
  db.thisNodeName = node;
  db.isOverloaded = overload;
  db.adjacencies = std::move(adjs);
  db.nodeLabel = 0;
  db.area = kArea;
  return db;
}

// --- grid (RoutingBenchmarkUtils.cpp:80-101, 136-201) ---------------------------------
std::vector<thrift::Adjacency> gridAdjs(int row, int col, int n) {
  std::vector<thrift::Adjacency> adjs;
  const int id = row * n + col;
  auto add = [&](int r, int c) {
    if (r < 0 || r >= n || c < 0 || c >= n) return;
    const uint32_t other = (uint32_t)(r * n + c);
    const std::string ifn = "if_" + std::to_string(id) + "_" + std::to_string(other);
    const std::string oif = "if_" + std::to_string(other) + "_" + std::to_string(id);
    adjs.push_back(adjacency(std::to_string(other), ifn, "fe80:" + hex2(other >> 16) + "::" + hex2(other & 0xffff),
                             "10." + std::to_string(other >> 16) + "." + std::to_string((other >> 8) & 0xff) + "." +
                                 std::to_string(other & 0xff),
                             (int32_t)(100001 + other), oif));
  };
  add(row, col + 1);  // createGridAdjacencys order: east, west, north, south
  add(row, col - 1);
  add(row - 1, col);
  add(row + 1, col);
  return adjs;
}

// --- fabric (RoutingBenchmarkUtils.cpp:103-134, 242-400) -------------------------------
constexpr int kSsw = 1, kFsw = 2, kRsw = 3, kSswsPerPlane = 36, kFswsPerPod = 8, kRswsPerPod = 48;
std::string fabName(int m, int a, int b) { return std::to_string(m) + "-" + std::to_string(a) + "-" + std::to_string(b); }
void fabAdj(const std::string& src, int m, int pod, int sw, std::vector<thrift::Adjacency>& adjs) {
  const std::string other = fabName(m, pod, sw);
  adjs.push_back(adjacency(other, "if_" + src + "_" + other, "fe80:" + hex2(m) + ":" + hex2(pod) + "::" + hex2(sw),
                           std::to_string(m) + "." + std::to_string(pod >> 8) + "." + std::to_string(pod & 0xff) + "." +
                               std::to_string(sw),
                           m * 100000 + pod * 100 + sw, "if_" + other + "_" + src));
}
std::vector<thrift::Adjacency> rswAdjs(int pod, int r) {
  std::vector<thrift::Adjacency> adjs;
  for (int f = 0; f < kFswsPerPod; ++f) fabAdj(fabName(kRsw, pod, r), kFsw, pod, f, adjs);
  return adjs;
}

struct Options {
  std::string topology = "grid", algo = "sp";
  uint32_t size = 10000, iters = 20, warmup = 2, cpuIters = 0, cpuThreads = 1;
  uint64_t seed = 1;
  bool check = false;
  bool allRoutes = false;  // --all-routes: every node's route DB (buildRouteDbs), host-side profiling
  size_t routeNodes = 0;   // --route-nodes N: only the first N nodes' DBs (profiling at full size)
  bool nodeLabels = false; // --node-labels: grid node labels (node-label MPLS routes in every DB)
  uint32_t routeIters = 0;  // --route-iters N: N memoised rebuilds of my route DB, then exit (profiling)
  // --fabric-prefixes: the intended fabric benchmark: one prefix per node (the reference's
  // createFabric advertises none, RoutingBenchmarkUtils.cpp:355-400, so its route build
  // runs no SPF; prefixes fd00:<i>::/128 in node-name order) and every SSW linked to its
  // plane's FSW in every pod (createFabric's emplace keeps the pod-0 adjacency only, which
  // leaves pods 1.. unreachable from pod 0)
  bool fabricPrefixes = false;
};

struct Bench {
  Options o;
  std::unordered_map<std::string, LinkState> als;
  PrefixState ps;
  std::string me;
  int n = 0, pods = 0;  // grid side / fabric pods
  bool ksp2 = false;
  std::mt19937_64 rng;
  std::optional<std::pair<int, int>> selected;  // the node of the previous iteration
  std::map<std::string, std::string> prefixOwner;  // advertised prefix (string form) -> node name

  explicit Bench(const Options& opt) : o(opt), rng(opt.seed) {
    ksp2 = o.algo == "ksp2";
    als.emplace(kArea, LinkState(kArea));
    LinkState& ls = als.at(kArea);
    if (o.topology == "grid") {
      n = (int)std::sqrt((double)o.size);
      me = "1";
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
          const uint32_t id = (uint32_t)(r * n + c);
          auto db = adjDb(std::to_string(id), gridAdjs(r, c, n), false);
          if (o.nodeLabels) db.nodeLabel = 100001 + id;  // profiling: node-label MPLS routes as openr_routes builds
          ls.updateAdjacencyDatabase(db);
          thrift::PrefixEntry e;  // createPrefixEntry(nodeToPrefixV6(nodeId + 0)), forwardingAlgorithm
          e.prefix = thrift::IpPrefix{"fc00:" + hex2(id >> 16) + "::" + hex2(id & 0xffff), 128};
          if (ksp2) {
            e.forwardingAlgorithm = thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
            e.forwardingType = thrift::PrefixForwardingType::SR_MPLS;
          }
          ps.updatePrefix(std::to_string(id), kArea, e);
          prefixOwner[e.prefix.toString()] = std::to_string(id);
        }
    } else {
      const int planes = kFswsPerPod;
      pods = ((int)o.size - planes * kSswsPerPlane) / (kFswsPerPod + kRswsPerPod);
      me = fabName(kFsw, 0, 0);
      for (int p = 0; p < planes; ++p)
        for (int s = 0; s < kSswsPerPlane; ++s) {  // emplace keeps the pod-0 adjacency only
          std::vector<thrift::Adjacency> adjs;
          // (the intended fabric: an SSW of plane p reaches FSW p of every pod)
          for (int pod = 0; pod < (o.fabricPrefixes ? pods : 1); ++pod) fabAdj(fabName(kSsw, p, s), kFsw, pod, p, adjs);
          ls.updateAdjacencyDatabase(adjDb(fabName(kSsw, p, s), adjs, false));
        }
      for (int pod = 0; pod < pods; ++pod)
        for (int f = 0; f < kFswsPerPod; ++f) {
          std::vector<thrift::Adjacency> adjs;
          for (int s = 0; s < kSswsPerPlane; ++s) fabAdj(fabName(kFsw, pod, f), kSsw, f, s, adjs);
          for (int r = 0; r < kRswsPerPod; ++r) fabAdj(fabName(kFsw, pod, f), kRsw, pod, r, adjs);
          ls.updateAdjacencyDatabase(adjDb(fabName(kFsw, pod, f), adjs, false));
        }
      for (int pod = 0; pod < pods; ++pod)
        for (int r = 0; r < kRswsPerPod; ++r) ls.updateAdjacencyDatabase(adjDb(fabName(kRsw, pod, r), rswAdjs(pod, r), false));
      if (o.fabricPrefixes) {
        std::vector<std::string> names;
        for (auto const& [name, _] : ls.getAdjacencyDatabases()) names.push_back(name);
        std::sort(names.begin(), names.end());
        for (uint32_t i = 0; i < names.size(); ++i) {
          thrift::PrefixEntry e;
          e.prefix = thrift::IpPrefix{"fd00:" + hex2(i >> 16) + "::" + hex2(i & 0xffff), 128};
          if (ksp2) {
            e.forwardingAlgorithm = thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
            e.forwardingType = thrift::PrefixForwardingType::SR_MPLS;
          }
          ps.updatePrefix(names[i], kArea, e);
          prefixOwner[e.prefix.toString()] = names[i];
        }
      }
    }
  }

  // updateRandomGridAdjs / updateRandomFabricAdjs: the re-advertised database
  thrift::AdjacencyDatabase nextUpdate() {
    const bool revert = selected.has_value();
    std::pair<int, int> s;
    if (revert) {
      s = *selected;
      selected.reset();
    } else {
      s = o.topology == "grid" ? std::make_pair((int)(rng() % n), (int)(rng() % n))
                               : std::make_pair((int)(rng() % pods), (int)(rng() % kRswsPerPod));
      selected = s;
    }
    if (o.topology == "grid") return adjDb(std::to_string(s.first * n + s.second), gridAdjs(s.first, s.second, n), !revert);
    return adjDb(fabName(kRsw, s.first, s.second), rswAdjs(s.first, s.second), !revert);
  }
};

// --- oracle check (SP_ECMP): routes rebuilt from oracle SPF runs -----------------------
struct OracleRows {
  const LinkState::CsrMirror& m;
  oracle_graph og;
  uint32_t nb = 1;
  std::map<uint32_t, std::pair<std::vector<uint64_t>, std::vector<uint8_t>>> rows;
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
    if (oracle_run_spf(&og, s, 1, nullptr, d.data(), h.data(), nb, nullptr, nullptr, nullptr) < 0)
      throw std::runtime_error("oracle_run_spf failed");
    return rows.emplace(s, std::make_pair(std::move(d), std::move(h))).first->second;
  }
};

// The route SpfSolver builds for prefix p of node dst with LFA on (Decision.cpp:1160-1257):
// shortest next-hop nodes of dst, RFC 5286 alternates dn[dst] < dm[dst] + dn[me], every up
// link to such a node, metric = link metric + the node's distance (i32).
NextHopSet expectedRoute(OracleRows& o, uint32_t me, uint32_t dst) {
  const auto& m = o.m;
  const auto& [dm, hm] = o.of(me);
  NextHopSet out;
  if (dst == me || dm[dst] == UINT64_MAX) return out;
  std::vector<uint32_t> nbrs;
  for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e)
    if (std::find(nbrs.begin(), nbrs.end(), m.col[e]) == nbrs.end()) nbrs.push_back(m.col[e]);
  std::map<uint32_t, uint64_t> nhNodes;
  for (size_t i = 0; i < nbrs.size(); ++i)
    if ((hm[(size_t)dst * o.nb + i / 8] >> (i % 8)) & 1u) nhNodes[nbrs[i]] = dm[dst] - dm[nbrs[i]];
  for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e) {
    if (!m.edgeUp[e]) continue;
    const uint32_t nn = m.col[e];
    const auto& dn = o.of(nn).first;
    if (dn[dst] == UINT64_MAX) continue;
    if (dn[dst] < dm[dst] + dn[me]) {
      auto it = nhNodes.find(nn);
      if (it == nhNodes.end() || it->second > dn[dst]) nhNodes[nn] = dn[dst];
    }
  }
  for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e) {
    const uint32_t nn = m.col[e];
    auto it = nhNodes.find(nn);
    if (it == nhNodes.end() || !m.edgeUp[e]) continue;
    const auto& link = m.links[m.linkId[e]];
    const auto& meName = m.names[me];
    out.insert(createNextHop(link->getNhV6FromNode(meName), link->getIfaceFromNode(meName),
                             (int32_t)(m.metric[e] + it->second), std::nullopt, kArea, m.names[nn]));
  }
  return out;
}

std::string flatten(const DecisionRouteDb& db) {
  std::string s;
  auto nhs = [&](const NextHopSet& set) {
    for (auto const& nh : set) {
      s += nh.address.addr + "%" + nh.address.ifName.value_or("") + "@" + nh.neighborNodeName.value_or("") + "#" +
           std::to_string(nh.metric);
      if (nh.mplsAction) {
        s += "a" + std::to_string((int)nh.mplsAction->action);
        if (nh.mplsAction->pushLabels)
          for (int32_t l : *nh.mplsAction->pushLabels) s += "," + std::to_string(l);
      }
      s += ";";
    }
  };
  for (auto const& [p, r] : db.unicastRoutes) {
    s += p.toString();
    nhs(r.nexthops);
    s += "\n";
  }
  for (auto const& [l, r] : db.mplsRoutes) {
    s += std::to_string(l) + ":";
    nhs(r.nexthops);
    s += "\n";
  }
  return s;
}

std::string checkRoutes(Bench& b, const DecisionRouteDb& db) {
  LinkState& ls = b.als.at(kArea);
  const auto& m = ls.csrMirror();
  const uint32_t me = m.id.at(b.me);
  OracleRows o(m);
  size_t bad = 0, checked = 0;
  if (!b.ksp2) {
    std::map<std::string, uint32_t> owner;  // prefix -> node id
    size_t reachable = 0;
    const auto& dm = o.of(me).first;
    for (auto const& [prefix, node] : b.prefixOwner) {
      const uint32_t v = m.id.at(node);
      owner[prefix] = v;
      reachable += v != me && dm[v] != UINT64_MAX;
    }
    ++checked;  // the route count: every reachable advertiser other than me
    if (db.unicastRoutes.size() != reachable) ++bad;
    for (auto const& [p, route] : db.unicastRoutes) {
      ++checked;
      if (route.nexthops != expectedRoute(o, me, owner.at(p.toString()))) ++bad;
    }
  } else {
    // every destination's k = 1, 2 paths vs the oracle, link for link
    const uint32_t NE = o.og.num_dir_edges;
    std::vector<uint32_t> pptr(NE + 2), pe(NE + 2);
    for (uint32_t d = 0; d < m.names.size(); ++d)
      for (uint32_t k = 1; k <= 2; ++k) {
        auto const& paths = ls.getKthPaths(b.me, m.names[d], k);
        const int64_t np = oracle_kth_paths(&o.og, me, d, k, pptr.data(), NE + 1, pe.data(), NE + 1);
        bool same = np >= 0 && (size_t)np == paths.size();
        for (int64_t i = 0; same && i < np; ++i) {
          same = paths[i].size() == pptr[i + 1] - pptr[i];
          for (uint32_t j = 0; same && j < paths[i].size(); ++j)
            same = paths[i][j].get() == m.links[m.linkId[pe[pptr[i] + j]]].get();
        }
        ++checked;
        bad += !same;
      }
    // the prefetched route DB against a call-by-call build on a fresh LinkState
    std::unordered_map<std::string, LinkState> fresh;
    fresh.emplace(kArea, LinkState(kArea));
    for (auto const& [name, adb] : ls.getAdjacencyDatabases()) fresh.at(kArea).updateAdjacencyDatabase(adb);
    setenv("OPENR_KSP2_PREFETCH", "0", 1);
    SpfSolver s2(b.me, false, true);
    auto db2 = s2.buildRouteDb(b.me, fresh, b.ps);
    unsetenv("OPENR_KSP2_PREFETCH");
    ++checked;
    if (!db2 || flatten(*db2) != flatten(db)) ++bad;
  }
  char buf[128];
  std::snprintf(buf, sizeof(buf), "%s (%zu of %zu checks failed)", bad ? "MISMATCH" : "ok", bad, checked);
  return buf;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) throw std::invalid_argument("missing value for " + a);
      return argv[++i];
    };
    if (a == "--topology") o.topology = next();
    else if (a == "--size") o.size = (uint32_t)std::stoul(next());
    else if (a == "--algo") o.algo = next();
    else if (a == "--iters") o.iters = (uint32_t)std::stoul(next());
    else if (a == "--warmup") o.warmup = (uint32_t)std::stoul(next());
    else if (a == "--cpu-iters") o.cpuIters = (uint32_t)std::stoul(next());
    else if (a == "--cpu-threads") o.cpuThreads = (uint32_t)std::stoul(next());
    else if (a == "--seed") o.seed = std::stoull(next());
    else if (a == "--check") o.check = true;
    else if (a == "--all-routes") o.allRoutes = true;
    else if (a == "--route-nodes" && i + 1 < argc) o.routeNodes = std::stoul(argv[++i]);
    else if (a == "--node-labels") o.nodeLabels = true;
    else if (a == "--route-iters") o.routeIters = (uint32_t)std::stoul(next());
    else if (a == "--fabric-prefixes") o.fabricPrefixes = true;
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if ((o.topology != "grid" && o.topology != "fabric") || (o.algo != "sp" && o.algo != "ksp2")) {
    std::fprintf(stderr, "--topology grid|fabric, --algo sp|ksp2\n");
    return 2;
  }
  try {
    const auto tb = clk::now();
    Bench b(o);
    LinkState& ls = b.als.at(kArea);
    if (o.allRoutes) {
      // every node's route DB through the streaming buildRouteDbs (the routes workload of
      // bench.py / openr_routes_build), tallied and freed on the building worker
      std::vector<std::string> nodes(ls.csrMirror().names);
      if (o.routeNodes && o.routeNodes < nodes.size()) nodes.resize(o.routeNodes);
      SpfSolver all(nodes[0], false, false);
      std::vector<uint64_t> cnt(nodes.size());
      double best = 1e30;
      for (uint32_t it = 0; it < std::max<uint32_t>(o.iters, 1); ++it) {
        const auto t0 = clk::now();
        std::atomic<uint64_t> tallyNs{0}, freeNs{0};
        all.buildRouteDbs(nodes, b.als, b.ps, [&](size_t i, std::optional<DecisionRouteDb>& db) {
          const auto c0 = clk::now();
          uint64_t c = 0;
          if (db)
            for (auto const& [p, r] : db->unicastRoutes) c += r.nexthops.size();
          cnt[i] = c;
          const auto c1 = clk::now();
          db.reset();
          const auto c2 = clk::now();
          tallyNs += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count();
          freeNs += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(c2 - c1).count();
        });
        best = std::min(best, msSince(t0));
        long hwm = 0;
        if (FILE* f = std::fopen("/proc/self/status", "r")) {
          char line[256];
          while (std::fgets(line, sizeof(line), f))
            if (!std::strncmp(line, "VmHWM:", 6)) hwm = std::atol(line + 6);
          std::fclose(f);
        }
        std::fprintf(stderr, "all-routes: tally %.1f ms, free %.1f ms (thread-summed), peak RSS %.0f MB\n",
                     tallyNs.load() / 1e6, freeNs.load() / 1e6, hwm / 1024.0);
      }
      uint64_t nhs = 0;
      for (auto c : cnt) nhs += c;
      std::printf("{\"workload\": \"all-routes\", \"nodes\": %zu, \"ms_best\": %.1f, \"nexthops\": %llu}\n",
                  nodes.size(), best, (unsigned long long)nhs);
      return 0;
    }
    SpfSolver solver(b.me, false, true);  // Decision(config, computeLfaPaths = true, ...)
    // initial publication: the first route DB (RoutingBenchmarkUtils.cpp:535-538)
    auto t0 = clk::now();
    auto db = solver.buildRouteDb(b.me, b.als, b.ps);
    const double msInitial = msSince(t0);
    const double msSetup = msSince(tb);
    if (!db) throw std::runtime_error("my node is not in the topology");
    if (o.routeIters) {  // route construction alone (every SPF memoised), for profilers
      const auto r0 = clk::now();
      for (uint32_t r = 0; r < o.routeIters; ++r) db = solver.buildRouteDb(b.me, b.als, b.ps);
      std::printf("{\"workload\": \"route-iters\", \"ms_per_build\": %.3f, \"routes\": %zu}\n",
                  msSince(r0) / o.routeIters, db->unicastRoutes.size());
      return 0;
    }
    double msUpdate = 0, msBuild = 0;
    uint64_t runs = 0, routes = 0;
    std::vector<double> per;
    for (uint32_t it = 0; it < o.warmup + o.iters; ++it) {
      auto upd = b.nextUpdate();
      SpfCounters::get().reset();
      const auto a0 = clk::now();
      auto ch = ls.updateAdjacencyDatabase(std::move(upd));
      const auto a1 = clk::now();
      db = solver.buildRouteDb(b.me, b.als, b.ps);
      const auto a2 = clk::now();
      if (!ch.topologyChanged || !db) throw std::runtime_error("update did not change the topology / no route DB");
      if (it < o.warmup) continue;
      msUpdate += std::chrono::duration<double, std::milli>(a1 - a0).count();
      msBuild += std::chrono::duration<double, std::milli>(a2 - a1).count();
      per.push_back(std::chrono::duration<double, std::milli>(a2 - a0).count());
      runs += SpfCounters::get().spfRuns();
      routes = db->unicastRoutes.size() + db->mplsRoutes.size();
    }
    const double K = std::max<uint32_t>(o.iters, 1);
    std::sort(per.begin(), per.end());
    std::string check = "skipped";
    if (o.check) check = checkRoutes(b, *db);
    // CPU leg: the reference's cost of one iteration on this host
    std::string cpu = "null";
    if (o.cpuIters) {
      const auto& m = ls.csrMirror();
      oracle_graph og{(uint32_t)m.names.size(), (uint32_t)m.col.size(), (uint32_t)m.links.size(), m.rowPtr.data(),
                      m.col.data(), m.metric.data(), m.linkId.data(), m.edgeUp.data(), m.overloaded.data(),
                      m.nameRank.data()};
      std::string pool;
      std::vector<uint64_t> off{0};
      for (auto const& nm : m.names) {
        pool += nm;
        off.push_back(pool.size());
      }
      // sources: my node + my neighbours (SP_ECMP with LFA); KSP2 adds one ignore-set run per
      // destination, priced from a sample of sources
      const double runsPerIter = (double)runs / K;
      const uint32_t me = m.id.at(b.me);
      std::vector<uint32_t> srcs{me};
      for (uint32_t e = m.rowPtr[me]; e < m.rowPtr[me + 1]; ++e) srcs.push_back(m.col[e]);
      const uint32_t want = (uint32_t)std::min<double>(std::max<double>(runsPerIter, 1.0), 64.0);
      for (uint32_t v = 0; srcs.size() < want && v < m.names.size(); v += std::max<uint32_t>(1, (uint32_t)m.names.size() / want))
        srcs.push_back(v);
      srcs.resize(std::min<size_t>(srcs.size(), std::max<uint32_t>(want, 1)));
      double spfSec = 0;
      for (uint32_t r = 0; r < o.cpuIters; ++r) {
        double sec = 0;
        if (faithful_all_sources(&og, pool.data(), off.data(), srcs.data(), (uint32_t)srcs.size(), 1,
                                 (int)o.cpuThreads, nullptr, nullptr, 1, &sec) != 0)
          throw std::runtime_error("faithful_all_sources failed");
        spfSec += sec;
      }
      const double msPerSpf = 1e3 * spfSec / o.cpuIters / (double)srcs.size();
      // route construction alone: the same build with every SPF memoised (a second call)
      double msRoutes = 0;
      for (uint32_t r = 0; r < o.cpuIters; ++r) {
        const auto c0 = clk::now();
        auto db3 = solver.buildRouteDb(b.me, b.als, b.ps);
        msRoutes += msSince(c0);
      }
      msRoutes /= o.cpuIters;
      // Decision rebuilds on one thread: the runs are serial. The adjacency update is the
      // same host LinkState work on both sides (its mirror patch included), so it is priced
      // at the measured update time.
      const double msAdj = msUpdate / K;
      const double msIter = msAdj + runsPerIter * msPerSpf + msRoutes;
      char buf[640];
      std::snprintf(buf, sizeof(buf),
                    "{\"ms_per_update\": %.3f, \"ms_update_adjdb\": %.3f, \"spf_runs_per_update\": %.1f, \"ms_per_spf\": %.3f, "
                    "\"ms_route_construction\": %.3f, \"cores\": 1, \"timing_threads\": %u, \"kind\": \"port\", \"sample\": \"%zu faithful "
                    "runSpf (oracle/spf_faithful.cpp) x %u, priced per run; route construction timed on the memoised "
                    "build; adjacency update as measured\"}",
                    msIter, msAdj, runsPerIter, msPerSpf, msRoutes, o.cpuThreads, srcs.size(), o.cpuIters);
      cpu = buf;
    }
    const auto& m = ls.csrMirror();
    std::printf(
        "{\"workload\": \"decision\", \"topology\": \"%s\", \"fabric_prefixes\": %s, \"size\": %u, \"nodes\": %zu, \"links\": %zu, "
        "\"algo\": \"%s\", \"my_node\": \"%s\", \"lfa\": true, \"iters\": %u, \"warmup\": %u, "
        "\"ms_per_update\": %.4f, \"ms_update_adjdb\": %.4f, \"ms_build_route_db\": %.4f, \"median_ms\": %.4f, "
        "\"spf_runs_per_update\": %.2f, \"routes\": %llu, \"ms_initial_route_db\": %.2f, \"ms_setup\": %.1f, "
        "\"check\": \"%s\", \"cpu_baseline\": %s}\n",
        o.topology.c_str(), o.fabricPrefixes ? "true" : "false", o.size, m.names.size(), m.links.size(), b.ksp2 ? "KSP2_ED_ECMP" : "SP_ECMP", b.me.c_str(),
        o.iters, o.warmup, (msUpdate + msBuild) / K, msUpdate / K, msBuild / K, per.empty() ? 0.0 : per[per.size() / 2],
        (double)runs / K, (unsigned long long)routes, msInitial, msSetup, check.c_str(), cpu.c_str());
    return check.rfind("MISMATCH", 0) == 0 ? 1 : 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "decision_bench: %s\n", e.what());
    return 1;
  }
}
