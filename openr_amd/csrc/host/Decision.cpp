// Decision.cpp — host mirror of openr::SpfSolver route build and openr::RibPolicy
// (see Decision.h). Each function names the reference lines it follows; the SPF results
// it reads come from the engine through LinkState (one batched prefetch per build).
#include "Decision.h"

#include "HostParallel.h"

#include <algorithm>
#include <limits>
#include <list>
#include <stdexcept>
#include <tuple>

namespace openr {

// --- Util.h / Util.cpp helpers ----------------------------------------------

bool isMplsLabelValid(int32_t mplsLabel) { return (mplsLabel & 0xfff00000) == 0; }  // Util.h:284

thrift::NextHopThrift createNextHop(thrift::BinaryAddress addr, std::optional<std::string> ifName, int32_t metric,
                                    std::optional<thrift::MplsAction> mplsAction,
                                    const std::optional<std::string>& area,
                                    const std::optional<std::string>& neighborNodeName) {  // Util.cpp:936-951
  thrift::NextHopThrift nh;
  nh.address = std::move(addr);
  nh.address.ifName = std::move(ifName);
  nh.metric = metric;
  nh.mplsAction = std::move(mplsAction);
  nh.area = area;
  nh.neighborNodeName = neighborNodeName;
  return nh;
}

thrift::MplsAction createMplsAction(thrift::MplsActionCode code, std::optional<int32_t> swapLabel,
                                    std::optional<std::vector<int32_t>> pushLabels) {  // Util.cpp:954-964
  thrift::MplsAction a;
  a.action = code;
  a.swapLabel = swapLabel;
  a.pushLabels = std::move(pushLabels);
  // checkMplsAction (Util.cpp:640-670): the label fields must match the action
  const bool swapOk = (code == thrift::MplsActionCode::SWAP) == a.swapLabel.has_value();
  const bool pushOk = (code == thrift::MplsActionCode::PUSH) == a.pushLabels.has_value();
  if (!swapOk || !pushOk) throw std::invalid_argument("inconsistent MplsAction");
  if (a.swapLabel && !isMplsLabelValid(*a.swapLabel)) throw std::invalid_argument("invalid swap label");
  if (a.pushLabels)
    for (int32_t l : *a.pushLabels)
      if (!isMplsLabelValid(l)) throw std::invalid_argument("invalid push label");
  return a;
}

// Util.h:548-578: (path_preference, source_preference, -distance), higher wins; the
// running best starts at (0, 0, 0), so entries below it are never selected.
std::set<NodeAndArea> selectBestPrefixMetrics(PrefixEntries const& prefixes) {
  std::tuple<int32_t, int32_t, int32_t> best{0, 0, 0};
  std::set<NodeAndArea> keys;
  for (auto const& [key, entry] : prefixes) {
    const std::tuple<int32_t, int32_t, int32_t> t{entry.metrics.path_preference, entry.metrics.source_preference,
                                                  entry.metrics.distance * -1};
    if (t < best) continue;
    if (t > best) {
      best = t;
      keys.clear();
    }
    keys.emplace(key);
  }
  return keys;
}

NodeAndArea selectBestNodeArea(std::set<NodeAndArea> const& all, std::string const& me) {  // Util.cpp:1057-1068
  NodeAndArea best = *all.begin();
  for (auto const& na : all)
    if (na.first == me) {
      best = na;
      break;
    }
  return best;
}

std::pair<thrift::PrefixForwardingType, thrift::PrefixForwardingAlgorithm> getPrefixForwardingTypeAndAlgorithm(
    const PrefixEntries& prefixEntries, const std::set<NodeAndArea>& bestNodeAreas) {  // Util.cpp:617-639
  std::pair<thrift::PrefixForwardingType, thrift::PrefixForwardingAlgorithm> r{
      thrift::PrefixForwardingType::SR_MPLS, thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP};
  if (prefixEntries.empty()) return {thrift::PrefixForwardingType::IP, thrift::PrefixForwardingAlgorithm::SP_ECMP};
  for (auto const& [na, e] : prefixEntries) {
    if (!bestNodeAreas.count(na)) continue;
    r.first = std::min(r.first, e.forwardingType);
    r.second = std::min(r.second, e.forwardingAlgorithm);
    if (r.first == thrift::PrefixForwardingType::IP && r.second == thrift::PrefixForwardingAlgorithm::SP_ECMP)
      return r;
  }
  return r;
}

// --- PrefixState ------------------------------------------------------------

void PrefixState::updatePrefix(const std::string& node, const std::string& area, const thrift::PrefixEntry& entry) {
  prefixes_[entry.prefix].insert_or_assign({node, area}, entry);
}

void PrefixState::deletePrefix(const std::string& node, const std::string& area, const thrift::IpPrefix& prefix) {
  auto it = prefixes_.find(prefix);
  if (it == prefixes_.end()) return;
  it->second.erase({node, area});
  if (it->second.empty()) prefixes_.erase(it);
}

// --- SpfSolver ----------------------------------------------------------------

SpfSolver::SpfSolver(const std::string& myNodeName, bool enableV4, bool computeLfaPaths, bool enableOrderedFib,
                     bool bgpDryRun, bool enableBestRouteSelection)
    : myNodeName_(myNodeName),
      enableV4_(enableV4),
      computeLfaPaths_(computeLfaPaths),
      enableOrderedFib_(enableOrderedFib),
      bgpDryRun_(bgpDryRun),
      enableBestRouteSelection_(enableBestRouteSelection) {}

void SpfSolver::updateStaticMplsRoutes(const std::unordered_map<int32_t, std::vector<thrift::NextHopThrift>>& add,
                                       const std::vector<int32_t>& del) {
  for (auto const& [label, nhs] : add) staticMplsRoutes_[label] = nhs;
  for (int32_t label : del) staticMplsRoutes_.erase(label);
}

// The SPFs a route build of `me` reads: me, and with LFA every up neighbour
// (Decision.cpp:1138, :1177) — one engine batch per area.
void SpfSolver::prefetch(const std::string& me, std::unordered_map<std::string, LinkState> const& als) const {
  for (auto const& [area, ls] : als) {
    if (!ls.hasNode(me)) continue;
    std::vector<std::string> nodes{me};
    if (computeLfaPaths_)
      for (auto const& link : ls.linksFromNode(me))
        if (link->isUp()) nodes.push_back(link->getOtherNodeName(me));
    ls.prefetchSpfResults(nodes, true);
  }
}

std::vector<std::optional<DecisionRouteDb>> SpfSolver::buildRouteDbs(
    const std::vector<std::string>& nodes, std::unordered_map<std::string, LinkState> const& als,
    PrefixState const& prefixState) {
  std::vector<std::optional<DecisionRouteDb>> out(nodes.size());
  buildRouteDbs(nodes, als, prefixState, [&](size_t i, std::optional<DecisionRouteDb>& db) { out[i] = std::move(db); });
  return out;
}

void SpfSolver::buildRouteDbs(const std::vector<std::string>& nodes,
                              std::unordered_map<std::string, LinkState> const& als, PrefixState const& prefixState,
                              const std::function<void(size_t, std::optional<DecisionRouteDb>&)>& sink) {
  // KSP2 builds memoise k-th paths and run link-ignoring SPFs as they go (getKthPaths):
  // those stay on this thread. Every other build only reads memoised SPFs once the
  // prefetch below has run, so nodes are built by independent solver copies.
  bool ksp2 = false;
  for (auto const& [_, entries] : prefixState.prefixes()) {
    for (auto const& [na, e] : entries) ksp2 |= e.forwardingAlgorithm == thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
    if (ksp2) break;
  }
  const unsigned workers = ksp2 ? 1u : parallelWorkers(nodes.size(), 1);
  auto known = [&](const std::string& n) {
    for (auto const& [_, ls] : als)
      if (ls.hasNode(n)) return true;
    return false;
  };
  for (auto const& [area, ls] : als) {  // one all-sources batch covers every node and its neighbours
    std::vector<std::string> present;
    for (auto const& n : nodes)
      // also the self-only result of a node this area lacks but another has
      // (createRouteForPrefix and the label routes read it in every area): prefetched
      // results count as SPF runs only when read, so counters equal the one-thread loop's
      if (ls.hasNode(n) || known(n)) present.push_back(n);
    if (computeLfaPaths_) {
      std::set<std::string> more(present.begin(), present.end());
      for (auto const& n : present)
        if (ls.hasNode(n))
          for (auto const& link : ls.linksFromNode(n))
            if (link->isUp()) more.insert(link->getOtherNodeName(n));
      present.assign(more.begin(), more.end());
    }
    ls.prefetchSpfResults(present, true);
  }
  if (workers <= 1) {
    for (size_t i = 0; i < nodes.size(); ++i) {
      auto db = buildRouteDb(nodes[i], als, prefixState);
      sink(i, db);
    }
    return;
  }
  std::vector<SpfSolver> solvers(workers, *this);  // config + static MPLS routes
  for (auto& s : solvers) {
    s.counters_ = DecisionCounters{};
    s.bestRoutesCache_.clear();
  }
  // the sequential loop leaves the cache of the last node some area knows (an unknown
  // node's build returns before touching it)
  size_t last = nodes.size();
  for (size_t i = nodes.size(); i-- > 0;)
    if (known(nodes[i])) {
      last = i;
      break;
    }
  {
    // the workers only read memoised SPFs: a read the prefetch above missed throws
    std::vector<std::unique_ptr<LinkState::MemoFreeze>> frozen;
    for (auto const& [_, ls] : als) frozen.push_back(std::make_unique<LinkState::MemoFreeze>(ls));
    parallelFor(nodes.size(), 1, workers, [&](unsigned w, size_t i) {
      auto db = solvers[w].buildRouteDb(nodes[i], als, prefixState);
      if (i == last) bestRoutesCache_ = solvers[w].bestRoutesCache_;
      sink(i, db);
    });
  }
  for (auto const& s : solvers) {
    auto const& c = s.counters_;
    counters_.route_build_runs += c.route_build_runs;
    counters_.get_route_for_prefix += c.get_route_for_prefix;
    counters_.no_route_to_prefix += c.no_route_to_prefix;
    counters_.skipped_unicast_route += c.skipped_unicast_route;
    counters_.skipped_mpls_route += c.skipped_mpls_route;
    counters_.duplicate_node_label += c.duplicate_node_label;
    counters_.no_route_to_label += c.no_route_to_label;
    counters_.incompatible_forwarding_type += c.incompatible_forwarding_type;
  }
}

// Decision.cpp:568-734
std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(const std::string& myNodeName,
                                                       std::unordered_map<std::string, LinkState> const& als,
                                                       PrefixState const& prefixState) {
  bool nodeExist = false;
  for (auto const& [_, ls] : als) nodeExist |= ls.hasNode(myNodeName);
  if (!nodeExist) return std::nullopt;
  counters_.route_build_runs++;
  prefetch(myNodeName, als);

  // KSP2 prefixes: every destination's first and second paths from here in one device
  // launch per area (LinkState::prefetchKthPaths stages them; selectBestPathsKsp2's
  // getKthPaths calls then take them in the order and with the counts of the reference)
  std::unordered_map<std::string, std::vector<std::string>> ksp2Dests;
  for (auto const& [_, entries] : prefixState.prefixes()) {
    bool ksp2 = false;
    for (auto const& [na, e] : entries) ksp2 |= e.forwardingAlgorithm == thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP;
    if (ksp2)
      for (auto const& [na, e] : entries) ksp2Dests[na.second].push_back(na.first);
  }
  for (auto const& [area, dests] : ksp2Dests) {
    auto ls = als.find(area);
    if (ls != als.end() && ls->second.hasNode(myNodeName)) ls->second.prefetchKthPaths(myNodeName, dests);
  }

  DecisionRouteDb routeDb;
  bestRoutesCache_.clear();
  for (auto const& [prefix, _] : prefixState.prefixes())
    if (auto r = createRouteForPrefix(myNodeName, als, prefixState, prefix)) routeDb.addUnicastRoute(std::move(*r));

  // MPLS routes for every node label (:593-680)
  std::unordered_map<int32_t, std::pair<std::string, RibMplsEntry>> labelToNode;
  for (auto const& [area, ls] : als) {
    for (auto const& [_, adjDb] : ls.getAdjacencyDatabases()) {
      const int32_t topLabel = adjDb.nodeLabel;
      if (topLabel == 0) continue;  // non-SR mode
      if (!isMplsLabelValid(topLabel)) {
        counters_.skipped_mpls_route++;
        continue;
      }
      auto it = labelToNode.find(topLabel);
      if (it != labelToNode.end()) {  // collision: the bigger node name keeps the label
        counters_.duplicate_node_label++;
        if (it->second.first < adjDb.thisNodeName) continue;
      }
      if (adjDb.thisNodeName == myNodeName) {
        thrift::NextHopThrift nh;
        nh.address.addr = "::";
        nh.area = area;
        nh.mplsAction = createMplsAction(thrift::MplsActionCode::POP_AND_LOOKUP);
        labelToNode.erase(topLabel);
        labelToNode.emplace(topLabel, std::make_pair(adjDb.thisNodeName, RibMplsEntry{topLabel, {nh}}));
        continue;
      }
      auto metricNhs = getNextHopsWithMetric(myNodeName, {{adjDb.thisNodeName, area}}, false, als);
      if (metricNhs.second.empty()) {
        counters_.no_route_to_label++;
        continue;
      }
      labelToNode.erase(topLabel);
      labelToNode.emplace(
          topLabel,
          std::make_pair(adjDb.thisNodeName,
                         RibMplsEntry{topLabel, getNextHopsThrift(myNodeName, {{adjDb.thisNodeName, area}}, false,
                                                                  false, metricNhs.first, metricNhs.second, topLabel,
                                                                  als)}));
    }
  }
  for (auto& [_, nodeToEntry] : labelToNode) routeDb.addMplsRoute(std::move(nodeToEntry.second));

  // MPLS routes for our adjacencies (:686-714)
  for (auto const& [_, ls] : als) {
    for (auto const& link : ls.linksFromNode(myNodeName)) {
      const int32_t topLabel = link->getAdjLabelFromNode(myNodeName);
      if (topLabel == 0) continue;
      if (!isMplsLabelValid(topLabel)) {
        counters_.skipped_mpls_route++;
        continue;
      }
      routeDb.addMplsRoute(RibMplsEntry{
          topLabel,
          {createNextHop(link->getNhV6FromNode(myNodeName), link->getIfaceFromNode(myNodeName),
                         static_cast<int32_t>(link->getMetricFromNode(myNodeName)),
                         createMplsAction(thrift::MplsActionCode::PHP), link->getArea(),
                         link->getOtherNodeName(myNodeName))}});
    }
  }
  // static routes (:719-724)
  for (auto const& [topLabel, nhs] : staticMplsRoutes_)
    routeDb.addMplsRoute(RibMplsEntry{topLabel, NextHopSet(nhs.begin(), nhs.end())});
  return routeDb;
}

// Decision.cpp:401-566
std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(const std::string& myNodeName,
                                                               std::unordered_map<std::string, LinkState> const& als,
                                                               PrefixState const& prefixState,
                                                               thrift::IpPrefix const& prefix) {
  counters_.get_route_for_prefix++;
  auto search = prefixState.prefixes().find(prefix);
  if (search == prefixState.prefixes().end()) return std::nullopt;
  bestRoutesCache_.erase(prefix);

  // entries of reachable nodes only
  PrefixEntries prefixEntries = search->second;
  for (auto const& [area, ls] : als) {
    // dense read of the memoised SPF (an unknown node's result holds only itself)
    auto const mySpf = ls.getSpfView(myNodeName);
    for (auto it = prefixEntries.begin(); it != prefixEntries.end();) {
      const auto& [node, pArea] = it->first;
      if (area != pArea || mySpf.reached(node)) ++it;
      else it = prefixEntries.erase(it);
    }
  }
  if (prefixEntries.empty()) {
    counters_.no_route_to_prefix++;
    return std::nullopt;
  }
  const bool isV4Prefix = prefix.isV4();
  if (isV4Prefix && !enableV4_) {
    counters_.skipped_unicast_route++;
    return std::nullopt;
  }
  bool hasBGP = false, hasNonBGP = false, missingMv = false, hasSelfPrependLabel = true;
  for (auto const& [na, e] : prefixEntries) {
    const bool isBGP = e.type == thrift::PrefixType::BGP;
    hasBGP |= isBGP;
    hasNonBGP |= !isBGP;
    if (na.first == myNodeName) hasSelfPrependLabel &= e.prependLabel.has_value();
    if (isBGP && !e.mv.has_value()) missingMv = true;
  }
  if (hasBGP) {
    if (hasNonBGP && !enableBestRouteSelection_) {
      counters_.skipped_unicast_route++;
      return std::nullopt;
    }
    if (missingMv) {
      counters_.skipped_unicast_route++;
      return std::nullopt;
    }
  }
  const auto best = selectBestRoutes(myNodeName, prefix, prefixEntries, hasBGP, als);
  if (!best.success) return std::nullopt;
  if (best.allNodeAreas.empty()) {
    counters_.no_route_to_prefix++;
    return std::nullopt;
  }
  bestRoutesCache_.insert_or_assign(prefix, best);
  if (best.hasNode(myNodeName) && !hasSelfPrependLabel) return std::nullopt;  // self-originated

  const auto [forwardingType, forwardingAlgo] = getPrefixForwardingTypeAndAlgorithm(prefixEntries, best.allNodeAreas);
  switch (forwardingAlgo) {
    case thrift::PrefixForwardingAlgorithm::SP_ECMP:
      return selectBestPathsSpf(myNodeName, prefix, best, prefixEntries, hasBGP, forwardingType, als, prefixState);
    case thrift::PrefixForwardingAlgorithm::KSP2_ED_ECMP:
      return selectBestPathsKsp2(myNodeName, prefix, best, prefixEntries, hasBGP, forwardingType, als, prefixState);
  }
  return std::nullopt;
}

// Decision.cpp:736-764
BestRouteSelectionResult SpfSolver::selectBestRoutes(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                                     PrefixEntries const& prefixEntries, bool isBgp,
                                                     std::unordered_map<std::string, LinkState> const& als) {
  BestRouteSelectionResult ret;
  if (enableBestRouteSelection_) {
    ret.allNodeAreas = selectBestPrefixMetrics(prefixEntries);
    if (ret.allNodeAreas.empty()) return ret;  // success = false: nothing above (0, 0, 0)
    ret.bestNodeArea = selectBestNodeArea(ret.allNodeAreas, myNodeName);
    ret.success = true;
  } else if (isBgp) {
    return runBestPathSelectionBgp(prefix, prefixEntries, als);
  } else {
    for (auto const& [na, _] : prefixEntries) ret.allNodeAreas.emplace(na);
    ret.bestNodeArea = *ret.allNodeAreas.begin();
    ret.success = true;
  }
  return maybeFilterDrainedNodes(std::move(ret), als);
}

// Decision.cpp:806-848: the advertisers whose metric vector is best (ties broken by the
// tie-breaker entities are multipath); an undecidable order skips the route
BestRouteSelectionResult SpfSolver::runBestPathSelectionBgp(thrift::IpPrefix const& prefix,
                                                            PrefixEntries const& prefixEntries,
                                                            std::unordered_map<std::string, LinkState> const& als) {
  using MetricVectorUtils::CompareResult;
  (void)prefix;
  BestRouteSelectionResult ret;
  std::optional<thrift::MetricVector> bestVector;
  for (auto const& [na, e] : prefixEntries) {
    const CompareResult r =
        bestVector ? MetricVectorUtils::compareMetricVectors(e.mv.value(), *bestVector) : CompareResult::WINNER;
    switch (r) {
      case CompareResult::WINNER:
        ret.allNodeAreas.clear();
        [[fallthrough]];
      case CompareResult::TIE_WINNER:
        bestVector = e.mv.value();
        ret.bestNodeArea = na;
        [[fallthrough]];
      case CompareResult::TIE_LOOSER:
        ret.allNodeAreas.emplace(na);
        break;
      case CompareResult::TIE:    // "Tie ordering prefix entries. Skipping route" (logged, not counted:
      case CompareResult::ERROR:  // Decision.cpp:830-837; createRouteForPrefix :503-505 adds nothing)
        return ret;
      default:
        break;
    }
  }
  ret.success = true;
  return maybeFilterDrainedNodes(std::move(ret), als);
}

// Decision.cpp:782-802
BestRouteSelectionResult SpfSolver::maybeFilterDrainedNodes(BestRouteSelectionResult&& result,
                                                            std::unordered_map<std::string, LinkState> const& als) const {
  BestRouteSelectionResult filtered = result;
  for (auto it = filtered.allNodeAreas.begin(); it != filtered.allNodeAreas.end();) {
    const auto& [node, area] = *it;
    if (als.at(area).isNodeOverloaded(node)) it = filtered.allNodeAreas.erase(it);
    else ++it;
  }
  // As in the reference, `filtered` is a copy of `result`, so this never fires and a
  // drained best node stays bestNodeArea (its prefix entry still exists).
  if (!filtered.allNodeAreas.empty() && filtered.bestNodeArea != result.bestNodeArea)
    filtered.bestNodeArea = *filtered.allNodeAreas.begin();
  return filtered.allNodeAreas.empty() ? result : filtered;
}

// Decision.cpp:766-780
std::optional<int64_t> SpfSolver::getMinNextHopThreshold(BestRouteSelectionResult const& nodes,
                                                         PrefixEntries const& prefixEntries) const {
  std::optional<int64_t> mx;
  for (auto const& na : nodes.allNodeAreas) {
    auto const& e = prefixEntries.at(na);
    if (e.minNexthop && (!mx || *e.minNexthop > *mx)) mx = e.minNexthop;
  }
  return mx;
}

// Decision.cpp:841-906
std::optional<RibUnicastEntry> SpfSolver::selectBestPathsSpf(std::string const& myNodeName,
                                                             thrift::IpPrefix const& prefix,
                                                             BestRouteSelectionResult const& best,
                                                             PrefixEntries const& prefixEntries, bool isBgp,
                                                             thrift::PrefixForwardingType forwardingType,
                                                             std::unordered_map<std::string, LinkState> const& als,
                                                             PrefixState const& prefixState) {
  const bool isV4Prefix = prefix.isV4();
  const bool perDestination = forwardingType == thrift::PrefixForwardingType::SR_MPLS;
  auto filtered = best.allNodeAreas;
  if (best.hasNode(myNodeName) && perDestination) {
    for (auto const& [na, e] : prefixEntries)
      if (na.first == myNodeName && e.prependLabel) {
        filtered.erase(na);
        break;
      }
  }
  const auto nhm = getNextHopsWithMetric(myNodeName, filtered, perDestination, als);
  if (nhm.second.empty()) {
    counters_.no_route_to_prefix++;
    return std::nullopt;
  }
  return addBestPaths(myNodeName, prefix, best, prefixEntries, prefixState, isBgp,
                      getNextHopsThrift(myNodeName, best.allNodeAreas, isV4Prefix, perDestination, nhm.first,
                                        nhm.second, std::nullopt, als, prefixEntries));
}

// Decision.cpp:907-1030
std::optional<RibUnicastEntry> SpfSolver::selectBestPathsKsp2(std::string const& myNodeName,
                                                              thrift::IpPrefix const& prefix,
                                                              BestRouteSelectionResult const& best,
                                                              PrefixEntries const& prefixEntries, bool isBgp,
                                                              thrift::PrefixForwardingType forwardingType,
                                                              std::unordered_map<std::string, LinkState> const& als,
                                                              PrefixState const& prefixState) {
  if (forwardingType != thrift::PrefixForwardingType::SR_MPLS) {
    counters_.incompatible_forwarding_type++;
    return std::nullopt;
  }
  NextHopSet nextHops;
  std::vector<LinkState::Path> paths;
  for (auto const& [area, ls] : als) {
    for (auto const& [node, bestArea] : best.allNodeAreas) {
      if (node == myNodeName && bestArea == area) continue;
      for (auto const& path : ls.getKthPaths(myNodeName, node, 1)) paths.push_back(path);
    }
    const size_t firstPathsSize = paths.size();
    for (auto const& [node, bestArea] : best.allNodeAreas) {
      if (area != bestArea) continue;
      for (auto const& secPath : ls.getKthPaths(myNodeName, node, 2)) {
        bool add = true;
        for (size_t i = 0; i < firstPathsSize; ++i)
          if (LinkState::pathAInPathB(paths[i], secPath)) {  // avoid double spraying (anycast)
            add = false;
            break;
          }
        if (add) paths.push_back(secPath);
      }
    }
  }
  if (paths.empty()) return std::nullopt;
  for (auto const& path : paths) {
    for (auto const& [area, ls] : als) {
      Metric cost = 0;
      std::list<int32_t> labels;
      std::string nextNodeName = myNodeName;
      for (auto const& link : path) {
        cost += link->getMetricFromNode(nextNodeName);
        nextNodeName = link->getOtherNodeName(nextNodeName);
        labels.push_front(ls.getAdjacencyDatabases().at(nextNodeName).nodeLabel);
      }
      labels.pop_back();  // first node's label: PHP
      auto const& prefixEntry = prefixEntries.at({nextNodeName, area});
      if (prefixEntry.prependLabel) labels.push_front(*prefixEntry.prependLabel);
      auto const& firstLink = path.front();
      std::optional<thrift::MplsAction> mplsAction;
      if (!labels.empty())
        mplsAction = createMplsAction(thrift::MplsActionCode::PUSH, std::nullopt,
                                      std::vector<int32_t>(labels.begin(), labels.end()));
      nextHops.emplace(createNextHop(
          prefix.isV4() ? firstLink->getNhV4FromNode(myNodeName) : firstLink->getNhV6FromNode(myNodeName),
          firstLink->getIfaceFromNode(myNodeName), static_cast<int32_t>(cost), mplsAction, firstLink->getArea(),
          firstLink->getOtherNodeName(myNodeName)));
    }
  }
  return addBestPaths(myNodeName, prefix, best, prefixEntries, prefixState, isBgp, std::move(nextHops));
}

// Decision.cpp:1032-1092
std::optional<RibUnicastEntry> SpfSolver::addBestPaths(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                                       BestRouteSelectionResult const& best,
                                                       PrefixEntries const& prefixEntries,
                                                       PrefixState const& prefixState, bool isBgp,
                                                       NextHopSet&& nextHops) {
  (void)prefixState;
  const auto minNextHop = getMinNextHopThreshold(best, prefixEntries);
  if (minNextHop && *minNextHop > (int64_t)nextHops.size()) return std::nullopt;
  if (best.hasNode(myNodeName)) {
    std::optional<int32_t> prependLabel;
    for (auto const& [na, e] : prefixEntries)
      if (na.first == myNodeName && e.prependLabel) {
        prependLabel = e.prependLabel;
        break;
      }
    if (!prependLabel) throw std::logic_error("self route must be advertised with a prepend label");
    auto it = staticMplsRoutes_.find(*prependLabel);
    if (it != staticMplsRoutes_.end())
      for (auto const& nh : it->second) nextHops.emplace(createNextHop(nh.address, std::nullopt, 0, std::nullopt));
  }
  RibUnicastEntry e;
  e.prefix = prefix;
  e.nexthops = std::move(nextHops);
  e.bestPrefixEntry = prefixEntries.at(best.bestNodeArea);
  e.bestArea = best.bestNodeArea.second;
  e.doNotInstall = isBgp && bgpDryRun_;
  return e;
}

// Decision.cpp:1094-1117
std::pair<Metric, std::unordered_set<std::string>> SpfSolver::getMinCostNodes(
    const LinkState::SpfView& spf, const std::set<NodeAndArea>& dstNodeAreas) const {
  Metric shortest = std::numeric_limits<Metric>::max();
  std::unordered_set<std::string> nodes;
  for (auto const& [dst, _] : dstNodeAreas) {
    if (!spf.reached(dst)) continue;
    const Metric d = spf.metric(dst);
    if (shortest >= d) {
      if (shortest > d) {
        shortest = d;
        nodes.clear();
      }
      nodes.emplace(dst);
    }
  }
  return {shortest, std::move(nodes)};
}

// Decision.cpp:1119-1208 (LFA: RFC 5286 condition at :1192)
std::pair<Metric, std::unordered_map<std::pair<std::string, std::string>, Metric>> SpfSolver::getNextHopsWithMetric(
    const std::string& me, const std::set<NodeAndArea>& dstNodeAreas, bool perDestination,
    std::unordered_map<std::string, LinkState> const& als) const {
  std::unordered_map<std::pair<std::string, std::string>, Metric> nextHopNodes;
  Metric shortestMetric = std::numeric_limits<Metric>::max();
  for (auto const& [area, ls] : als) {
    // dense reads of the memoised SPFs (LinkState::SpfView): same results as getSpfResult,
    // no SpfResult map materialised per route build
    auto const fromHere = ls.getSpfView(me);
    auto const mm = getMinCostNodes(fromHere, dstNodeAreas);
    if (shortestMetric < mm.first) continue;
    if (shortestMetric > mm.first) {
      shortestMetric = mm.first;
      nextHopNodes.clear();
    }
    if (mm.second.empty()) continue;
    for (auto const& dst : mm.second) {
      const std::string dstRef = perDestination ? dst : "";
      // getMetricFromAToB(me, nh) reads the same (already counted) result: nh != me
      for (auto const& nh : fromHere.nextHops(dst))
        nextHopNodes[std::make_pair(nh, dstRef)] = shortestMetric - fromHere.metric(nh);
    }
    if (computeLfaPaths_) {
      for (auto const& link : ls.linksFromNode(me)) {
        if (!link->isUp()) continue;
        const auto& nbr = link->getOtherNodeName(me);
        auto const fromNbr = ls.getSpfView(nbr);
        const Metric nbrToHere = fromNbr.metric(me);
        for (auto const& [dst, dstArea] : dstNodeAreas) {
          if (area != dstArea) continue;
          if (!fromNbr.reached(dst)) continue;
          const Metric dNbr = fromNbr.metric(dst);
          if (dNbr < shortestMetric + nbrToHere) {  // RFC 5286
            const auto key = std::make_pair(nbr, perDestination ? dst : std::string());
            auto it = nextHopNodes.find(key);
            if (it == nextHopNodes.end()) nextHopNodes.emplace(key, dNbr);
            else if (it->second > dNbr) it->second = dNbr;
          }
        }
      }
    }
  }
  return {shortestMetric, nextHopNodes};
}

// Decision.cpp:1210-1317
NextHopSet SpfSolver::getNextHopsThrift(const std::string& me, const std::set<NodeAndArea>& dstNodeAreas, bool isV4,
                                        bool perDestination, Metric minMetric,
                                        std::unordered_map<std::pair<std::string, std::string>, Metric> nextHopNodes,
                                        std::optional<int32_t> swapLabel,
                                        std::unordered_map<std::string, LinkState> const& als,
                                        PrefixEntries const& prefixEntries) {
  if (nextHopNodes.empty()) throw std::logic_error("getNextHopsThrift: no next-hop nodes");
  NextHopSet nextHops;
  const std::set<NodeAndArea> anyDst{{"", ""}};
  for (auto const& [area, ls] : als) {
    for (auto const& link : ls.linksFromNode(me)) {
      for (auto const& [dstNode, dstArea] : perDestination ? dstNodeAreas : anyDst) {
        if (!dstArea.empty() && area != dstArea) continue;
        const auto& neighborNode = link->getOtherNodeName(me);
        const auto search = nextHopNodes.find(std::make_pair(neighborNode, dstNode));
        if (search == nextHopNodes.end() || !link->isUp()) continue;
        if (!dstNode.empty() && dstNodeAreas.count({neighborNode, area}) && neighborNode != dstNode) continue;
        const Metric distOverLink = link->getMetricFromNode(me) + search->second;
        if (!computeLfaPaths_ && distOverLink != minMetric) continue;
        std::optional<thrift::MplsAction> mplsAction;
        if (swapLabel) {
          const bool isNextHopAlsoDst = dstNodeAreas.count({neighborNode, area}) != 0;
          mplsAction = createMplsAction(isNextHopAlsoDst ? thrift::MplsActionCode::PHP : thrift::MplsActionCode::SWAP,
                                        isNextHopAlsoDst ? std::nullopt : swapLabel);
        }
        if (!dstNode.empty()) {
          std::vector<int32_t> pushLabels;
          auto const& dstPrefixEntry = prefixEntries.at({dstNode, area});
          if (dstPrefixEntry.prependLabel) {
            pushLabels.push_back(*dstPrefixEntry.prependLabel);
            if (!isMplsLabelValid(pushLabels.back())) continue;
          }
          if (dstNode != neighborNode) {
            pushLabels.push_back(ls.getAdjacencyDatabases().at(dstNode).nodeLabel);
            if (!isMplsLabelValid(pushLabels.back())) continue;
          }
          if (!pushLabels.empty())
            mplsAction = createMplsAction(thrift::MplsActionCode::PUSH, std::nullopt, std::move(pushLabels));
        }
        // createNextHop narrows the u64 distance to the i32 metric (Util.h:440-446)
        nextHops.emplace(createNextHop(isV4 ? link->getNhV4FromNode(me) : link->getNhV6FromNode(me),
                                       link->getIfaceFromNode(me), static_cast<int32_t>(distOverLink), mplsAction,
                                       link->getArea(), link->getOtherNodeName(me)));
      }
    }
  }
  return nextHops;
}

// --- RibPolicy (RibPolicy.cpp:61-111, 165-199) ----------------------------------

bool RibPolicyStatement::applyAction(RibUnicastEntry& route) const {
  if (!match(route)) return false;
  NextHopSet newNexthops;
  for (auto const& nh : route.nexthops) {
    int32_t w = defaultWeight;  // precedence: neighbour > area > default
    if (nh.area) {
      auto it = areaToWeight.find(*nh.area);
      if (it != areaToWeight.end()) w = it->second;
    }
    if (nh.neighborNodeName) {
      auto it = neighborToWeight.find(*nh.neighborNodeName);
      if (it != neighborToWeight.end()) w = it->second;
    }
    if (w > 0) {
      auto n = nh;
      n.weight = w;
      newNexthops.emplace(std::move(n));
    }
  }
  if (newNexthops.empty()) {  // every next-hop dropped: keep the route as is (RibPolicy.cpp:98-104)
    ++RibPolicyCounters::get().invalidatedRoutes;
    return false;
  }
  route.nexthops = std::move(newNexthops);
  return true;
}

RibPolicy::RibPolicy(std::vector<RibPolicyStatement> statements, int64_t ttlSecs)
    : statements_(std::move(statements)),
      validUntil_(std::chrono::steady_clock::now() + std::chrono::seconds(ttlSecs)) {
  if (statements_.empty()) throw std::invalid_argument("Missing policy.statements attribute");
  for (auto const& s : statements_)
    if (s.prefixes.empty()) throw std::invalid_argument("Missing policy_statement.matcher.prefixes attribute");
}

RibPolicyCounters& RibPolicyCounters::get() {
  static RibPolicyCounters c;
  return c;
}

bool RibPolicy::isActive() const { return validUntil_ > std::chrono::steady_clock::now(); }

bool RibPolicy::applyAction(RibUnicastEntry& route) const {
  for (auto const& s : statements_)
    if (s.applyAction(route)) return true;
  return false;
}

std::vector<thrift::IpPrefix> RibPolicy::applyPolicy(std::map<thrift::IpPrefix, RibUnicastEntry>& entries) const {
  std::vector<thrift::IpPrefix> updated;
  if (!isActive()) return updated;
  for (auto& [prefix, route] : entries)
    if (applyAction(route)) updated.push_back(prefix);
  return updated;
}

}  // namespace openr

// ---------------------------------------------------------------------------
// MetricVectorUtils (Util.cpp:1100-1246): entities compared in decreasing priority; a
// loner (type present on one side only) decides by its CompareType; tie-breaker
// entities give TIE_WINNER / TIE_LOOSER (multipath kept); the first decisive result wins.
// ---------------------------------------------------------------------------
namespace openr {
namespace MetricVectorUtils {

CompareResult operator!(CompareResult r) {
  switch (r) {
    case CompareResult::WINNER: return CompareResult::LOOSER;
    case CompareResult::TIE_WINNER: return CompareResult::TIE_LOOSER;
    case CompareResult::TIE: return CompareResult::TIE;
    case CompareResult::TIE_LOOSER: return CompareResult::TIE_WINNER;
    case CompareResult::LOOSER: return CompareResult::WINNER;
    case CompareResult::ERROR: return CompareResult::ERROR;
  }
  return CompareResult::ERROR;
}

bool isDecisive(CompareResult r) {
  return r == CompareResult::WINNER || r == CompareResult::LOOSER || r == CompareResult::ERROR;
}

bool isSorted(thrift::MetricVector const& mv) {
  int64_t prior = std::numeric_limits<int64_t>::max();
  for (auto const& e : mv.metrics) {
    if (e.priority > prior) return false;
    prior = e.priority;
  }
  return true;
}

CompareResult compareMetrics(std::vector<int64_t> const& l, std::vector<int64_t> const& r, bool tieBreaker) {
  if (l.size() != r.size()) return CompareResult::ERROR;
  for (size_t i = 0; i < l.size(); ++i) {
    if (l[i] > r[i]) return tieBreaker ? CompareResult::TIE_WINNER : CompareResult::WINNER;
    if (l[i] < r[i]) return tieBreaker ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
  }
  return CompareResult::TIE;
}

CompareResult resultForLoner(thrift::MetricEntity const& e) {
  if (e.op == thrift::CompareType::WIN_IF_PRESENT)
    return e.isBestPathTieBreaker ? CompareResult::TIE_WINNER : CompareResult::WINNER;
  if (e.op == thrift::CompareType::WIN_IF_NOT_PRESENT)
    return e.isBestPathTieBreaker ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
  return CompareResult::TIE;  // IGNORE_IF_NOT_PRESENT
}

void maybeUpdate(CompareResult& target, CompareResult update) {
  if (isDecisive(update) || target == CompareResult::TIE) target = update;
}

// Util.cpp:1143-1157: the reference sorts its (const) arguments in place by decreasing
// priority (std::sort through a const_cast); the caller observes the sorted order, which
// its own tests rely on (UtilTest.cpp:952-956 index the vectors after a comparison)
void sortMetricVector(thrift::MetricVector const& mv) {
  if (isSorted(mv)) return;
  auto& m = const_cast<std::vector<thrift::MetricEntity>&>(mv.metrics);
  std::sort(m.begin(), m.end(),
            [](thrift::MetricEntity const& a, thrift::MetricEntity const& b) { return a.priority > b.priority; });
}

CompareResult compareMetricVectors(thrift::MetricVector const& lv, thrift::MetricVector const& rv) {
  CompareResult result = CompareResult::TIE;
  if (lv.version != rv.version) return CompareResult::ERROR;
  sortMetricVector(lv);
  sortMetricVector(rv);
  auto const &l = lv.metrics, &r = rv.metrics;
  auto li = l.begin(), ri = r.begin();
  while (!isDecisive(result) && li != l.end() && ri != r.end()) {
    if (li->type == ri->type) {
      if (li->isBestPathTieBreaker != ri->isBestPathTieBreaker) maybeUpdate(result, CompareResult::ERROR);
      else maybeUpdate(result, compareMetrics(li->metric, ri->metric, li->isBestPathTieBreaker));
      ++li;
      ++ri;
    } else if (li->priority > ri->priority) {
      maybeUpdate(result, resultForLoner(*li));
      ++li;
    } else if (li->priority < ri->priority) {
      maybeUpdate(result, !resultForLoner(*ri));
      ++ri;
    } else {  // same priority, different types
      maybeUpdate(result, CompareResult::ERROR);
    }
  }
  while (!isDecisive(result) && li != l.end()) maybeUpdate(result, resultForLoner(*li++));
  while (!isDecisive(result) && ri != r.end()) maybeUpdate(result, !resultForLoner(*ri++));
  return result;
}

}  // namespace MetricVectorUtils
}  // namespace openr
