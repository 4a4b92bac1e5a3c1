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

namespace {
std::atomic<uint64_t> g_prefixStateUids{0};
}
PrefixState::PrefixState() : uid_(++g_prefixStateUids) {}
PrefixState::PrefixState(const PrefixState& o) : prefixes_(o.prefixes_), uid_(++g_prefixStateUids) {}
PrefixState& PrefixState::operator=(const PrefixState& o) {
  prefixes_ = o.prefixes_;
  ++version_;
  return *this;
}

void PrefixState::updatePrefix(const std::string& node, const std::string& area, const thrift::PrefixEntry& entry) {
  prefixes_[entry.prefix].insert_or_assign({node, area}, entry);
  ++version_;
}

void PrefixState::deletePrefix(const std::string& node, const std::string& area, const thrift::IpPrefix& prefix) {
  auto it = prefixes_.find(prefix);
  if (it == prefixes_.end()) return;
  ++version_;
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
    HostPhase ph("buildRouteDbs: prefetch (one area)");
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
  HostPhase phBuild("buildRouteDbs: per-node builds");
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
    s.bestLazy_.clear();
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
      if (i == last) {
        bestRoutesCache_ = solvers[w].bestRoutesCache_;
        bestLazy_ = solvers[w].bestLazy_;
      }
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

namespace {
// label -> slot of a route build's node-label candidates: open addressing over valid MPLS
// labels (never 0), one allocation per build instead of a hash node per label
class LabelSlots {
 public:
  size_t size() const { return n_; }
  void reserve(size_t n) {
    if (2 * n <= keys_.size()) return;
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    std::vector<int32_t> k(cap, 0);
    std::vector<uint32_t> v(cap, 0);
    const size_t m = cap - 1;
    for (size_t i = 0; i < keys_.size(); ++i)
      if (keys_[i]) {
        size_t h = hash(keys_[i]) & m;
        while (k[h]) h = (h + 1) & m;
        k[h] = keys_[i];
        v[h] = vals_[i];
      }
    keys_.swap(k);
    vals_.swap(v);
  }
  const uint32_t* find(int32_t label) const {
    if (keys_.empty()) return nullptr;
    const size_t m = keys_.size() - 1;
    for (size_t h = hash(label) & m;; h = (h + 1) & m) {
      if (keys_[h] == label) return &vals_[h];
      if (!keys_[h]) return nullptr;
    }
  }
  std::pair<uint32_t*, bool> emplace(int32_t label, uint32_t slot) {
    reserve(n_ + 1);
    const size_t m = keys_.size() - 1;
    size_t h = hash(label) & m;
    for (; keys_[h]; h = (h + 1) & m)
      if (keys_[h] == label) return {&vals_[h], false};
    keys_[h] = label;
    vals_[h] = slot;
    ++n_;
    return {&vals_[h], true};
  }

 private:
  static size_t hash(int32_t label) { return (size_t)((uint32_t)label * 2654435761u); }
  std::vector<int32_t> keys_;
  std::vector<uint32_t> vals_;
  size_t n_ = 0;
};
}  // namespace

// Decision.cpp:568-734
std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(const std::string& myNodeName,
                                                       std::unordered_map<std::string, LinkState> const& als,
                                                       PrefixState const& prefixState) {
  bool nodeExist = false;
  for (auto const& [_, ls] : als) nodeExist |= ls.hasNode(myNodeName);
  if (!nodeExist) return std::nullopt;
  counters_.route_build_runs++;
  // the SPFs this build reads (prefix routes, node-label routes) in one batch; a build with
  // neither reads none, as the reference's (Decision.cpp:589-680), so nothing is solved
  bool readsSpf = !prefixState.prefixes().empty();
  for (auto const& [_, ls] : als) readsSpf |= ls.labeledNodeCount() != 0;
  if (readsSpf) prefetch(myNodeName, als);
  // the views / fast-path context live for this build only (released again below): a
  // LinkState update between two builds moves or frees the rows they point at
  resetViews();
  viewsOf_ = myNodeName;

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
  routeDb.unicastRoutes.reserve(prefixState.prefixes().size());  // at most one route per prefix
  bestRoutesCache_.clear();
  bestLazy_.clear();
  // advertiser ids of the single-advertiser prefixes on the fast path's mirror, computed
  // once per (PrefixState contents, mirror)
  const std::vector<uint32_t>* dstIds = nullptr;
  // (set up only when there is a prefix: it reads my SPF, which counts as a run, as the
  // first createRouteForPrefix would)
  if (!prefixState.prefixes().empty() && fastSetup(als, myNodeName)) {
    auto& c = dstIds_;
    if (c.psUid != prefixState.uid() || c.psVersion != prefixState.version() || c.mirrorGen != fast_.m->generation) {
      c.ids.clear();
      c.ids.reserve(prefixState.prefixes().size());
      for (auto const& [prefix, entries] : prefixState.prefixes()) {
        uint32_t id = UINT32_MAX;
        if (entries.size() == 1) {
          auto it = fast_.m->id.find(entries.begin()->first.first);
          if (it != fast_.m->id.end()) id = it->second;
        }
        c.ids.push_back(id);
      }
      c.psUid = prefixState.uid();
      c.psVersion = prefixState.version();
      c.mirrorGen = fast_.m->generation;
    }
    dstIds = &c.ids;
  }
  size_t pi = 0;
  for (auto const& [prefix, entries] : prefixState.prefixes()) {  // key order
    const uint32_t dstId = dstIds ? (*dstIds)[pi] : UINT32_MAX;
    ++pi;
    if (fast_.state == 1 && fastRoute(myNodeName, prefix, entries, dstId, routeDb.unicastRoutes)) continue;
    auto r = createRouteForPrefix(myNodeName, als, prefixState, prefix, entries, true);
    if (r) routeDb.unicastRoutes.insert_or_assign(routeDb.unicastRoutes.end(), prefix, std::move(*r));
  }

  // MPLS routes for every node label (:593-680). The reference's label -> (node, route) map
  // is kept as label -> slot of `cand` (same visiting order, collisions and counters); the
  // winners then enter the DB in label order.
  LabelSlots labelToNode;
  std::vector<std::pair<const std::string*, RibMplsEntry>> cand;
  auto put = [&](int32_t label, const std::string* node, RibMplsEntry&& entry) {
    auto [slot, fresh] = labelToNode.emplace(label, (uint32_t)cand.size());
    if (fresh) cand.emplace_back(node, std::move(entry));
    else cand[*slot] = std::make_pair(node, std::move(entry));
  };
  for (auto const& [area, ls] : als) {
    if (!ls.labeledNodeCount()) continue;  // every label is 0 (non-SR mode): nothing to visit
    labelToNode.reserve(labelToNode.size() + ls.labeledNodeCount() + 1u);
    // the labelled adjacency databases in getAdjacencyDatabases() order, with mirror ids
    // (the fast path reads my row's mirror: a retired snapshot's ids need the name lookup)
    const auto& labeled = ls.labeledNodes();
    const bool sameMirror = fast_.state == 1 && fast_.m == &ls.csrMirror();
    for (auto const& ln : labeled) {
      const int32_t topLabel = ln.label;
      const std::string& nodeName = *ln.name;
      if (!isMplsLabelValid(topLabel)) {
        counters_.skipped_mpls_route++;
        continue;
      }
      if (const uint32_t* slot = labelToNode.find(topLabel)) {  // collision: the bigger node name keeps the label
        counters_.duplicate_node_label++;
        if (*cand[*slot].first < nodeName) continue;
      }
      if (nodeName == myNodeName) {
        thrift::NextHopThrift nh;
        nh.address.addr = "::";
        nh.area = area;
        nh.mplsAction = createMplsAction(thrift::MplsActionCode::POP_AND_LOOKUP);
        put(topLabel, &nodeName, RibMplsEntry{topLabel, {nh}});
        continue;
      }
      if (fast_.state == 1 && fast_.ls == &ls) {
        NextHopSet fnh;
        uint32_t did = ln.id;
        if (!sameMirror) {
          auto f = fast_.m->id.find(nodeName);
          did = f == fast_.m->id.end() ? UINT32_MAX : f->second;
        }
        const int fr = fastLabelNextHops(myNodeName, did, topLabel, &fnh);
        if (fr == 0) {
          counters_.no_route_to_label++;
          continue;
        }
        if (fr == 1) {
          put(topLabel, &nodeName, RibMplsEntry{topLabel, std::move(fnh)});
          continue;
        }
      }
      auto metricNhs = getNextHopsWithMetric(myNodeName, {{nodeName, area}}, false, als);
      if (metricNhs.second.empty()) {
        counters_.no_route_to_label++;
        continue;
      }
      put(topLabel, &nodeName,
          RibMplsEntry{topLabel, getNextHopsThrift(myNodeName, {{nodeName, area}}, false, false,
                                                   metricNhs.first, metricNhs.second, topLabel, als)});
    }
  }
  // label order through (label, slot) words: the entries move once, into the DB
  std::vector<uint64_t> order(cand.size());
  for (size_t i = 0; i < cand.size(); ++i) order[i] = ((uint64_t)(uint32_t)cand[i].second.label << 32) | i;
  std::sort(order.begin(), order.end());
  routeDb.mplsRoutes.reserve(cand.size() + staticMplsRoutes_.size() + 64u);
  for (const uint64_t o : order) {
    RibMplsEntry& entry = cand[(uint32_t)o].second;
    const int32_t label = entry.label;
    routeDb.mplsRoutes.emplace_hint(routeDb.mplsRoutes.end(), label, std::move(entry));
  }

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
  resetViews();
  return routeDb;
}

void SpfSolver::resetViews() const {
  views_.clear();
  viewsOf_.clear();
  fast_ = FastCtx{};
  ksp2Protos_ = Ksp2Protos{};
}

// Decision.cpp:401-566
std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(const std::string& myNodeName,
                                                               std::unordered_map<std::string, LinkState> const& als,
                                                               PrefixState const& prefixState,
                                                               thrift::IpPrefix const& prefix) {
  auto search = prefixState.prefixes().find(prefix);
  if (search == prefixState.prefixes().end()) {
    counters_.get_route_for_prefix++;
    return std::nullopt;
  }
  return createRouteForPrefix(myNodeName, als, prefixState, prefix, search->second, false);
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(const std::string& myNodeName,
                                                               std::unordered_map<std::string, LinkState> const& als,
                                                               PrefixState const& prefixState, thrift::IpPrefix const& prefix,
                                                               PrefixEntries const& allEntries, bool inOrder) {
  counters_.get_route_for_prefix++;
  // buildRouteDb cleared the cache and visits each prefix once, in key order
  if (!inOrder) {
    flushBestRoutes();
    bestRoutesCache_.erase(prefix);
  }
  // a call outside buildRouteDb (Decision::rebuildRoutes on an incremental prefix update,
  // Decision.cpp:1897-1904) takes fresh views of the current memo and drops them on return:
  // views cached by an earlier build may point at rows a LinkState update has since freed
  struct ViewScope {
    const SpfSolver* s;
    ~ViewScope() {
      if (s) s->resetViews();
    }
  } scope{inOrder ? nullptr : this};
  if (!inOrder) resetViews();

  // entries of reachable nodes only (the reference filters a copy; the entries are used
  // in place when every advertiser is reachable)
  PrefixEntries filteredEntries;
  const PrefixEntries* entries = &allEntries;
  for (auto const& [area, ls] : als) {
    // dense read of the memoised SPF (an unknown node's result holds only itself)
    auto const& mySpf = views(ls, myNodeName).mine;
    for (auto const& [na, e] : *entries) {
      if (area == na.second && !mySpf.reached(na.first)) {
        if (entries != &filteredEntries) {
          filteredEntries = *entries;
          entries = &filteredEntries;
        }
        break;
      }
    }
    if (entries == &filteredEntries)
      for (auto it = filteredEntries.begin(); it != filteredEntries.end();) {
        const auto& [node, pArea] = it->first;
        if (area != pArea || mySpf.reached(node)) ++it;
        else it = filteredEntries.erase(it);
      }
  }
  const PrefixEntries& prefixEntries = *entries;
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
  if (inOrder) bestRoutesCache_.insert_or_assign(bestRoutesCache_.end(), prefix, best);
  else bestRoutesCache_.insert_or_assign(prefix, best);
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
  bool anyDrained = false;
  for (auto const& [node, area] : result.allNodeAreas) anyDrained |= als.at(area).isNodeOverloaded(node);
  if (!anyDrained) return std::move(result);  // nothing to filter: the same result, uncopied
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
  std::set<NodeAndArea> filteredCopy;
  const std::set<NodeAndArea>* filtered = &best.allNodeAreas;
  if (best.hasNode(myNodeName) && perDestination) {
    for (auto const& [na, e] : prefixEntries)
      if (na.first == myNodeName && e.prependLabel) {
        filteredCopy = best.allNodeAreas;
        filteredCopy.erase(na);
        filtered = &filteredCopy;
        break;
      }
  }
  const auto nhm = getNextHopsWithMetric(myNodeName, *filtered, perDestination, als);
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
  // token form (round 5): one area whose LinkState staged every pair this prefix reads
  // (prefetchKthPaths) builds the next hops on its mirror's ids
  if (als.size() == 1) {
    auto const& [area, ls] = *als.begin();
    std::vector<const std::string*> need;
    for (auto const& [node, bestArea] : best.allNodeAreas)
      if (!(node == myNodeName && bestArea == area)) need.push_back(&node);
    if (!need.empty() && ls.kthPathTokensStaged(myNodeName, need)) {
      bool any = false;
      NextHopSet nh = ksp2NextHopsFromTokens(myNodeName, prefix, best, prefixEntries, area, ls, &any);
      if (!any) return std::nullopt;
      return addBestPaths(myNodeName, prefix, best, prefixEntries, prefixState, isBgp, std::move(nh));
    }
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

// selectBestPathsKsp2 (Decision.cpp:907-1030) on token rows: a path is [len, e_1 .. e_len]
// of mirror edge ids from me. pathAInPathB compares link ids (Link equality is identity of
// the (node, interface) pairs, one Link object per pair in a LinkState); the cost sums the
// edges' metrics from their tails (getMetricFromNode); the label stack is the node labels
// of the hops after the first, last hop first, under the advertiser's prepend label.
NextHopSet SpfSolver::ksp2NextHopsFromTokens(const std::string& me, thrift::IpPrefix const& prefix,
                                             BestRouteSelectionResult const& best, PrefixEntries const& prefixEntries,
                                             const std::string& area, const LinkState& ls, bool* any) {
  const LinkState::CsrMirror& m = ls.csrMirror();
  std::vector<const uint32_t*> paths;
  auto addAll = [&](const uint32_t* row) {
    const uint32_t* p = row + 1;
    for (uint32_t i = 0; i < row[0]; ++i, p += 1 + p[0]) paths.push_back(p);
  };
  for (auto const& [node, bestArea] : best.allNodeAreas) {
    if (node == me && bestArea == area) continue;
    addAll(ls.kthPathTokens(me, node, 1));
  }
  const size_t firstPathsSize = paths.size();
  auto inPath = [&](const uint32_t* a, const uint32_t* b) {  // LinkState::pathAInPathB on link ids
    const uint32_t la = a[0], lb = b[0];
    if (la > lb) return false;
    for (uint32_t start = 0; start + la <= lb; ++start) {
      uint32_t k = 0;
      while (k < la && m.linkId[a[1 + k]] == m.linkId[b[1 + start + k]]) ++k;
      if (k == la) return true;
    }
    return false;
  };
  for (auto const& [node, bestArea] : best.allNodeAreas) {
    if (area != bestArea) continue;
    if (node == me) {
      // an anycast prefix this node also advertises: getKthPaths(me, me, 2) is empty in the
      // reference (traceOnePath(me, me) is the empty path, LinkState.cpp:404-406). prefetchKthPaths
      // stages no (me, me) row, so take the general path for its memo and counter effects.
      (void)ls.getKthPaths(me, me, 2);
      continue;
    }
    const uint32_t* row = ls.kthPathTokens(me, node, 2);
    if (!row) throw std::logic_error("ksp2NextHopsFromTokens: (" + me + ", " + node + ") not staged");
    const uint32_t* p = row + 1;
    for (uint32_t i = 0; i < row[0]; ++i, p += 1 + p[0]) {
      bool add = true;
      for (size_t j = 0; j < firstPathsSize && add; ++j) add = !inPath(paths[j], p);
      if (add) paths.push_back(p);
    }
  }
  *any = !paths.empty();
  NextHopSet nextHops;
  if (paths.empty()) return nextHops;
  auto& pr = ksp2Protos_;
  const uint32_t meId = m.id.at(me);
  if (pr.ls != &ls || pr.generation != m.generation || pr.me != meId) {
    pr = Ksp2Protos{};
    pr.ls = &ls;
    pr.generation = m.generation;
    pr.me = meId;
    pr.row0 = m.rowPtr[meId];
    const size_t deg = m.rowPtr[meId + 1] - m.rowPtr[meId];
    pr.p4.resize(deg);
    pr.p6.resize(deg);
    pr.ready.assign(deg, 0);
  }
  const auto& labelOf = ls.nodeLabelsById();
  const bool v4 = prefix.isV4();
  std::vector<int32_t> labels;
  for (const uint32_t* p : paths) {
    const uint32_t len = p[0];
    const uint32_t* e = p + 1;
    Metric cost = 0;
    for (uint32_t j = 0; j < len; ++j) {
      cost += m.metric[e[j]];
      if (labelOf[m.col[e[j]]] == LinkState::kNoNodeLabel)  // getAdjacencyDatabases().at(node)
        throw std::out_of_range("selectBestPathsKsp2: no adjacency database for " + m.names[m.col[e[j]]]);
    }
    const std::string& dst = m.names[m.col[e[len - 1]]];
    auto const& prefixEntry = prefixEntries.at({dst, area});
    labels.clear();
    if (prefixEntry.prependLabel) labels.push_back(*prefixEntry.prependLabel);
    for (uint32_t j = len; j-- > 1;) labels.push_back((int32_t)labelOf[m.col[e[j]]]);  // first hop's label: PHP
    const uint32_t slot = e[0] - pr.row0;
    if (!pr.ready[slot]) {
      auto const& link = m.links[m.linkId[e[0]]];
      const std::string& nbr = link->getOtherNodeName(me);
      pr.p6[slot] = createNextHop(link->getNhV6FromNode(me), link->getIfaceFromNode(me), 0, std::nullopt, link->getArea(), nbr);
      pr.p4[slot] = createNextHop(link->getNhV4FromNode(me), link->getIfaceFromNode(me), 0, std::nullopt, link->getArea(), nbr);
      pr.ready[slot] = 1;
    }
    thrift::NextHopThrift nh = v4 ? pr.p4[slot] : pr.p6[slot];
    nh.metric = static_cast<int32_t>(cost);
    if (!labels.empty()) nh.mplsAction = createMplsAction(thrift::MplsActionCode::PUSH, std::nullopt, labels);
    nextHops.emplace(std::move(nh));
  }
  return nextHops;
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
    // no SpfResult map materialised per route build; views taken once per build
    auto const& fromHere = views(ls, me).mine;
    auto const mm = getMinCostNodes(fromHere, dstNodeAreas);
    if (shortestMetric < mm.first) continue;
    if (shortestMetric > mm.first) {
      shortestMetric = mm.first;
      nextHopNodes.clear();
    }
    if (mm.second.empty()) continue;
    static const std::string kNoDst;
    for (auto const& dst : mm.second) {
      const std::string& dstRef = perDestination ? dst : kNoDst;
      // getMetricFromAToB(me, nh) reads the same (already counted) result: nh != me
      fromHere.forEachNextHop(dst, [&](const std::string& nh, Metric dNh) {
        nextHopNodes[std::make_pair(nh, dstRef)] = shortestMetric - dNh;
      });
    }
    if (computeLfaPaths_) {
      for (auto const& nb : lfaViews(ls, me).nbrs) {  // up links of me, linksFromNode order
        const auto& nbr = *nb.name;
        const Metric nbrToHere = nb.toMe;
        for (auto const& [dst, dstArea] : dstNodeAreas) {
          if (area != dstArea) continue;
          if (!nb.view.reached(dst)) continue;
          const Metric dNbr = nb.view.metric(dst);
          if (dNbr < shortestMetric + nbrToHere) {  // RFC 5286
            auto key = std::make_pair(nbr, perDestination ? dst : kNoDst);
            auto it = nextHopNodes.find(key);
            if (it == nextHopNodes.end()) nextHopNodes.emplace(std::move(key), dNbr);
            else if (it->second > dNbr) it->second = dNbr;
          }
        }
      }
    }
  }
  return {shortestMetric, std::move(nextHopNodes)};
}

bool SpfSolver::fastSetup(std::unordered_map<std::string, LinkState> const& als, const std::string& me) {
  if (fast_.state) return fast_.state == 1;
  fast_.state = 2;
  if (!fastEnabled_ || als.size() != 1 || enableBestRouteSelection_) return false;
  const auto& [area, ls] = *als.begin();
  const auto& mine = views(ls, me).mine;  // read by createRouteForPrefix for every prefix too
  const LinkState::CsrMirror* m = mine.mirror();
  if (!m) return false;
  auto it = m->id.find(me);
  if (it == m->id.end()) return false;
  fast_.ls = &ls;
  fast_.area = &area;
  fast_.m = m;
  fast_.me = it->second;
  const auto& bits = mine.nhNeighbours();
  auto bitOf = [&](uint32_t id) -> uint32_t {
    for (uint32_t i = 0; i < bits.size(); ++i)
      if (bits[i] == id) return i;
    return UINT32_MAX;
  };
  for (auto const& link : ls.linksFromNode(me)) {
    const std::string& nbr = link->getOtherNodeName(me);
    auto nid = m->id.find(nbr);
    if (nid == m->id.end()) return false;
    const uint32_t b = bitOf(nid->second);
    if (b == UINT32_MAX) return false;
    FastLink fl{link.get(), b, link->isUp(), link->getMetricFromNode(me), &nbr, nid->second, {}, {}};
    fl.proto6 = createNextHop(link->getNhV6FromNode(me), link->getIfaceFromNode(me), 0, std::nullopt, link->getArea(), nbr);
    fl.proto4 = createNextHop(link->getNhV4FromNode(me), link->getIfaceFromNode(me), 0, std::nullopt, link->getArea(), nbr);
    fast_.links.push_back(std::move(fl));
  }
  // in NextHopThrift order (address, interface: distinct per link, so the metric never
  // decides), so a v6 route's set is filled at its end
  std::sort(fast_.links.begin(), fast_.links.end(),
            [](const FastLink& a, const FastLink& b) { return a.proto6 < b.proto6; });
  fast_.val.assign(bits.size(), 0);
  fast_.has.assign(bits.size(), 0);
  fast_.state = 1;
  return true;
}

// getNextHopsWithMetric(me, {dst}, perDestination = false) on ids, into fast_.has / val per
// next-hop bit (d = my distance to dst, reached): 1 when there is a next-hop node, 0 when
// there is none, -1 when an LFA neighbour's row is not on my mirror (the general path
// serves the rest of this build)
int SpfSolver::fastNextHopNodes(const std::string& me, uint32_t dst, Metric d) {
  const auto& mine = views_.front().mine;
  const uint32_t nb = mine.nhBytes();
  const uint8_t* hv = mine.nhRow() + (size_t)dst * nb;
  const auto& bits = mine.nhNeighbours();
  bool any = false;
  for (uint32_t i = 0; i < bits.size(); ++i) {
    fast_.has[i] = (hv[i >> 3] >> (i & 7)) & 1u;
    if (fast_.has[i]) {
      fast_.val[i] = d - mine.dist(bits[i]);
      any = true;
    }
  }
  if (computeLfaPaths_) {
    auto& av = lfaViews(*fast_.ls, me);
    if (!fast_.lfaReady) {
      for (auto const& nv : av.nbrs) {
        uint32_t b = UINT32_MAX;
        if (nv.view.mirror() == fast_.m) {
          const uint32_t id = fast_.m->id.at(*nv.name);
          for (uint32_t i = 0; i < bits.size(); ++i)
            if (bits[i] == id) b = i;
        }
        if (b == UINT32_MAX) {  // a neighbour's row on another mirror / map-backed: general path
          fast_.state = 2;
          ++fastFallbacks_;
          return -1;
        }
        fast_.lfaBit.push_back(b);
      }
      fast_.lfaReady = true;
    }
    for (size_t k = 0; k < av.nbrs.size(); ++k) {
      const Metric dn = av.nbrs[k].view.dist(dst);
      if (dn == UINT64_MAX || !(dn < d + av.nbrs[k].toMe)) continue;
      const uint32_t b = fast_.lfaBit[k];
      if (!fast_.has[b]) {
        fast_.has[b] = 1;
        fast_.val[b] = dn;
        any = true;
      } else if (fast_.val[b] > dn) {
        fast_.val[b] = dn;
      }
    }
  }
  return any ? 1 : 0;
}

int SpfSolver::fastLabelNextHops(const std::string& me, uint32_t dst, int32_t label, NextHopSet* out) {
  if (dst == UINT32_MAX) return -1;
  const Metric d = views_.front().mine.dist(dst);
  if (d == UINT64_MAX) return 0;  // getMinCostNodes: dst not reached, no next-hop node
  const int nn = fastNextHopNodes(me, dst, d);
  if (nn <= 0) return nn;
  auto takes = [&](const FastLink& fl) {
    return fast_.has[fl.nbrBit] && fl.up && (computeLfaPaths_ || fl.metric + fast_.val[fl.nbrBit] == d);
  };
  size_t want = 0;
  for (auto const& fl : fast_.links) want += takes(fl) ? 1u : 0u;
  out->reserve(want);  // one allocation per label route
  for (auto const& fl : fast_.links) {  // getNextHopsThrift, in NextHopThrift order
    if (!takes(fl)) continue;
    const Metric over = fl.metric + fast_.val[fl.nbrBit];
    thrift::NextHopThrift nh = fl.proto6;
    nh.metric = static_cast<int32_t>(over);
    const bool php = fl.nbrId == dst;  // the next hop is the label's node
    nh.mplsAction = createMplsAction(php ? thrift::MplsActionCode::PHP : thrift::MplsActionCode::SWAP,
                                     php ? std::nullopt : std::optional<int32_t>(label));
    out->emplace_hint(out->end(), std::move(nh));
  }
  return 1;
}

bool SpfSolver::fastRoute(const std::string& me, thrift::IpPrefix const& prefix, PrefixEntries const& entries,
                          uint32_t dstId, UnicastRoutes& routes) {
  if (entries.size() != 1) return false;
  const auto& [na, e] = *entries.begin();
  if (na.second != *fast_.area || e.type == thrift::PrefixType::BGP ||
      e.forwardingAlgorithm != thrift::PrefixForwardingAlgorithm::SP_ECMP || e.forwardingType != thrift::PrefixForwardingType::IP)
    return false;
  const auto& mine = views_.front().mine;  // fastSetup: views_ holds this one area
  counters_.get_route_for_prefix++;
  const Metric d = dstId == UINT32_MAX ? UINT64_MAX : mine.dist(dstId);
  if (d == UINT64_MAX) {  // advertiser not reached: entry filtered out
    counters_.no_route_to_prefix++;
    return true;
  }
  const uint32_t dst = dstId;
  if (prefix.isV4() && !enableV4_) {
    counters_.skipped_unicast_route++;
    return true;
  }
  // selectBestRoutes: the single advertiser (maybeFilterDrainedNodes keeps a lone drained one)
  bestLazy_.emplace_back(prefix, na);  // the best-route cache entry {success, {na}, na}
  if (dst == fast_.me) {  // self-originated; with a prepend label no next hop leads to it
    if (e.prependLabel) counters_.no_route_to_prefix++;
    return true;
  }
  // getNextHopsWithMetric(me, {dst}, false): shortest next hops, then RFC 5286 alternates
  const int nn = fastNextHopNodes(me, dst, d);
  if (nn < 0) {  // the general path serves this prefix: undo what it will count again
    counters_.get_route_for_prefix--;
    bestLazy_.pop_back();
    return false;
  }
  if (nn == 0) {
    counters_.no_route_to_prefix++;
    return true;
  }
  // getNextHopsThrift(me, {dst}, isV4, false, d, ...): every up link to a next-hop node
  NextHopSet nextHops;
  const bool v4 = prefix.isV4();
  auto takes = [&](const FastLink& fl) {
    return fast_.has[fl.nbrBit] && fl.up && (computeLfaPaths_ || fl.metric + fast_.val[fl.nbrBit] == d);
  };
  size_t want = 0;
  for (auto const& fl : fast_.links) want += takes(fl) ? 1u : 0u;
  nextHops.reserve(want);  // one allocation per route
  for (auto const& fl : fast_.links) {
    if (!takes(fl)) continue;
    const Metric over = fl.metric + fast_.val[fl.nbrBit];
    thrift::NextHopThrift nh = v4 ? fl.proto4 : fl.proto6;
    nh.metric = static_cast<int32_t>(over);
    nextHops.emplace_hint(nextHops.end(), std::move(nh));
  }
  // addBestPaths
  if (e.minNexthop && *e.minNexthop > (int64_t)nextHops.size()) return true;
  auto it = routes.emplace_hint(routes.end(), std::piecewise_construct, std::forward_as_tuple(prefix),
                                std::forward_as_tuple());
  RibUnicastEntry& r = it->second;
  r.prefix = prefix;
  r.nexthops = std::move(nextHops);
  r.bestPrefixEntry = e;
  r.bestArea = na.second;
  r.doNotInstall = false;  // not BGP
  return true;
}

void SpfSolver::flushBestRoutes() const {
  for (auto& [prefix, na] : bestLazy_) {
    BestRouteSelectionResult best;
    best.allNodeAreas.emplace(na);
    best.bestNodeArea = na;
    best.success = true;
    bestRoutesCache_.insert_or_assign(std::move(prefix), std::move(best));
  }
  bestLazy_.clear();
}

std::map<thrift::IpPrefix, BestRouteSelectionResult> const& SpfSolver::getBestRoutesCache() const {
  flushBestRoutes();
  return bestRoutesCache_;
}

SpfSolver::AreaViews& SpfSolver::views(const LinkState& ls, const std::string& me) const {
  if (viewsOf_ != me) {  // a caller outside buildRouteDb (or another node): start over
    views_.clear();
    viewsOf_ = me;
  }
  for (auto& av : views_)
    if (av.ls == &ls) return av;
  AreaViews av;
  av.ls = &ls;
  av.mine = ls.getSpfView(me);
  views_.push_back(std::move(av));
  return views_.back();
}

SpfSolver::AreaViews& SpfSolver::lfaViews(const LinkState& ls, const std::string& me) const {
  AreaViews& av = views(ls, me);
  if (!av.nbrsReady) {
    for (auto const& link : ls.linksFromNode(me)) {
      if (!link->isUp()) continue;
      const auto& nbr = link->getOtherNodeName(me);
      NbrView nv{&nbr, ls.getSpfView(nbr), 0};
      nv.toMe = nv.view.metric(me);
      av.nbrs.push_back(std::move(nv));
    }
    av.nbrsReady = true;
  }
  return av;
}

// Decision.cpp:1210-1317
NextHopSet SpfSolver::getNextHopsThrift(const std::string& me, const std::set<NodeAndArea>& dstNodeAreas, bool isV4,
                                        bool perDestination, Metric minMetric,
                                        std::unordered_map<std::pair<std::string, std::string>, Metric> const& nextHopNodes,
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

std::vector<thrift::IpPrefix> RibPolicy::applyPolicy(UnicastRoutes& entries) const {
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
