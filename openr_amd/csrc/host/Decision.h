// Decision.h — host mirror of openr::SpfSolver (route build) and openr::RibPolicy.
//
// Reference: /root/reference/openr/decision/Decision.{h,cpp} (SpfSolver::SpfSolverImpl,
// :401-1317), RibEntry.h, RibPolicy.{h,cpp}, common/Util.{h,cpp} (route helpers).
// Same names, argument meaning and results for the SP_ECMP and KSP2_ED_ECMP algorithms
// with IP and SR_MPLS forwarding, LFA, node- and adjacency-label MPLS routes, static
// MPLS routes, min-nexthop and best-route selection by PrefixMetrics.
//
// What changes is where the SPF results come from: every getSpfResult here is served by
// the engine (LinkState.cpp over the C-ABI), and buildRouteDb first prefetches the SPFs
// it will read — this node plus, with LFA, every up neighbour — in ONE batched device
// launch (LinkState::prefetchSpfResults) instead of one Dijkstra per call.
// buildRouteDbs() does the same for a list of nodes (the getRouteMap /
// GridTopologyFixture workload: all nodes' route DBs from one all-sources batch).
//
// Not mirrored: BGP metric-vector best path selection (runBestPathSelectionBgp; a BGP
// prefix without enableBestRouteSelection is skipped with an error counter), ordered-FIB
// hold timers (Decision event plumbing), thrift serialization.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <map>
#include <optional>
#include <stdexcept>
#include <tuple>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "LinkState.h"

namespace openr {

using Metric = LinkStateMetric;
using NodeAndArea = std::pair<std::string, std::string>;

namespace thrift {

enum class PrefixType : int32_t { LOOPBACK = 1, DEFAULT = 2, BGP = 3, PREFIX_ALLOCATOR = 4, BREEZE = 5, RIB = 6 };
enum class PrefixForwardingType : int32_t { IP = 0, SR_MPLS = 1 };
enum class PrefixForwardingAlgorithm : int32_t { SP_ECMP = 0, KSP2_ED_ECMP = 1 };
enum class MplsActionCode : int32_t { PUSH = 0, SWAP = 1, PHP = 2, POP_AND_LOOKUP = 3, NOOP = 4 };

// Network.thrift IpPrefix: `addr` is the textual address ("10.0.0.1", "fc00::1");
// an address with a '.' and no ':' is IPv4 (the reference tests the binary size).
struct IpPrefix {
  std::string addr;
  int16_t prefixLength = 0;
  bool isV4() const { return addr.find(':') == std::string::npos; }
  bool operator<(const IpPrefix& o) const { return std::tie(addr, prefixLength) < std::tie(o.addr, o.prefixLength); }
  bool operator==(const IpPrefix& o) const { return addr == o.addr && prefixLength == o.prefixLength; }
  std::string toString() const { return addr + "/" + std::to_string(prefixLength); }
};

// Lsdb.thrift:165-213 (deprecated BGP metric vectors, still honoured by the route build)
enum class CompareType : int32_t { WIN_IF_PRESENT = 1, WIN_IF_NOT_PRESENT = 2, IGNORE_IF_NOT_PRESENT = 3 };
struct MetricEntity {
  int64_t type = 0;
  int64_t priority = 0;
  CompareType op = CompareType::WIN_IF_PRESENT;
  bool isBestPathTieBreaker = false;
  std::vector<int64_t> metric;
};
struct MetricVector {
  int64_t version = 0;
  std::vector<MetricEntity> metrics;  // expected sorted by decreasing priority
};

struct PrefixMetrics {  // Lsdb.thrift:228 (defaults 1, 0, 0, 0)
  int32_t version = 1;
  int32_t path_preference = 0;
  int32_t source_preference = 0;
  int32_t distance = 0;
};

struct PrefixEntry {  // Lsdb.thrift:269
  IpPrefix prefix;
  PrefixType type = PrefixType::LOOPBACK;
  PrefixForwardingType forwardingType = PrefixForwardingType::IP;
  PrefixForwardingAlgorithm forwardingAlgorithm = PrefixForwardingAlgorithm::SP_ECMP;
  std::string data;                // opaque payload (BGP routes carry it to the RIB)
  std::optional<MetricVector> mv;  // deprecated BGP metric vector
  std::optional<int64_t> minNexthop;
  std::optional<int32_t> prependLabel;
  PrefixMetrics metrics;
};

struct MplsAction {  // Network.thrift MplsAction
  MplsActionCode action = MplsActionCode::NOOP;
  std::optional<int32_t> swapLabel;
  std::optional<std::vector<int32_t>> pushLabels;
  bool operator<(const MplsAction& o) const {
    return std::tie(action, swapLabel, pushLabels) < std::tie(o.action, o.swapLabel, o.pushLabels);
  }
  bool operator==(const MplsAction& o) const {
    return action == o.action && swapLabel == o.swapLabel && pushLabels == o.pushLabels;
  }
};

struct NextHopThrift {  // Network.thrift NextHopThrift
  BinaryAddress address;
  int32_t weight = 0;
  std::optional<MplsAction> mplsAction;
  int32_t metric = 0;
  std::optional<std::string> area;
  std::optional<std::string> neighborNodeName;
  bool operator<(const NextHopThrift& o) const {
    return std::tie(address.addr, address.ifName, weight, mplsAction, metric, area, neighborNodeName) <
           std::tie(o.address.addr, o.address.ifName, o.weight, o.mplsAction, o.metric, o.area, o.neighborNodeName);
  }
  bool operator==(const NextHopThrift& o) const { return !(*this < o) && !(o < *this); }
};

}  // namespace thrift

// Set semantics of the reference's unordered_set<NextHopThrift>, ordered for tests.
// Util.h:505-540 MetricVectorUtils (metric vector comparison for BGP best paths)
namespace MetricVectorUtils {
enum class CompareResult { WINNER, TIE_WINNER, TIE, TIE_LOOSER, LOOSER, ERROR };
CompareResult operator!(CompareResult r);
bool isDecisive(CompareResult r);
bool isSorted(thrift::MetricVector const& mv);
void sortMetricVector(thrift::MetricVector const& mv);  // in place, as the reference
CompareResult compareMetrics(std::vector<int64_t> const& l, std::vector<int64_t> const& r, bool tieBreaker);
CompareResult resultForLoner(thrift::MetricEntity const& e);
void maybeUpdate(CompareResult& target, CompareResult update);
CompareResult compareMetricVectors(thrift::MetricVector const& l, thrift::MetricVector const& r);
}  // namespace MetricVectorUtils

// The reference's unordered_set<NextHopThrift> as a sorted vector: set semantics, iteration
// in NextHopThrift order (deterministic for tests), and one allocation per route instead
// of one tree node per next hop (the all-node route build allocates ~200 M next hops).
// Iterators are const, as a set's; an insert or erase invalidates them, as a vector's.
class NextHopSet {
 public:
  using value_type = thrift::NextHopThrift;
  using key_type = thrift::NextHopThrift;
  using const_iterator = std::vector<value_type>::const_iterator;
  using iterator = const_iterator;
  using size_type = size_t;
  using reference = const value_type&;
  using const_reference = const value_type&;

  NextHopSet() = default;
  NextHopSet(std::initializer_list<value_type> il) {
    v_.reserve(il.size());
    for (auto const& x : il) insert(x);
  }
  template <class It>
  NextHopSet(It b, It e) {
    insert(b, e);
  }
  const_iterator begin() const { return v_.begin(); }
  const_iterator end() const { return v_.end(); }
  const_iterator cbegin() const { return v_.begin(); }
  const_iterator cend() const { return v_.end(); }
  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  void clear() { v_.clear(); }
  void reserve(size_t n) { v_.reserve(n); }

  std::pair<iterator, bool> insert(const value_type& x) { return put(value_type(x)); }
  std::pair<iterator, bool> insert(value_type&& x) { return put(std::move(x)); }
  iterator insert(const_iterator hint, const value_type& x) { return putHint(hint, value_type(x)); }
  iterator insert(const_iterator hint, value_type&& x) { return putHint(hint, std::move(x)); }
  template <class It>
  void insert(It b, It e) {
    for (; b != e; ++b) insert(*b);
  }
  template <class... A>
  std::pair<iterator, bool> emplace(A&&... a) {
    return put(value_type(std::forward<A>(a)...));
  }
  template <class... A>
  iterator emplace_hint(const_iterator hint, A&&... a) {
    return putHint(hint, value_type(std::forward<A>(a)...));
  }
  iterator find(const value_type& x) const {
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    return it != v_.end() && !(x < *it) ? it : v_.end();
  }
  size_t count(const value_type& x) const { return find(x) != end() ? 1u : 0u; }
  bool contains(const value_type& x) const { return find(x) != end(); }
  iterator erase(const_iterator it) { return v_.erase(it); }
  size_t erase(const value_type& x) {
    auto it = find(x);
    if (it == end()) return 0;
    v_.erase(it);
    return 1;
  }
  bool operator==(const NextHopSet& o) const { return v_ == o.v_; }
  bool operator!=(const NextHopSet& o) const { return !(v_ == o.v_); }
  bool operator<(const NextHopSet& o) const { return v_ < o.v_; }

 private:
  std::pair<iterator, bool> put(value_type&& x) {
    if (v_.empty() || v_.back() < x) {  // in order (the route builds insert sorted)
      v_.push_back(std::move(x));
      return {v_.end() - 1, true};
    }
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    if (it != v_.end() && !(x < *it)) return {it, false};
    const auto at = it - v_.begin();
    v_.insert(it, std::move(x));
    return {v_.begin() + at, true};
  }
  iterator putHint(const_iterator, value_type&& x) { return put(std::move(x)).first; }
  std::vector<value_type> v_;
};
using PrefixEntries = std::unordered_map<NodeAndArea, thrift::PrefixEntry>;

struct RibUnicastEntry {  // RibEntry.h:37
  thrift::IpPrefix prefix;
  NextHopSet nexthops;
  thrift::PrefixEntry bestPrefixEntry;
  std::string bestArea;
  bool doNotInstall = false;
};

struct RibMplsEntry {  // RibEntry.h:92
  int32_t label = 0;
  NextHopSet nexthops;
};

// The reference's route maps (Decision.h:80: unordered_map<CIDRNetwork, RibUnicastEntry>,
// unordered_map<int32_t, RibMplsEntry>) as sorted vectors of (key, value): map lookups,
// iteration in key order (deterministic for tests), and no per-route node allocation. A
// route build inserts in key order (an append); an insert elsewhere shifts the tail, and
// like a vector's it invalidates iterators and references.
template <class K, class V>
class FlatMap {
 public:
  using key_type = K;
  using mapped_type = V;
  using value_type = std::pair<K, V>;
  using iterator = typename std::vector<value_type>::iterator;
  using const_iterator = typename std::vector<value_type>::const_iterator;
  using size_type = size_t;

  FlatMap() = default;
  FlatMap(std::initializer_list<value_type> il) {
    for (auto const& x : il) insert_or_assign(x.first, x.second);
  }
  iterator begin() { return v_.begin(); }
  iterator end() { return v_.end(); }
  const_iterator begin() const { return v_.begin(); }
  const_iterator end() const { return v_.end(); }
  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  void clear() { v_.clear(); }
  void reserve(size_t n) { v_.reserve(n); }

  iterator find(const K& k) {
    auto it = lower(k);
    return it != v_.end() && !(k < it->first) ? it : v_.end();
  }
  const_iterator find(const K& k) const { return const_cast<FlatMap*>(this)->find(k); }
  size_t count(const K& k) const { return find(k) != end() ? 1u : 0u; }
  bool contains(const K& k) const { return find(k) != end(); }
  V& at(const K& k) {
    auto it = find(k);
    if (it == v_.end()) throw std::out_of_range("FlatMap::at");
    return it->second;
  }
  const V& at(const K& k) const { return const_cast<FlatMap*>(this)->at(k); }
  V& operator[](const K& k) { return emplace(std::piecewise_construct, std::forward_as_tuple(k), std::forward_as_tuple()).first->second; }

  template <class M>
  std::pair<iterator, bool> insert_or_assign(const K& k, M&& m) {
    if (v_.empty() || v_.back().first < k) {  // in key order: an append
      v_.emplace_back(k, std::forward<M>(m));
      return {v_.end() - 1, true};
    }
    auto it = lower(k);
    if (it != v_.end() && !(k < it->first)) {
      it->second = std::forward<M>(m);
      return {it, false};
    }
    const auto at = it - v_.begin();
    v_.emplace(it, k, std::forward<M>(m));
    return {v_.begin() + at, true};
  }
  template <class M>
  iterator insert_or_assign(const_iterator, const K& k, M&& m) {
    return insert_or_assign(k, std::forward<M>(m)).first;
  }
  std::pair<iterator, bool> insert(value_type x) { return put(std::move(x)); }
  template <class... A>
  std::pair<iterator, bool> emplace(A&&... a) {
    return put(value_type(std::forward<A>(a)...));
  }
  template <class... A>
  iterator emplace_hint(const_iterator, A&&... a) {
    return put(value_type(std::forward<A>(a)...)).first;
  }
  iterator erase(const_iterator it) { return v_.erase(it); }
  size_t erase(const K& k) {
    auto it = find(k);
    if (it == v_.end()) return 0;
    v_.erase(it);
    return 1;
  }
  bool operator==(const FlatMap& o) const { return v_ == o.v_; }
  bool operator!=(const FlatMap& o) const { return !(v_ == o.v_); }

 private:
  iterator lower(const K& k) {
    return std::lower_bound(v_.begin(), v_.end(), k, [](const value_type& a, const K& b) { return a.first < b; });
  }
  // inserts x unless its key is present; returns (the key's element, inserted)
  std::pair<iterator, bool> put(value_type&& x) {
    if (v_.empty() || v_.back().first < x.first) {  // in key order: an append
      v_.push_back(std::move(x));
      return {v_.end() - 1, true};
    }
    auto it = lower(x.first);
    if (it != v_.end() && !(x.first < it->first)) return {it, false};
    const auto at = it - v_.begin();
    v_.insert(it, std::move(x));
    return {v_.begin() + at, true};
  }
  std::vector<value_type> v_;
};
using UnicastRoutes = FlatMap<thrift::IpPrefix, RibUnicastEntry>;
using MplsRoutes = FlatMap<int32_t, RibMplsEntry>;

struct DecisionRouteDb {  // Decision.h:80
  UnicastRoutes unicastRoutes;
  MplsRoutes mplsRoutes;
  void addUnicastRoute(RibUnicastEntry&& e) { unicastRoutes.insert_or_assign(e.prefix, std::move(e)); }
  void addMplsRoute(RibMplsEntry&& e) { mplsRoutes.insert_or_assign(e.label, std::move(e)); }
};

// PrefixState (decision/PrefixState.h): prefix -> (node, area) -> PrefixEntry.
class PrefixState {
 public:
  using Entries = std::map<thrift::IpPrefix, PrefixEntries>;
  PrefixState();
  PrefixState(const PrefixState& o);
  PrefixState& operator=(const PrefixState& o);
  void updatePrefix(const std::string& node, const std::string& area, const thrift::PrefixEntry& entry);
  void deletePrefix(const std::string& node, const std::string& area, const thrift::IpPrefix& prefix);
  Entries const& prefixes() const { return prefixes_; }
  // (uid, version) names this object's current contents: a process-wide id per object
  // and a count of its mutations (route builds key per-prefix caches on it)
  uint64_t uid() const { return uid_; }
  uint64_t version() const { return version_; }

 private:
  Entries prefixes_;
  uint64_t uid_ = 0, version_ = 0;
};

struct BestRouteSelectionResult {  // Decision.h
  bool success = false;
  std::set<NodeAndArea> allNodeAreas;
  NodeAndArea bestNodeArea;
  bool hasNode(const std::string& node) const {
    for (auto const& na : allNodeAreas)
      if (na.first == node) return true;
    return false;
  }
};

struct DecisionCounters {  // fb303 decision.* counters the route build bumps
  uint64_t route_build_runs = 0, get_route_for_prefix = 0, no_route_to_prefix = 0, skipped_unicast_route = 0,
           skipped_mpls_route = 0, duplicate_node_label = 0, no_route_to_label = 0,
           incompatible_forwarding_type = 0;
};

// Util.h helpers
bool isMplsLabelValid(int32_t mplsLabel);
thrift::NextHopThrift createNextHop(thrift::BinaryAddress addr, std::optional<std::string> ifName, int32_t metric,
                                    std::optional<thrift::MplsAction> mplsAction,
                                    const std::optional<std::string>& area = std::nullopt,
                                    const std::optional<std::string>& neighborNodeName = std::nullopt);
thrift::MplsAction createMplsAction(thrift::MplsActionCode code, std::optional<int32_t> swapLabel = std::nullopt,
                                    std::optional<std::vector<int32_t>> pushLabels = std::nullopt);
std::set<NodeAndArea> selectBestPrefixMetrics(PrefixEntries const& prefixes);
NodeAndArea selectBestNodeArea(std::set<NodeAndArea> const& allNodeAreas, std::string const& myNodeName);
std::pair<thrift::PrefixForwardingType, thrift::PrefixForwardingAlgorithm> getPrefixForwardingTypeAndAlgorithm(
    const PrefixEntries& prefixEntries, const std::set<NodeAndArea>& bestNodeAreas);

class SpfSolver {
 public:
  SpfSolver(const std::string& myNodeName, bool enableV4, bool computeLfaPaths, bool enableOrderedFib = false,
            bool bgpDryRun = false, bool enableBestRouteSelection = false);

  // tests: off = every route through the general createRouteForPrefix / label path (the
  // id-based fast path must build the same DBs)
  void setFastPathForTesting(bool on) { fastEnabled_ = on; }
  // builds whose fast path handed the rest of the build to the general path (an LFA
  // neighbour's row on another mirror)
  uint64_t fastFallbacksForTesting() const { return fastFallbacks_; }

  // static MPLS routes (updateStaticRoutes): label -> next-hops
  void updateStaticMplsRoutes(const std::unordered_map<int32_t, std::vector<thrift::NextHopThrift>>& add,
                              const std::vector<int32_t>& del);

  std::optional<DecisionRouteDb> buildRouteDb(const std::string& myNodeName,
                                              std::unordered_map<std::string, LinkState> const& areaLinkStates,
                                              PrefixState const& prefixState);

  // Batched: the route DBs of many nodes (getRouteMap), after one all-sources prefetch
  // per area. Entry i is buildRouteDb(nodes[i], ...).
  std::vector<std::optional<DecisionRouteDb>> buildRouteDbs(
      const std::vector<std::string>& nodes, std::unordered_map<std::string, LinkState> const& areaLinkStates,
      PrefixState const& prefixState);

  // Streaming form: sink(i, db) runs on the host worker that built entry i (entries in no
  // particular order; HostParallel.h) and the DB is destroyed there when the sink returns,
  // so a consumer that applies policy or programs routes per node touches each DB while
  // it is cache-hot and frees it into the allocating thread's arena.
  void buildRouteDbs(const std::vector<std::string>& nodes,
                     std::unordered_map<std::string, LinkState> const& areaLinkStates, PrefixState const& prefixState,
                     const std::function<void(size_t, std::optional<DecisionRouteDb>&)>& sink);

  // (buildRouteDb walks prefixState.prefixes() in key order and hands each entry set in:
  // no second lookup, and the best-route cache and route map grow at their ends)
  std::optional<RibUnicastEntry> createRouteForPrefix(const std::string& myNodeName,
                                                      std::unordered_map<std::string, LinkState> const& areaLinkStates,
                                                      PrefixState const& prefixState, thrift::IpPrefix const& prefix,
                                                      PrefixEntries const& entries, bool inOrder);
  std::optional<RibUnicastEntry> createRouteForPrefix(const std::string& myNodeName,
                                                      std::unordered_map<std::string, LinkState> const& areaLinkStates,
                                                      PrefixState const& prefixState, thrift::IpPrefix const& prefix);

  std::map<thrift::IpPrefix, BestRouteSelectionResult> const& getBestRoutesCache() const;
  DecisionCounters const& counters() const { return counters_; }

 private:
  BestRouteSelectionResult selectBestRoutes(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                            PrefixEntries const& prefixEntries, bool isBgp,
                                            std::unordered_map<std::string, LinkState> const& areaLinkStates);
  BestRouteSelectionResult runBestPathSelectionBgp(thrift::IpPrefix const& prefix, PrefixEntries const& prefixEntries,
                                                   std::unordered_map<std::string, LinkState> const& areaLinkStates);
  BestRouteSelectionResult maybeFilterDrainedNodes(
      BestRouteSelectionResult&& result, std::unordered_map<std::string, LinkState> const& areaLinkStates) const;
  std::optional<int64_t> getMinNextHopThreshold(BestRouteSelectionResult const& nodes,
                                                PrefixEntries const& prefixEntries) const;
  std::optional<RibUnicastEntry> selectBestPathsSpf(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                                    BestRouteSelectionResult const& best,
                                                    PrefixEntries const& prefixEntries, bool isBgp,
                                                    thrift::PrefixForwardingType forwardingType,
                                                    std::unordered_map<std::string, LinkState> const& areaLinkStates,
                                                    PrefixState const& prefixState);
  std::optional<RibUnicastEntry> selectBestPathsKsp2(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                                     BestRouteSelectionResult const& best,
                                                     PrefixEntries const& prefixEntries, bool isBgp,
                                                     thrift::PrefixForwardingType forwardingType,
                                                     std::unordered_map<std::string, LinkState> const& areaLinkStates,
                                                     PrefixState const& prefixState);
  std::optional<RibUnicastEntry> addBestPaths(std::string const& myNodeName, thrift::IpPrefix const& prefix,
                                              BestRouteSelectionResult const& best, PrefixEntries const& prefixEntries,
                                              PrefixState const& prefixState, bool isBgp, NextHopSet&& nextHops);
  std::pair<Metric, std::unordered_set<std::string>> getMinCostNodes(
      const LinkState::SpfView& spf, const std::set<NodeAndArea>& dstNodeAreas) const;
  std::pair<Metric, std::unordered_map<std::pair<std::string, std::string>, Metric>> getNextHopsWithMetric(
      const std::string& myNodeName, const std::set<NodeAndArea>& dstNodeAreas, bool perDestination,
      std::unordered_map<std::string, LinkState> const& areaLinkStates) const;
  NextHopSet getNextHopsThrift(const std::string& myNodeName, const std::set<NodeAndArea>& dstNodeAreas, bool isV4,
                               bool perDestination, Metric minMetric,
                               std::unordered_map<std::pair<std::string, std::string>, Metric> const& nextHopNodes,
                               std::optional<int32_t> swapLabel,
                               std::unordered_map<std::string, LinkState> const& areaLinkStates,
                               PrefixEntries const& prefixEntries = {});
  void prefetch(const std::string& myNodeName, std::unordered_map<std::string, LinkState> const& areaLinkStates) const;

  // Per route build: the memoised SPF views a build of `me` reads, taken from the
  // LinkState once per build instead of once per prefix (the first read of each still
  // counts its SPF run where the reference's first getSpfResult would). Cleared by
  // buildRouteDb; filled lazily, so a build reads exactly the SPFs the reference does.
  struct NbrView {
    const std::string* name;  // the Link's copy of the neighbour name
    LinkState::SpfView view;
    Metric toMe;              // neighbour -> me (getMetricFromAToB)
  };
  struct AreaViews {
    const LinkState* ls = nullptr;
    LinkState::SpfView mine;
    bool nbrsReady = false;
    std::vector<NbrView> nbrs;  // LFA: up links of me, linksFromNode order
  };
  mutable std::string viewsOf_;
  mutable std::vector<AreaViews> views_;
  void resetViews() const;  // drop views_ and fast_ (they point into the LinkState memo)

  // SP_ECMP / IP fast path of buildRouteDb (one area, dense memo rows from one mirror): the
  // route of a prefix with a single advertiser computed on node ids — the same
  // RibUnicastEntry, counters and best-route cache entry as createRouteForPrefix, without
  // name lookups per route. fast_.state: 0 not set up, 1 usable, 2 not usable (general path).
  struct FastLink {
    const Link* link;
    uint32_t nbrBit;  // the neighbour's next-hop bit in my row
    bool up;
    Metric metric;    // from me
    const std::string* nbr;
    uint32_t nbrId;   // the neighbour's node id on the mirror
    // getNextHopsThrift's NextHopThrift over this link (v6 / v4 next-hop address), metric 0:
    // a route copies it and sets the metric
    thrift::NextHopThrift proto6, proto4;
  };
  struct FastCtx {
    int state = 0;
    const LinkState* ls = nullptr;
    const std::string* area = nullptr;
    const LinkState::CsrMirror* m = nullptr;
    uint32_t me = 0;
    std::vector<FastLink> links;
    bool lfaReady = false;
    std::vector<uint32_t> lfaBit;  // per lfaViews(ls, me).nbrs entry: its neighbour's next-hop bit
    std::vector<Metric> val;       // per next-hop bit: nextHopNodes value
    std::vector<uint8_t> has;
  };
  mutable FastCtx fast_;
  bool fastSetup(std::unordered_map<std::string, LinkState> const& areaLinkStates, const std::string& me);
  bool fastEnabled_ = true;
  uint64_t fastFallbacks_ = 0;
  int fastNextHopNodes(const std::string& me, uint32_t dst, Metric d);
  // the node-label MPLS route's next hops towards dst (getNextHopsWithMetric +
  // getNextHopsThrift with swapLabel = label, perDestination = false): 1 = *out built, 0 =
  // no next-hop node (no route to the label), -1 = not on the fast path (general path)
  int fastLabelNextHops(const std::string& me, uint32_t dst, int32_t label, NextHopSet* out);
  // true when the prefix was served: its route, if any, is appended to `routes` (prefixes
  // arrive in key order, so the route is built in place at the end)
  bool fastRoute(const std::string& me, thrift::IpPrefix const& prefix, PrefixEntries const& entries, uint32_t dstId,
                 UnicastRoutes& routes);
  // selectBestPathsKsp2 on the staged token rows of one area (LinkState::kthPathTokens):
  // the same paths, pathAInPathB filter, label stacks, costs and next hops, on ids
  NextHopSet ksp2NextHopsFromTokens(const std::string& me, thrift::IpPrefix const& prefix,
                                    BestRouteSelectionResult const& best, PrefixEntries const& prefixEntries,
                                    const std::string& area, const LinkState& ls, bool* any);
  struct Ksp2Protos {  // per build: my links' next-hop fields by position in my mirror row
    const LinkState* ls = nullptr;
    uint64_t generation = 0;
    uint32_t me = UINT32_MAX, row0 = 0;
    std::vector<thrift::NextHopThrift> p4, p6;
    std::vector<uint8_t> ready;
  };
  mutable Ksp2Protos ksp2Protos_;
  AreaViews& views(const LinkState& ls, const std::string& me) const;
  AreaViews& lfaViews(const LinkState& ls, const std::string& me) const;

  const std::string myNodeName_;
  const bool enableV4_, computeLfaPaths_, enableOrderedFib_, bgpDryRun_, enableBestRouteSelection_;
  std::unordered_map<int32_t, std::vector<thrift::NextHopThrift>> staticMplsRoutes_;
  mutable std::map<thrift::IpPrefix, BestRouteSelectionResult> bestRoutesCache_;
  // best-route cache entries of single-advertiser routes built on the fast path, merged
  // into bestRoutesCache_ when it is read (flushBestRoutes)
  mutable std::vector<std::pair<thrift::IpPrefix, NodeAndArea>> bestLazy_;
  void flushBestRoutes() const;
  // advertiser node ids of a PrefixState's single-advertiser prefixes, in key order, on
  // one mirror (UINT32_MAX: several advertisers / unknown node)
  struct DstIds {
    uint64_t psUid = 0, psVersion = 0, mirrorGen = 0;
    std::vector<uint32_t> ids;
  };
  DstIds dstIds_;
  DecisionCounters counters_;
};

// RibPolicy (RibPolicy.{h,cpp}): statements matching prefixes; action set_weight with
// neighbor > area > default precedence; weight 0 drops a next-hop; a route whose every
// next-hop would be dropped is kept unchanged.
struct RibPolicyStatement {
  std::string name;
  std::set<thrift::IpPrefix> prefixes;  // matcher.prefixes (required)
  int32_t defaultWeight = 0;            // action.set_weight
  std::unordered_map<std::string, int32_t> areaToWeight, neighborToWeight;
  bool match(const RibUnicastEntry& route) const { return prefixes.count(route.prefix) > 0; }
  bool applyAction(RibUnicastEntry& route) const;
};

// fb303 decision.rib_policy.* counters (process-wide, like fb303::fbData)
struct RibPolicyCounters {
  static RibPolicyCounters& get();
  std::atomic<uint64_t> invalidatedRoutes{0};  // decision.rib_policy.invalidated_routes (RibPolicy.cpp:98-104)
};

class RibPolicy {
 public:
  explicit RibPolicy(std::vector<RibPolicyStatement> statements, int64_t ttlSecs = 3600);
  bool isActive() const;
  bool applyAction(RibUnicastEntry& route) const;  // first matching statement wins
  // prefixes of the routes the policy transformed
  std::vector<thrift::IpPrefix> applyPolicy(UnicastRoutes& unicastEntries) const;

 private:
  std::vector<RibPolicyStatement> statements_;
  std::chrono::steady_clock::time_point validUntil_;
};

}  // namespace openr
