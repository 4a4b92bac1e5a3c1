// LinkState.cpp — host mirror of openr::LinkState (see LinkState.h).
//
// Topology bookkeeping restates the reference behaviour (LinkState.cpp:54-760):
// bidirectional link formation, hold-down values, change detection and memo
// invalidation happen at the same points with the same results, so that
// linksFromNode() iterates in the same order as the reference on the same
// standard library. runSpf is the GPU engine behind include/openr_spf.h.
#include "LinkState.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <sstream>

#include "HostParallel.h"
#include "../../../include/openr_spf.h"

namespace openr {

// ---------------------------------------------------------------------------
// counters
// ---------------------------------------------------------------------------
SpfCounters& SpfCounters::get() {
  static SpfCounters c;
  return c;
}
void SpfCounters::addSpfRun(double ms, uint64_t runs) {
  std::lock_guard<std::mutex> g(mu_);
  runs_ += runs;
  msSum_ += ms;
  samples_ += 1;
}
void SpfCounters::reset() {
  std::lock_guard<std::mutex> g(mu_);
  runs_ = samples_ = 0;
  msSum_ = 0.0;
}
uint64_t SpfCounters::spfRuns() const {
  std::lock_guard<std::mutex> g(mu_);
  return runs_;
}
double SpfCounters::spfMsAvg() const {
  std::lock_guard<std::mutex> g(mu_);
  return samples_ ? msSum_ / (double)samples_ : 0.0;
}

// ---------------------------------------------------------------------------
// HoldableValue (reference LinkState.cpp:54-125)
// ---------------------------------------------------------------------------
template <class T>
HoldableValue<T>::HoldableValue(T val) : val_(val) {}

template <class T>
void HoldableValue<T>::operator=(T val) {
  val_ = val;
  heldVal_.reset();
  holdTtl_ = 0;
}

template <class T>
const T& HoldableValue<T>::value() const {
  return heldVal_ ? *heldVal_ : val_;
}

template <class T>
bool HoldableValue<T>::hasHold() const {
  return heldVal_.has_value();
}

template <class T>
bool HoldableValue<T>::decrementTtl() {
  if (!heldVal_) return false;
  if (--holdTtl_ != 0) return false;
  heldVal_.reset();
  return true;
}

template <class T>
bool HoldableValue<T>::updateValue(T val, LinkStateMetric holdUpTtl, LinkStateMetric holdDownTtl) {
  if (val == val_) return false;  // same value: no-op
  if (hasHold()) {
    // a second change during a hold falls back to a fast update
    heldVal_.reset();
    holdTtl_ = 0;
  } else {
    holdTtl_ = isChangeBringingUp(val) ? holdUpTtl : holdDownTtl;
    if (holdTtl_ != 0) heldVal_ = val_;
  }
  val_ = val;
  return !hasHold();
}

template <>
bool HoldableValue<bool>::isChangeBringingUp(bool val) const {
  return val_ && !val;  // overload cleared
}

template <>
bool HoldableValue<LinkStateMetric>::isChangeBringingUp(LinkStateMetric val) const {
  return val < val_;  // metric improved
}

template class HoldableValue<LinkStateMetric>;
template class HoldableValue<bool>;

// ---------------------------------------------------------------------------
// Link (reference LinkState.cpp:127-377)
// ---------------------------------------------------------------------------
namespace {
using NamePair = std::pair<std::string, std::string>;
std::pair<NamePair, NamePair> orderEnds(const std::string& n1, const std::string& if1, const std::string& n2,
                                        const std::string& if2) {
  return std::minmax(NamePair(n1, if1), NamePair(n2, if2));
}
}  // namespace

Link::Link(const std::string& area, const std::string& nodeName1, const std::string& if1,
           const std::string& nodeName2, const std::string& if2)
    : area_(area),
      orderedNames_(orderEnds(nodeName1, if1, nodeName2, if2)),
      hash(std::hash<std::pair<NamePair, NamePair>>()(orderedNames_)) {
  ends_[0].node = nodeName1;
  ends_[0].iface = if1;
  ends_[1].node = nodeName2;
  ends_[1].iface = if2;
}

Link::Link(const std::string& area, const std::string& nodeName1, const thrift::Adjacency& adj1,
           const std::string& nodeName2, const thrift::Adjacency& adj2)
    : Link(area, nodeName1, adj1.ifName, nodeName2, adj2.ifName) {
  const thrift::Adjacency* adjs[2] = {&adj1, &adj2};
  for (int i = 0; i < 2; ++i) {
    End& end = ends_[i];
    // i32 Adjacency.metric -> u64 LinkStateMetric (negative values wrap)
    end.metric = static_cast<LinkStateMetric>(adjs[i]->metric);
    end.overload = adjs[i]->isOverloaded;
    end.adjLabel = adjs[i]->adjLabel;
    end.nhV4 = adjs[i]->nextHopV4;
    end.nhV6 = adjs[i]->nextHopV6;
  }
}

int Link::sideOf(const std::string& nodeName) const {
  if (ends_[0].node == nodeName) return 0;
  if (ends_[1].node == nodeName) return 1;
  throw std::invalid_argument(nodeName);
}

const std::string& Link::getOtherNodeName(const std::string& nodeName) const {
  return ends_[1 - sideOf(nodeName)].node;
}
const std::string& Link::firstNodeName() const { return orderedNames_.first.first; }
const std::string& Link::secondNodeName() const { return orderedNames_.second.first; }
const std::string& Link::getIfaceFromNode(const std::string& nodeName) const {
  return ends_[sideOf(nodeName)].iface;
}
LinkStateMetric Link::getMetricFromNode(const std::string& nodeName) const {
  return ends_[sideOf(nodeName)].metric.value();
}
int32_t Link::getAdjLabelFromNode(const std::string& nodeName) const { return ends_[sideOf(nodeName)].adjLabel; }
bool Link::getOverloadFromNode(const std::string& nodeName) const {
  return ends_[sideOf(nodeName)].overload.value();
}
const thrift::BinaryAddress& Link::getNhV4FromNode(const std::string& nodeName) const {
  return ends_[sideOf(nodeName)].nhV4;
}
const thrift::BinaryAddress& Link::getNhV6FromNode(const std::string& nodeName) const {
  return ends_[sideOf(nodeName)].nhV6;
}
void Link::setNhV4FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV4) {
  ends_[sideOf(nodeName)].nhV4 = nhV4;
}
void Link::setNhV6FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV6) {
  ends_[sideOf(nodeName)].nhV6 = nhV6;
}
void Link::setHoldUpTtl(LinkStateMetric ttl) { holdUpTtl_ = ttl; }

bool Link::isUp() const {
  return holdUpTtl_ == 0 && !ends_[0].overload.value() && !ends_[1].overload.value();
}

bool Link::decrementHolds() {
  bool expired = false;
  if (holdUpTtl_ != 0) expired |= (--holdUpTtl_ == 0);
  for (End& end : ends_) {
    expired |= end.metric.decrementTtl();
    expired |= end.overload.decrementTtl();
  }
  return expired;
}

bool Link::hasHolds() const {
  if (holdUpTtl_ != 0) return true;
  for (const End& end : ends_)
    if (end.metric.hasHold() || end.overload.hasHold()) return true;
  return false;
}

bool Link::setMetricFromNode(const std::string& nodeName, LinkStateMetric d, LinkStateMetric holdUpTtl,
                             LinkStateMetric holdDownTtl) {
  return ends_[sideOf(nodeName)].metric.updateValue(d, holdUpTtl, holdDownTtl);
}

void Link::setAdjLabelFromNode(const std::string& nodeName, int32_t adjLabel) {
  ends_[sideOf(nodeName)].adjLabel = adjLabel;
}

bool Link::setOverloadFromNode(const std::string& nodeName, bool overload, LinkStateMetric holdUpTtl,
                               LinkStateMetric holdDownTtl) {
  const bool wasUp = isUp();
  ends_[sideOf(nodeName)].overload.updateValue(overload, holdUpTtl, holdDownTtl);
  // simplex overloads are not modelled: only an up/down flip changes topology
  return wasUp != isUp();
}

bool Link::operator<(const Link& other) const {
  if (hash != other.hash) return hash < other.hash;
  return orderedNames_ < other.orderedNames_;
}

bool Link::operator==(const Link& other) const { return hash == other.hash && orderedNames_ == other.orderedNames_; }

std::string Link::toString() const {
  std::ostringstream os;
  os << area_ << " - " << ends_[0].node << "%" << ends_[0].iface << " <---> " << ends_[1].node << "%"
     << ends_[1].iface;
  return os.str();
}

std::string Link::directionalToString(const std::string& fromNode) const {
  const int s = sideOf(fromNode);
  std::ostringstream os;
  os << area_ << " - " << ends_[s].node << "%" << ends_[s].iface << " ---> " << ends_[1 - s].node << "%"
     << ends_[1 - s].iface;
  return os.str();
}

// ---------------------------------------------------------------------------
// engine handle
// ---------------------------------------------------------------------------
class SpfEngineHandle {
 public:
  SpfEngineHandle() {
    int dev = -1;
    if (const char* e = std::getenv("OPENR_SPF_DEVICE")) dev = std::atoi(e);
    int rc = dev >= 0 ? openr_spf_create(&dev, 1, &ctx_) : openr_spf_create(nullptr, 0, &ctx_);
    check(rc, "openr_spf_create");
  }
  ~SpfEngineHandle() { openr_spf_destroy(ctx_); }
  SpfEngineHandle(const SpfEngineHandle&) = delete;
  SpfEngineHandle& operator=(const SpfEngineHandle&) = delete;

  static void check(int rc, const char* what) {
    if (rc != OPENR_SPF_OK)
      throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " + openr_spf_last_error());
  }
  openr_spf_ctx* ctx() { return ctx_; }
  const void* owner = nullptr;   // LinkState whose graph is loaded
  uint64_t generation = 0;       // its mirror generation

 private:
  openr_spf_ctx* ctx_ = nullptr;
};

// ---------------------------------------------------------------------------
// LinkState (reference LinkState.cpp:379-803)
// ---------------------------------------------------------------------------
LinkState::LinkState(const std::string& area) : area_(area) {}

size_t LinkState::LinkPtrHash::operator()(const std::shared_ptr<Link>& l) const { return l->hash; }
bool LinkState::LinkPtrLess::operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const {
  return *lhs < *rhs;
}
bool LinkState::LinkPtrEqual::operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const {
  return *lhs == *rhs;
}

bool LinkState::pathAInPathB(Path const& a, Path const& b) {
  if (a.size() > b.size()) return false;
  for (size_t start = 0; start + a.size() <= b.size(); ++start) {
    size_t k = 0;
    while (k < a.size() && *a[k] == *b[start + k]) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

std::optional<LinkState::Path> LinkState::traceOnePath(std::string const& src, std::string const& dest,
                                                       SpfResult const& result, LinkSet& linksToIgnore) const {
  if (src == dest) return Path{};
  for (auto const& pl : result.at(dest).pathLinks()) {
    if (!linksToIgnore.insert(pl.link).second) continue;  // link already used by a path
    if (auto path = traceOnePath(src, pl.prevNode, result, linksToIgnore)) {
      path->push_back(pl.link);
      return path;
    }
  }
  return std::nullopt;
}

void LinkState::addLink(std::shared_ptr<Link> link) {
  if (!linkMap_[link->firstNodeName()].insert(link).second || !linkMap_[link->secondNodeName()].insert(link).second ||
      !allLinks_.insert(link).second)
    throw std::logic_error("addLink: duplicate link " + link->toString());
  markMirrorDirty();
}

void LinkState::removeLink(std::shared_ptr<Link> link) {
  if (!linkMap_.at(link->firstNodeName()).erase(link) || !linkMap_.at(link->secondNodeName()).erase(link) ||
      !allLinks_.erase(link))
    throw std::logic_error("removeLink: unknown link " + link->toString());
  markMirrorDirty();
}

void LinkState::removeNode(const std::string& nodeName) {
  auto it = linkMap_.find(nodeName);
  if (it == linkMap_.end()) return;  // node never had links (empty adjacency db)
  for (auto const& link : it->second) {
    if (!linkMap_.at(link->getOtherNodeName(nodeName)).erase(link) || !allLinks_.erase(link))
      throw std::logic_error("removeNode: inconsistent link map for " + nodeName);
  }
  linkMap_.erase(it);
  nodeOverloads_.erase(nodeName);
  markMirrorDirty();
}

const LinkState::LinkSet& LinkState::linksFromNode(const std::string& nodeName) const {
  static const LinkSet kEmpty;
  auto it = linkMap_.find(nodeName);
  return it == linkMap_.end() ? kEmpty : it->second;
}

std::vector<std::shared_ptr<Link>> LinkState::orderedLinksFromNode(const std::string& nodeName) const {
  const LinkSet& set = linksFromNode(nodeName);
  std::vector<std::shared_ptr<Link>> links(set.begin(), set.end());
  std::sort(links.begin(), links.end(), LinkPtrLess{});
  return links;
}

bool LinkState::updateNodeOverloaded(const std::string& nodeName, bool isOverloaded, LinkStateMetric holdUpTtl,
                                     LinkStateMetric holdDownTtl) {
  auto it = nodeOverloads_.find(nodeName);
  if (it != nodeOverloads_.end()) {
    // the mirror carries the effective (hold-aware) value: rebuild it only when that changed
    const bool changed = it->second.updateValue(isOverloaded, holdUpTtl, holdDownTtl);
    if (changed) attrNodes_.push_back(nodeName);  // attribute only: patched in place (applyAttrPatch)
    return changed;
  }
  nodeOverloads_.emplace(nodeName, HoldableValue<bool>{isOverloaded});
  markMirrorDirty();
  return false;  // a new node is not a topology change
}

bool LinkState::isNodeOverloaded(const std::string& nodeName) const {
  auto it = nodeOverloads_.find(nodeName);
  return it != nodeOverloads_.end() && it->second.value();
}

LinkState::LinkStateChange LinkState::decrementHolds() {
  LinkStateChange change;
  std::vector<std::shared_ptr<Link>> links;
  std::vector<std::string> nodes;
  for (auto& link : allLinks_)
    if (link->decrementHolds()) {
      change.topologyChanged = true;
      links.push_back(link);
    }
  for (auto& kv : nodeOverloads_)
    if (kv.second.decrementTtl()) {
      change.topologyChanged = true;
      nodes.push_back(kv.first);
    }
  if (change.topologyChanged) {
    clearMemos();  // LinkState.cpp:509-512
    applyAttrPatch(links, nodes);  // held values only: the link structure is unchanged
  }
  return change;
}

bool LinkState::hasHolds() const {
  for (auto& link : allLinks_)
    if (link->hasHolds()) return true;
  for (auto& kv : nodeOverloads_)
    if (kv.second.hasHold()) return true;
  return false;
}

void LinkState::indexAdjacencies(const std::string& nodeName) {
  auto& idx = ifIndex_[nodeName];
  idx.clear();
  const auto& adjs = adjacencyDatabases_.at(nodeName).adjacencies;
  for (uint32_t i = 0; i < adjs.size(); ++i) idx[adjs[i].ifName].push_back(i);
}

std::shared_ptr<Link> LinkState::maybeMakeLink(const std::string& nodeName, const thrift::Adjacency& adj) const {
  // a Link exists only if the other end advertises the reverse adjacency: the first
  // adjacency of the other node (LinkState.cpp:531-547 scans its list in order) with
  // otherNodeName == nodeName, ifName == adj.otherIfName, otherIfName == adj.ifName;
  // only positions whose ifName matches can qualify, so the index lists exactly those
  auto it = adjacencyDatabases_.find(adj.otherNodeName);
  if (it == adjacencyDatabases_.end()) return nullptr;
  auto ix = ifIndex_.find(adj.otherNodeName);
  if (ix == ifIndex_.end()) return nullptr;
  auto pos = ix->second.find(adj.otherIfName);
  if (pos == ix->second.end()) return nullptr;
  for (uint32_t i : pos->second) {
    const auto& back = it->second.adjacencies[i];
    if (back.otherNodeName == nodeName && adj.ifName == back.otherIfName)
      return std::make_shared<Link>(area_, nodeName, adj, adj.otherNodeName, back);
  }
  return nullptr;
}

std::vector<std::shared_ptr<Link>> LinkState::getOrderedLinkSet(const thrift::AdjacencyDatabase& adjDb) const {
  std::vector<std::shared_ptr<Link>> links;
  links.reserve(adjDb.adjacencies.size());
  for (const auto& adj : adjDb.adjacencies)
    if (auto link = maybeMakeLink(adjDb.thisNodeName, adj)) links.push_back(std::move(link));
  std::sort(links.begin(), links.end(), LinkPtrLess{});
  return links;
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(thrift::AdjacencyDatabase const& newDb,
                                                              LinkStateMetric holdUpTtl,
                                                              LinkStateMetric holdDownTtl) {
  return updateAdjacencyDatabase(thrift::AdjacencyDatabase(newDb), holdUpTtl, holdDownTtl);
}

LinkState::LinkStateChange LinkState::updateAdjacencyDatabase(thrift::AdjacencyDatabase&& db,
                                                              LinkStateMetric holdUpTtl,
                                                              LinkStateMetric holdDownTtl) {
  LinkStateChange change;
  const std::string nodeName = db.thisNodeName;
  // the CSR mirror changes only with the topology (addLink / removeLink mark it, and so
  // does an effective metric / overload / up-down change below); a re-advertisement that
  // changes nothing, or only labels and next-hop addresses, keeps mirror and device graph

  attrLinks_.clear();
  attrNodes_.clear();
  thrift::AdjacencyDatabase& stored = adjacencyDatabases_[nodeName];
  thrift::AdjacencyDatabase prior(std::move(stored));
  stored = std::move(db);
  labeledNodes_ += (stored.nodeLabel != 0 ? 1 : 0) - (prior.nodeLabel != 0 ? 1 : 0);
  ++adjDbVersion_;
  const thrift::AdjacencyDatabase& newDb = stored;
  indexAdjacencies(nodeName);

  // both sides ordered by <hash, names> so one merge pass finds adds/removes/updates
  const auto oldLinks = orderedLinksFromNode(nodeName);
  const auto newLinks = getOrderedLinkSet(newDb);

  change.topologyChanged |= updateNodeOverloaded(nodeName, newDb.isOverloaded, holdUpTtl, holdDownTtl);
  change.nodeLabelChanged = prior.nodeLabel != newDb.nodeLabel;

  size_t ni = 0, oi = 0;
  while (ni < newLinks.size() || oi < oldLinks.size()) {
    const bool takeNew = ni < newLinks.size() && (oi == oldLinks.size() || *newLinks[ni] < *oldLinks[oi]);
    const bool takeOld = !takeNew && oi < oldLinks.size() && (ni == newLinks.size() || *oldLinks[oi] < *newLinks[ni]);
    if (takeNew) {  // link came up (possibly held down)
      newLinks[ni]->setHoldUpTtl(holdUpTtl);
      change.topologyChanged |= newLinks[ni]->isUp();
      addLink(newLinks[ni]);
      ++ni;
      continue;
    }
    if (takeOld) {  // link went away
      change.topologyChanged |= oldLinks[oi]->isUp();
      removeLink(oldLinks[oi]);
      ++oi;
      continue;
    }
    // same link on both sides: update the object we already hold
    Link& cur = *oldLinks[oi];
    const Link& upd = *newLinks[ni];
    bool attr = false;
    if (upd.getMetricFromNode(nodeName) != cur.getMetricFromNode(nodeName))
      attr |= cur.setMetricFromNode(nodeName, upd.getMetricFromNode(nodeName), holdUpTtl, holdDownTtl);
    if (upd.getOverloadFromNode(nodeName) != cur.getOverloadFromNode(nodeName))
      attr |= cur.setOverloadFromNode(nodeName, upd.getOverloadFromNode(nodeName), holdUpTtl, holdDownTtl);
    if (attr) {
      change.topologyChanged = true;
      attrLinks_.push_back(oldLinks[oi]);
    }
    if (upd.getAdjLabelFromNode(nodeName) != cur.getAdjLabelFromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setAdjLabelFromNode(nodeName, upd.getAdjLabelFromNode(nodeName));
    }
    if (upd.getNhV4FromNode(nodeName) != cur.getNhV4FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setNhV4FromNode(nodeName, upd.getNhV4FromNode(nodeName));
    }
    if (upd.getNhV6FromNode(nodeName) != cur.getNhV6FromNode(nodeName)) {
      change.linkAttributesChanged = true;
      cur.setNhV6FromNode(nodeName, upd.getNhV6FromNode(nodeName));
    }
    ++ni;
    ++oi;
  }
  if (change.topologyChanged) {
    clearMemos();  // LinkState.cpp:714-717
    // links added / removed marked the mirror for a rebuild already; otherwise only
    // attributes moved (metric, Link::isUp, node overload): patch in place
    applyAttrPatch(attrLinks_, attrNodes_);
  }
  attrLinks_.clear();
  attrNodes_.clear();
  return change;
}

LinkState::LinkStateChange LinkState::deleteAdjacencyDatabase(const std::string& nodeName) {
  LinkStateChange change;
  auto it = adjacencyDatabases_.find(nodeName);
  if (it != adjacencyDatabases_.end()) {
    removeNode(nodeName);
    if (it->second.nodeLabel != 0) --labeledNodes_;
    ++adjDbVersion_;
    adjacencyDatabases_.erase(it);
    ifIndex_.erase(nodeName);
    clearMemos();
    markMirrorDirty();
    change.topologyChanged = true;
  }
  return change;
}

std::optional<LinkStateMetric> LinkState::getMetricFromAToB(std::string const& a, std::string const& b,
                                                            bool useLinkMetric) const {
  if (a == b) return 0;
  auto const& res = getSpfResult(a, useLinkMetric);
  auto it = res.find(b);
  if (it == res.end()) return std::nullopt;
  return it->second.metric();
}

LinkStateMetric LinkState::getMaxHopsToNode(const std::string& nodeName) const {
  LinkStateMetric best = 0;
  for (auto const& kv : getSpfResult(nodeName, false)) best = std::max(best, kv.second.metric());
  return best;
}

void LinkState::throwIfFrozen(const char* what, const std::string& key) const {
  if (frozen_.v.load(std::memory_order_relaxed))
    throw std::logic_error(std::string("LinkState::") + what + "(" + key +
                           "): memo miss while the memo is frozen (a parallel route build read a result its "
                           "prefetch did not cover)");
}

std::vector<LinkState::Path> const& LinkState::getKthPaths(const std::string& src, const std::string& dest,
                                                           size_t k) const {
  if (k < 1) throw std::invalid_argument("getKthPaths: k must be >= 1");  // CHECK_GE(k, 1)
  const auto key = std::make_tuple(src, dest, k);
  auto it = kthPathResults_.find(key);
  if (it != kthPathResults_.end()) return it->second;
  throwIfFrozen("getKthPaths", src + "->" + dest);
  if (k <= 2) {  // device-traced token rows (prefetchKthPaths): counted like the calls below
    if (const uint32_t* row = kthPathTokens(src, dest, k)) {
      std::vector<Path> paths;
      decodeTokens(row, paths);
      return kthPathResults_.emplace(key, std::move(paths)).first->second;
    }
  }
  if (k <= 2) {  // prefetched: replay the memo and counter effects of the call sequence below
    auto st = kthStaged_.find(std::make_pair(src, dest));
    if (st != kthStaged_.end()) {
      if (k == 1) {
        getSpfResult(src, true);
        return kthPathResults_.emplace(key, st->second.k1).first->second;
      }
      bool anyLink = false;
      for (auto const& path : getKthPaths(src, dest, 1)) anyLink |= !path.empty();
      if (anyLink) SpfCounters::get().addSpfRun(st->second.ms);  // runSpf(src, true, ignore)
      else getSpfResult(src, true);
      auto paths = std::move(st->second.k2);
      kthStaged_.erase(st);
      return kthPathResults_.emplace(key, std::move(paths)).first->second;
    }
  }
  LinkSet ignore;
  for (size_t i = 1; i < k; ++i)
    for (auto const& path : getKthPaths(src, dest, i))
      for (auto const& link : path) ignore.insert(link);
  std::vector<Path> paths;
  SpfResult fresh;
  const SpfResult* res = nullptr;
  if (ignore.empty()) {
    res = &getSpfResult(src, true);
  } else {
    fresh = runSpf(src, true, ignore);
    res = &fresh;
  }
  if (res->count(dest)) {
    LinkSet visited;
    auto path = traceOnePath(src, dest, *res, visited);
    while (path && !path->empty()) {
      paths.push_back(std::move(*path));
      path = traceOnePath(src, dest, *res, visited);
    }
  }
  return kthPathResults_.emplace(key, std::move(paths)).first->second;
}

LinkState::SpfResult const& LinkState::getSpfResult(const std::string& nodeName, bool useLinkMetric) const {
  const auto key = std::make_pair(nodeName, useLinkMetric);
  auto it = spfResults_.find(key);
  if (it == spfResults_.end()) {  // LinkState.cpp:793-803: a miss runs the SPF
    throwIfFrozen("getSpfResult", nodeName);
    prefetchSpfResults({nodeName}, useLinkMetric);
    it = spfResults_.find(key);
  }
  if (!it->second.counted.v.exchange(1, std::memory_order_relaxed))
    SpfCounters::get().addSpfRun(it->second.ms);  // its logical run counts at this first read
  return materialize(it->second, useLinkMetric);
}

// The memo entry's SpfResult map, built from its dense row on first read (once, also when
// several route-build workers read it together)
const LinkState::SpfResult& LinkState::materialize(const MemoEntry& e, bool useLinkMetric) const {
  if (e.row == UINT32_MAX) return e.res;
  MemoEntry& me = const_cast<MemoEntry&>(e);
  std::call_once(*me.once.f, [&]() {
    const CsrMirror& m = e.snap ? e.snap->mirror : mirror_;
    const DenseRows& d = e.snap ? e.snap->rows[useLinkMetric ? 1 : 0] : dense_[useLinkMetric ? 1 : 0];
    const uint32_t V = (uint32_t)m.names.size(), src = d.src[e.row];
    std::vector<uint64_t> distv(V);
    d.load(e.row, 1, distv.data());
    const uint64_t* dist = distv.data();
    const uint8_t* h = d.nh.data() + (size_t)e.row * V * d.nb;
    const std::vector<uint32_t>& nbrs = d.nbrs[e.row];
    SpfResult res;
    res.reserve(V);
    for (uint32_t v = 0; v < V; ++v) {
      if (dist[v] == UINT64_MAX) continue;
      NodeSpfResult r(dist[v]);
      const uint8_t* hv = h + (size_t)v * d.nb;
      for (uint32_t i = 0; i < nbrs.size(); ++i)
        if ((hv[i >> 3] >> (i & 7)) & 1u) r.addNextHop(m.names[nbrs[i]]);
      res.emplace(m.names[v], std::move(r));
    }
    // pathLinks (LinkState.cpp:846-873): every usable in-edge u->v out of an expanding
    // node u (not overloaded, or the source) with dist[u] + w == dist[v]; with metrics in
    // [1, 2^31-1] these are exactly the links the reference's relaxations appended, and its
    // (metric, name) pop order then row position orders them
    std::vector<uint32_t> order;
    const uint32_t E = (uint32_t)m.col.size();
    for (uint32_t e2 = 0; e2 < E; ++e2) {
      const uint32_t u = m.edgeOwner[e2], v = m.col[e2];
      if (!m.edgeUp[e2] || dist[u] == UINT64_MAX || dist[v] == UINT64_MAX || u == v) continue;
      if (m.overloaded[u] && u != src) continue;
      const uint64_t w = useLinkMetric ? m.metric[e2] : 1u;
      if (dist[u] + w == dist[v]) order.push_back(e2);
    }
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
      const uint32_t ux = m.edgeOwner[x], uy = m.edgeOwner[y];
      if (dist[ux] != dist[uy]) return dist[ux] < dist[uy];
      if (m.nameRank[ux] != m.nameRank[uy]) return m.nameRank[ux] < m.nameRank[uy];
      return x < y;
    });
    for (uint32_t e2 : order) res.at(m.names[m.col[e2]]).addPath(m.links[m.linkId[e2]], m.names[m.edgeOwner[e2]]);
    me.res = std::move(res);
  });
  return e.res;
}

void LinkState::prefetchSpfResults(const std::vector<std::string>& nodes, bool useLinkMetric) const {
  std::vector<std::string> missing;
  for (auto const& n : nodes)
    if (!spfResults_.count(std::make_pair(n, useLinkMetric))) missing.push_back(n);
  std::sort(missing.begin(), missing.end());
  missing.erase(std::unique(missing.begin(), missing.end()), missing.end());
  if (missing.empty()) return;
  throwIfFrozen("prefetchSpfResults", missing.front());
  auto entry = [&](const std::string& n) -> MemoEntry& {
    return spfResults_
        .emplace(std::piecewise_construct, std::forward_as_tuple(std::make_pair(n, useLinkMetric)),
                 std::forward_as_tuple())
        .first->second;
  };
  if (!denseEligible(useLinkMetric)) {  // zero / wrapped metrics: exact pop order, materialised now
    double ms = 0;
    auto results = runSpfBatch(missing, useLinkMetric, std::vector<const LinkSet*>(missing.size(), nullptr), &ms);
    for (size_t i = 0; i < missing.size(); ++i) {
      MemoEntry& e = entry(missing[i]);
      e.res = std::move(results[i]);
      e.ms = ms / (double)missing.size();
    }
    return;
  }
  const CsrMirror& m = csrMirror();
  ensureEngineGraph();
  DenseRows& d = dense_[useLinkMetric ? 1 : 0];
  double rms = 0;
  const size_t kept = d.src.size();
  refreshDense(useLinkMetric, &rms);  // rows a patch left stale: only affected ones re-solved
  const double keptMs = kept ? rms / (double)kept : 0.0;
  std::vector<uint32_t> ids;
  std::vector<const std::string*> idName;
  for (auto const& n : missing) {
    auto it = m.id.find(n);
    if (it == m.id.end()) {  // unknown to the graph: the reference pops only the source itself
      entry(n).res.emplace(n, NodeSpfResult(0));
      continue;
    }
    auto sl = d.slot.find(it->second);
    if (sl != d.slot.end()) {  // a row kept (and refreshed) across attribute changes
      MemoEntry& e = entry(n);
      e.row = sl->second;
      e.ms = keptMs;
      continue;
    }
    ids.push_back(it->second);
    idName.push_back(&n);
  }
  if (ids.empty()) return;
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t V = (uint32_t)m.names.size(), n = (uint32_t)ids.size();
  uint32_t nb = 1;
  SpfEngineHandle::check(openr_spf_nh_bytes(engine_->ctx(), &nb), "openr_spf_nh_bytes");
  if (d.src.empty()) d.nb = nb;
  const size_t r0 = d.src.size();
  d.V = V;
  {
    HostPhase ph("prefetch: resize rows");
    d.resizeRows(r0 + n);
  }
  // the engine's u64 rows through a staging buffer of at most ~64 MB
  const uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(n, (64u << 20) / (8u * (size_t)std::max(V, 1u))));
  std::vector<uint64_t> stage((size_t)chunk * V);
  double msSolve = 0, msStore = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += chunk) {
    const uint32_t k = std::min(chunk, n - c0);
    HostPhase ps("");
    SpfEngineHandle::check(openr_spf_solve(engine_->ctx(), ids.data() + c0, k,
                                           useLinkMetric ? (uint32_t)OPENR_SPF_USE_LINK_METRIC : 0u, stage.data(),
                                           d.nh.data() + (r0 + c0) * V * d.nb, d.nb, nullptr),
                           "openr_spf_solve");
    msSolve += ps.ms();
    HostPhase pt("");
    d.store(r0 + c0, k, stage.data());
    msStore += pt.ms();
  }
  if (hostProf()) std::fprintf(stderr, "[host] prefetch: %u rows, solve + D2H %.1f ms, store %.1f ms\n", n, msSolve, msStore);
  HostPhase pn("prefetch: neighbour maps + memo entries");
  d.nbrs.resize(r0 + n);
  std::vector<uint32_t> buf(V ? V : 1);
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t nn = 0;
    SpfEngineHandle::check(openr_spf_neighbor_map(engine_->ctx(), ids[k], buf.data(), (uint32_t)buf.size(), &nn),
                           "openr_spf_neighbor_map");
    d.nbrs[r0 + k].assign(buf.begin(), buf.begin() + nn);
    d.slot[ids[k]] = (uint32_t)(r0 + k);
    d.src.push_back(ids[k]);
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / n;
  for (uint32_t k = 0; k < n; ++k) {
    MemoEntry& e = entry(*idName[k]);
    e.row = (uint32_t)(r0 + k);
    e.ms = ms;
  }
}

// ---------------------------------------------------------------------------
// SpfView: dense reads of a memo entry (route build fast path)
// ---------------------------------------------------------------------------
LinkState::SpfView LinkState::getSpfView(const std::string& nodeName, bool useLinkMetric) const {
  const auto key = std::make_pair(nodeName, useLinkMetric);
  auto it = spfResults_.find(key);
  if (it == spfResults_.end()) {
    throwIfFrozen("getSpfView", nodeName);
    prefetchSpfResults({nodeName}, useLinkMetric);
    it = spfResults_.find(key);
  }
  if (!it->second.counted.v.exchange(1, std::memory_order_relaxed)) SpfCounters::get().addSpfRun(it->second.ms);
  SpfView v;
  const MemoEntry& e = it->second;
  if (e.row == UINT32_MAX) {
    v.map_ = &e.res;
    return v;
  }
  v.m_ = e.snap ? &e.snap->mirror : &mirror_;
  v.rows_ = e.snap ? &e.snap->rows[useLinkMetric ? 1 : 0] : &dense_[useLinkMetric ? 1 : 0];
  v.row_ = e.row;
  v.keep_ = e.snap;
  return v;
}

void LinkState::DenseRows::resizeRows(size_t rows) {
  if (wide) dist64.resize(rows * V);
  else dist32.resize(rows * V);
  nh.resize(rows * V * nb);
}

void LinkState::DenseRows::store(size_t r0, size_t n, const uint64_t* rows) {
  const size_t cnt = n * V;
  if (!wide) {
    bool fits = true;
    for (size_t i = 0; i < cnt && fits; ++i) fits = rows[i] == UINT64_MAX || rows[i] < UINT32_MAX;
    if (!fits) {  // a finite distance past u32: every row widens
      dist64.resize(dist32.size());
      for (size_t i = 0; i < dist32.size(); ++i) dist64[i] = dist32[i] == UINT32_MAX ? UINT64_MAX : dist32[i];
      std::vector<uint32_t>().swap(dist32);
      wide = true;
    }
  }
  if (wide) {
    std::copy(rows, rows + cnt, dist64.begin() + r0 * V);
    return;
  }
  uint32_t* o = dist32.data() + r0 * V;
  for (size_t i = 0; i < cnt; ++i) o[i] = rows[i] == UINT64_MAX ? UINT32_MAX : (uint32_t)rows[i];
}

void LinkState::DenseRows::load(size_t r0, size_t n, uint64_t* rows) const {
  const size_t cnt = n * V;
  if (wide) {
    std::copy(dist64.begin() + r0 * V, dist64.begin() + r0 * V + cnt, rows);
    return;
  }
  const uint32_t* x = dist32.data() + r0 * V;
  for (size_t i = 0; i < cnt; ++i) rows[i] = x[i] == UINT32_MAX ? UINT64_MAX : (uint64_t)x[i];
}

const uint8_t* LinkState::SpfView::nh(uint32_t v) const {
  const DenseRows& d = *static_cast<const DenseRows*>(rows_);
  return d.nh.data() + ((size_t)row_ * m_->names.size() + v) * d.nb;
}

uint32_t LinkState::SpfView::nhBytes() const { return static_cast<const DenseRows*>(rows_)->nb; }

const std::vector<uint32_t>& LinkState::SpfView::nhNeighbours() const {
  return static_cast<const DenseRows*>(rows_)->nbrs[row_];
}

int32_t LinkState::SpfView::id(const std::string& node) const {
  auto it = m_->id.find(node);
  if (it == m_->id.end() || dist(it->second) == UINT64_MAX) return -1;
  return (int32_t)it->second;
}

bool LinkState::SpfView::reached(const std::string& node) const {
  if (map_) return map_->count(node) != 0;
  return id(node) >= 0;
}

LinkStateMetric LinkState::SpfView::metric(const std::string& node) const {
  if (map_) return map_->at(node).metric();
  const int32_t v = id(node);
  if (v < 0) throw std::out_of_range("SpfView::metric: " + node + " not reached");
  return dist((uint32_t)v);
}

std::vector<std::string> LinkState::SpfView::nextHops(const std::string& node) const {
  std::vector<std::string> out;
  if (map_) {
    auto const& nh = map_->at(node).nextHops();
    out.assign(nh.begin(), nh.end());
    return out;
  }
  const int32_t v = id(node);
  if (v < 0) throw std::out_of_range("SpfView::nextHops: " + node + " not reached");
  const DenseRows& d = *static_cast<const DenseRows*>(rows_);
  const uint8_t* hv = nh((uint32_t)v);
  const std::vector<uint32_t>& nbrs = d.nbrs[row_];
  for (uint32_t i = 0; i < nbrs.size(); ++i)
    if ((hv[i >> 3] >> (i & 7)) & 1u) out.push_back(m_->names[nbrs[i]]);
  return out;
}

void LinkState::retireDenseRows() {
  // rows are indexed by the ids of mirror_ (they were solved on it; a pending patch would
  // have cleared the memo first, so no entry points at a stale row)
  if (mirrorDirty_) return;
  // live entries per row set; a set most of whose rows are still referenced moves into the
  // snapshot whole, a sparsely referenced one keeps only those rows (the rest
  // would stay resident beside the fresh rows until every entry is cleared)
  std::vector<MemoEntry*> live[2];
  for (auto& kv : spfResults_) {
    MemoEntry& e = kv.second;
    if (e.row == UINT32_MAX || e.snap) continue;
    live[kv.first.second ? 1 : 0].push_back(&e);
  }
  if (live[0].empty() && live[1].empty()) return;
  auto snap = std::make_shared<RowSnapshot>();
  snap->mirror = std::move(mirror_);
  for (int um = 0; um < 2; ++um) {
    DenseRows& d = dense_[um];
    if (live[um].empty()) continue;
    if (2 * live[um].size() >= d.src.size()) {
      ustats_.rowsRetired += d.src.size();
      snap->rows[um] = std::move(d);
    } else {
      ustats_.rowsRetired += live[um].size();
      DenseRows& o = snap->rows[um];
      o.nb = d.nb;
      o.V = d.V;
      o.wide = d.wide;
      o.stale = d.stale;
      o.resizeRows(live[um].size());
      const size_t V = d.V, nbv = (size_t)d.V * d.nb;
      for (uint32_t k = 0; k < live[um].size(); ++k) {
        MemoEntry& e = *live[um][k];
        const size_t r = e.row;
        if (d.wide) std::copy_n(d.dist64.begin() + r * V, V, o.dist64.begin() + k * V);
        else std::copy_n(d.dist32.begin() + r * V, V, o.dist32.begin() + k * V);
        std::copy_n(d.nh.begin() + r * nbv, nbv, o.nh.begin() + k * nbv);
        o.src.push_back(d.src[r]);
        o.slot.emplace(d.src[r], k);
        o.nbrs.push_back(d.nbrs[r]);
        e.row = k;
      }
    }
  }
  for (auto& l : live)
    for (MemoEntry* e : l) e->snap = snap;
}

// ---------------------------------------------------------------------------
// CSR mirror + engine-backed runSpf
// ---------------------------------------------------------------------------
const LinkState::CsrMirror& LinkState::csrMirror() const {
  if (!mirrorDirty_) return mirror_;
  CsrMirror m;
  // node set: every node with an adjacency database or a link; ids in name order
  for (auto const& kv : adjacencyDatabases_) m.names.push_back(kv.first);
  for (auto const& kv : linkMap_)
    if (!adjacencyDatabases_.count(kv.first)) m.names.push_back(kv.first);
  std::sort(m.names.begin(), m.names.end());
  const uint32_t V = (uint32_t)m.names.size();
  m.id.reserve(V);  // lookup-only: bucket count is not observable
  for (uint32_t i = 0; i < V; ++i) m.id.emplace(m.names[i], i);
  m.nameRank.resize(V);
  for (uint32_t i = 0; i < V; ++i) m.nameRank[i] = i;
  auto& linkIds = m.linkIndex;
  // every link appears in the rows of its two ends: size the columns once
  const size_t maxE = 2 * allLinks_.size();
  linkIds.reserve(allLinks_.size());
  m.links.reserve(allLinks_.size());
  m.linkEdges.reserve(2 * allLinks_.size());
  m.col.reserve(maxE);
  m.metric.reserve(maxE);
  m.linkId.reserve(maxE);
  m.edgeUp.reserve(maxE);
  m.edgeOwner.reserve(maxE);
  m.rowPtr.assign(V + 1, 0);
  m.overloaded.assign(V, 0);
  for (uint32_t u = 0; u < V; ++u) {
    const std::string& name = m.names[u];
    m.overloaded[u] = isNodeOverloaded(name) ? 1 : 0;
    // row order == linksFromNode(u) iteration order (pathLinks order among parallel links)
    for (auto const& link : linksFromNode(name)) {
      auto ins = linkIds.emplace(link.get(), (uint32_t)m.links.size());
      if (ins.second) m.links.push_back(link);
      if (ins.second) m.linkEdges.insert(m.linkEdges.end(), {UINT32_MAX, UINT32_MAX});
      m.linkEdges[2 * ins.first->second + (m.linkEdges[2 * ins.first->second] == UINT32_MAX ? 0 : 1)] =
          (uint32_t)m.col.size();
      m.col.push_back(m.id.at(link->getOtherNodeName(name)));
      m.metric.push_back(link->getMetricFromNode(name));
      if (link->isUp() && (m.metric.back() == 0 || m.metric.back() > 0x7FFFFFFFull)) m.metricsPositive = false;
      m.linkId.push_back(ins.first->second);
      m.edgeUp.push_back(link->isUp() ? 1 : 0);
      m.edgeOwner.push_back(u);
    }
    m.rowPtr[u + 1] = (uint32_t)m.col.size();
  }
  mirror_ = std::move(m);
  mirrorDirty_ = false;
  // process-wide: a graph uploaded by another LinkState (or by an earlier object at this
  // address) never matches this mirror's generation
  static std::atomic<uint64_t> generations{0};
  mirrorGeneration_ = ++generations;
  mirror_.generation = mirrorGeneration_;
  return mirror_;
}

// the engine holds this LinkState's current mirror (uploaded on first use after a rebuild)
void LinkState::ensureEngineGraph() const {
  const CsrMirror& m = csrMirror();
  if (!engine_) engine_ = std::make_shared<SpfEngineHandle>();
  if (engine_->owner == this && engine_->generation == mirrorGeneration_) return;
  openr_spf_graph g{};
  g.num_nodes = (uint32_t)m.names.size();
  g.num_dir_edges = (uint32_t)m.col.size();
  g.num_links = (uint32_t)m.links.size();
  g.row_ptr = m.rowPtr.data();
  g.col = m.col.data();
  g.metric = m.metric.data();
  g.link_id = m.linkId.data();
  g.edge_up = m.edgeUp.data();
  g.node_overloaded = m.overloaded.data();
  g.name_rank = m.nameRank.data();
  SpfEngineHandle::check(openr_spf_set_graph(engine_->ctx(), &g), "openr_spf_set_graph");
  engine_->owner = this;
  engine_->generation = mirrorGeneration_;
  ++ustats_.graphUploads;
  // rows the memo holds were solved on this same mirror; rows a patch left stale need the
  // engine's delta, which the upload discards
  for (auto& d : dense_)
    if (d.stale) d.clear();
}

// ---------------------------------------------------------------------------
// Attribute-only changes (round 3): the reference clears its memo and
// re-runs every SPF it is asked for (LinkState.cpp:509-512, 714-717). Here the memo's
// results are cleared the same way, but the engine's resident graph is patched in place
// (openr_spf_patch_graph: no CSR rebuild, no upload) and the memo's dense rows stay: the
// next read refreshes them (openr_spf_refresh: only rows the change can affect are
// re-solved) instead of re-solving every source.
// ---------------------------------------------------------------------------
void LinkState::applyAttrPatch(const std::vector<std::shared_ptr<Link>>& links, const std::vector<std::string>& nodes) {
  if (mirrorDirty_) return;  // the structure changed too: the mirror is rebuilt on next use
  if (links.empty() && nodes.empty()) return;
  CsrMirror& m = mirror_;
  std::vector<uint32_t> eids, lids, nids;
  std::vector<uint64_t> emet;
  std::vector<uint8_t> lup, novl;
  for (auto const& link : links) {
    auto it = m.linkIndex.find(link.get());
    if (it == m.linkIndex.end()) {  // not in the mirror (cannot happen for a same-structure update)
      markMirrorDirty();
      return;
    }
    const uint32_t lid = it->second;
    const bool up = link->isUp();
    lids.push_back(lid);
    lup.push_back(up ? 1 : 0);
    for (int k = 0; k < 2; ++k) {
      const uint32_t e = m.linkEdges[2 * lid + k];
      if (e == UINT32_MAX) continue;
      const uint64_t w = link->getMetricFromNode(m.names[m.edgeOwner[e]]);
      m.metric[e] = w;
      m.edgeUp[e] = up ? 1 : 0;
      eids.push_back(e);
      emet.push_back(w);
    }
  }
  for (auto const& name : nodes) {
    auto it = m.id.find(name);
    if (it == m.id.end()) {
      markMirrorDirty();
      return;
    }
    nids.push_back(it->second);
    novl.push_back(isNodeOverloaded(name) ? 1 : 0);
    m.overloaded[it->second] = novl.back();
  }
  m.metricsPositive = true;
  for (size_t e = 0; e < m.col.size(); ++e)
    if (m.edgeUp[e] && (m.metric[e] == 0 || m.metric[e] > 0x7FFFFFFFull)) m.metricsPositive = false;
  if (!engine_ || engine_->owner != this || engine_->generation != mirrorGeneration_) {
    // the engine does not hold this graph: the next use uploads the patched mirror
    dense_[0].clear();
    dense_[1].clear();
    return;
  }
  // stale rows must be refreshed against the delta they are stale for before a new patch
  // starts the next one
  for (int um = 0; um < 2; ++um)
    if (dense_[um].stale) {
      double ms = 0;
      refreshDense(um != 0, &ms);
    }
  openr_spf_patch pt{};
  pt.n_edges = (uint32_t)eids.size();
  pt.edge_ids = eids.data();
  pt.metric = emet.data();
  pt.n_links = (uint32_t)lids.size();
  pt.link_ids = lids.data();
  pt.link_up = lup.data();
  pt.n_nodes = (uint32_t)nids.size();
  pt.node_ids = nids.data();
  pt.node_overloaded = novl.data();
  SpfEngineHandle::check(openr_spf_patch_graph(engine_->ctx(), &pt), "openr_spf_patch_graph");
  ++ustats_.patches;
  for (int um = 0; um < 2; ++um) {
    if (dense_[um].src.empty()) continue;
    if (um && !m.metricsPositive) dense_[um].clear();  // pathLinks then need the exact pop order
    else dense_[um].stale = true;
  }
}

bool LinkState::denseEligible(bool useLinkMetric) const {
  return !useLinkMetric || csrMirror().metricsPositive;
}

void LinkState::refreshDense(bool useLinkMetric, double* ms) const {
  DenseRows& d = dense_[useLinkMetric ? 1 : 0];
  *ms = 0;
  if (!d.stale) return;
  d.stale = false;
  if (d.src.empty()) return;
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t resolved = 0;
  // the rows pass through the engine as u64 rows, a bounded chunk at a time (rows refresh
  // independently; the patch delta stays until the next patch)
  const uint32_t V = d.V, n = (uint32_t)d.src.size();
  const uint32_t chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(n, (64u << 20) / (8u * (size_t)std::max(V, 1u))));
  std::vector<uint64_t> stage((size_t)chunk * V);
  for (uint32_t c0 = 0; c0 < n; c0 += chunk) {
    const uint32_t k = std::min(chunk, n - c0);
    d.load(c0, k, stage.data());
    uint32_t r = 0;
    SpfEngineHandle::check(openr_spf_refresh(engine_->ctx(), d.src.data() + c0, k,
                                             useLinkMetric ? (uint32_t)OPENR_SPF_USE_LINK_METRIC : 0u, stage.data(),
                                             d.nh.data() + (size_t)c0 * V * d.nb, d.nb, nullptr, &r),
                           "openr_spf_refresh");
    d.store(c0, k, stage.data());
    resolved += r;
  }
  ++ustats_.refreshes;
  ustats_.rowsRefreshed += resolved;
  ustats_.rowsKept += d.src.size();
  *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void LinkState::prefetchKthPaths(const std::string& src, const std::vector<std::string>& dests) const {
  if (const char* e = std::getenv("OPENR_KSP2_PREFETCH"))  // 0: the call-by-call path (tests)
    if (std::atoi(e) == 0) return;
  const CsrMirror& m = csrMirror();
  if (!m.metricsPositive) return;  // the device tracer needs metrics in [1, 2^31-1]
  auto s = m.id.find(src);
  if (s == m.id.end()) return;
  const uint32_t V = (uint32_t)m.names.size();
  KspRows* rows = nullptr;
  if (auto it = kspRows_.find(src); it != kspRows_.end()) rows = &it->second;
  std::vector<uint32_t> dst;
  for (auto const& d : dests) {
    auto it = m.id.find(d);
    if (it == m.id.end() || d == src || kthPathResults_.count(std::make_tuple(src, d, size_t(2))) ||
        kthStaged_.count(std::make_pair(src, d)) || (rows && rows->off[it->second] != UINT32_MAX))
      continue;
    dst.push_back(it->second);
  }
  std::sort(dst.begin(), dst.end());
  dst.erase(std::unique(dst.begin(), dst.end()), dst.end());
  if (dst.empty()) return;
  const auto t0 = std::chrono::steady_clock::now();
  ensureEngineGraph();
  const uint32_t n = (uint32_t)dst.size(), cap = 512;  // tokens per pair: [n_paths, (len, edges..)..]
  // the engine writes every row it serves (unserved rows keep the 0xFFFFFFFF marker): no
  // zero fill, and the n x 512 token buffers persist across calls (a fresh 40 MB buffer per
  // G100 build page-faulted on the engine's copy into it)
  uint32_t* tok1 = kspScratch_.get((size_t)2 * n * cap);
  uint32_t* tok2 = tok1 + (size_t)n * cap;
  const std::vector<uint32_t> srcs(n, s->second);
  for (uint32_t i = 0; i < n; ++i) tok1[(size_t)i * cap] = tok2[(size_t)i * cap] = 0xFFFFFFFFu;
  const int rc = openr_spf_ksp2(engine_->ctx(), srcs.data(), dst.data(), n, cap, tok1, tok2);
  if (rc == OPENR_SPF_ENOTSUP) return;
  if (rc != OPENR_SPF_E2BIG) SpfEngineHandle::check(rc, "openr_spf_ksp2");  // E2BIG: overflowed rows stay unmarked
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / n;
  // staged as compact token rows on this mirror's edge ids (no Path / shared_ptr<Link>
  // per hop): k = 1 row then k = 2 row per destination
  if (!rows) {
    rows = &kspRows_[src];
    rows->src = s->second;
    rows->off.assign(V, UINT32_MAX);
    rows->memo.assign(V, 0);
  }
  rows->ms = ms;
  size_t need = rows->tok.size();
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t* r1 = &tok1[(size_t)i * cap];
    const uint32_t* r2 = &tok2[(size_t)i * cap];
    if (r1[0] != 0xFFFFFFFFu && r2[0] != 0xFFFFFFFFu) need += tokenRowLength(r1) + tokenRowLength(r2);
  }
  rows->tok.reserve(need);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t* r1 = &tok1[(size_t)i * cap];
    const uint32_t* r2 = &tok2[(size_t)i * cap];
    if (r1[0] == 0xFFFFFFFFu || r2[0] == 0xFFFFFFFFu) continue;  // overflowed: getKthPaths' own path
    rows->off[dst[i]] = (uint32_t)rows->tok.size();
    rows->tok.insert(rows->tok.end(), r1, r1 + tokenRowLength(r1));
    rows->tok.insert(rows->tok.end(), r2, r2 + tokenRowLength(r2));
    // a k = 1 entry the memo already holds is read as a memo hit
    if (kthPathResults_.count(std::make_tuple(src, m.names[dst[i]], size_t(1)))) rows->memo[dst[i]] |= 1u;
  }
}

LinkState::KspScratch::~KspScratch() { openr_spf_host_free(p); }

uint32_t* LinkState::KspScratch::get(size_t n) {
  if (cap < n) {
    openr_spf_host_free(p);
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    SpfEngineHandle::check(openr_spf_host_alloc(n * sizeof(uint32_t), &q), "openr_spf_host_alloc");
    p = static_cast<uint32_t*>(q);
    cap = n;
  }
  return p;
}

size_t LinkState::tokenRowLength(const uint32_t* row) {
  size_t at = 1;
  for (uint32_t p = 0; p < row[0]; ++p) at += 1 + row[at];
  return at;
}

void LinkState::decodeTokens(const uint32_t* row, std::vector<Path>& out) const {
  size_t at = 1;
  for (uint32_t p = 0; p < row[0]; ++p) {
    const uint32_t len = row[at++];
    Path path;
    path.reserve(len);
    for (uint32_t j = 0; j < len; ++j) path.push_back(mirror_.links[mirror_.linkId[row[at++]]]);
    out.push_back(std::move(path));
  }
}

const uint32_t* LinkState::kthPathTokens(const std::string& src, const std::string& dest, size_t k) const {
  if (k < 1 || k > 2 || kspRows_.empty() || mirrorDirty_) return nullptr;
  auto it = kspRows_.find(src);
  if (it == kspRows_.end()) return nullptr;
  auto d = mirror_.id.find(dest);
  if (d == mirror_.id.end()) return nullptr;
  KspRows& r = it->second;
  const uint32_t o = r.off[d->second];
  if (o == UINT32_MAX) return nullptr;
  const uint32_t* row1 = r.tok.data() + o;
  uint8_t& memo = r.memo[d->second];
  // getKthPaths(src, dest, 1): the first path computation reads getSpfResult(src, true)
  // (counted on its first read; the later ones are memo hits)
  auto k1 = [&]() {
    if (memo & 1u) return;
    throwIfFrozen("getKthPaths", src + "->" + dest);
    if (!r.spfRead) {
      // the memo read and its counting, without materialising the SpfResult map (the
      // token rows carry the paths)
      getSpfView(src, true);
      r.spfRead = true;  // the memo entry stays until clearMemos, which drops these rows too
    }
    memo |= 1u;
  };
  k1();
  if (k == 1) return row1;
  const uint32_t* row2 = row1 + tokenRowLength(row1);
  if (!(memo & 2u)) {  // getKthPaths(src, dest, 2): runSpf(src, true, k = 1 links) when there are any
    throwIfFrozen("getKthPaths", src + "->" + dest);
    if (row1[0] > 0) SpfCounters::get().addSpfRun(r.ms);
    memo |= 2u;
  }
  return row2;
}

bool LinkState::kthPathTokensStaged(const std::string& src, const std::vector<const std::string*>& dests) const {
  if (kspRows_.empty() || mirrorDirty_) return false;
  auto it = kspRows_.find(src);
  if (it == kspRows_.end()) return false;
  for (const std::string* d : dests) {
    auto id = mirror_.id.find(*d);
    if (id == mirror_.id.end() || it->second.off[id->second] == UINT32_MAX) return false;
  }
  return true;
}

void LinkState::convertKspRows() const {
  if (kspRows_.empty()) return;
  if (!mirrorDirty_) {
    for (auto& [src, r] : kspRows_) {
      for (uint32_t d = 0; d < r.off.size(); ++d) {
        if (r.off[d] == UINT32_MAX) continue;
        const uint32_t* row1 = r.tok.data() + r.off[d];
        const uint32_t* row2 = row1 + tokenRowLength(row1);
        const std::string& dn = mirror_.names[d];
        StagedKsp2 st;
        st.ms = r.ms;
        decodeTokens(row1, st.k1);
        decodeTokens(row2, st.k2);
        if (r.memo[d] & 1u) kthPathResults_.emplace(std::make_tuple(src, dn, size_t(1)), st.k1);
        if (r.memo[d] & 2u) kthPathResults_.emplace(std::make_tuple(src, dn, size_t(2)), std::move(st.k2));
        else kthStaged_.emplace(std::make_pair(src, dn), std::move(st));
      }
    }
  }
  kspRows_.clear();
}

const std::vector<LinkState::LabeledNode>& LinkState::labeledNodes() const {
  const CsrMirror& m = csrMirror();
  std::lock_guard<std::mutex> g(cacheMu_.m);
  if (labeledList_.gen != mirrorGeneration_ || labeledList_.adjVer != adjDbVersion_) {
    labeledList_.list.clear();
    labeledList_.list.reserve(labeledNodes_);
    for (auto const& [name, db] : adjacencyDatabases_) {
      if (db.nodeLabel == 0) continue;
      auto it = m.id.find(name);
      labeledList_.list.push_back(LabeledNode{db.nodeLabel, &db.thisNodeName, it == m.id.end() ? UINT32_MAX : it->second});
    }
    labeledList_.gen = mirrorGeneration_;
    labeledList_.adjVer = adjDbVersion_;
  }
  return labeledList_.list;
}

const std::vector<int64_t>& LinkState::nodeLabelsById() const {
  const CsrMirror& m = csrMirror();
  std::lock_guard<std::mutex> g(cacheMu_.m);
  if (nodeLabelsGen_ != mirrorGeneration_ || nodeLabelsAdjVer_ != adjDbVersion_) {
    nodeLabelsById_.assign(m.names.size(), kNoNodeLabel);
    for (uint32_t i = 0; i < m.names.size(); ++i) {
      auto it = adjacencyDatabases_.find(m.names[i]);
      if (it != adjacencyDatabases_.end()) nodeLabelsById_[i] = it->second.nodeLabel;
    }
    nodeLabelsGen_ = mirrorGeneration_;
    nodeLabelsAdjVer_ = adjDbVersion_;
  }
  return nodeLabelsById_;
}

std::vector<LinkState::SpfResult> LinkState::runSpfBatch(const std::vector<std::string>& srcs, bool useLinkMetric,
                                                         const std::vector<const LinkSet*>& ignores,
                                                         double* msOut) const {
  const auto t0 = std::chrono::steady_clock::now();
  const CsrMirror& m = csrMirror();
  std::vector<SpfResult> out(srcs.size());
  // sources unknown to the graph: the reference pops only the source itself
  std::vector<uint32_t> ids;
  std::vector<size_t> slot;
  for (size_t i = 0; i < srcs.size(); ++i) {
    auto it = m.id.find(srcs[i]);
    if (it == m.id.end()) {
      out[i].emplace(srcs[i], NodeSpfResult(0));
    } else {
      ids.push_back(it->second);
      slot.push_back(i);
    }
  }
  if (!ids.empty()) {
    ensureEngineGraph();
    const uint32_t V = (uint32_t)m.names.size(), E = (uint32_t)m.col.size(), tw = (E + 63) / 64;
    uint32_t nb = 1;
    SpfEngineHandle::check(openr_spf_nh_bytes(engine_->ctx(), &nb), "openr_spf_nh_bytes");
    const size_t n = ids.size();
    std::vector<uint64_t> dist(n * V), tight(n * std::max<uint32_t>(tw, 1));
    std::vector<uint8_t> nh(n * V * nb);
    const uint32_t flags = (useLinkMetric ? (uint32_t)OPENR_SPF_USE_LINK_METRIC : 0u) | (uint32_t)OPENR_SPF_EMIT_TIGHT;
    // zero / wrapped metrics: pop order is history-dependent, take it from the exact kernel
    const bool wantOrder = useLinkMetric && !m.metricsPositive;
    std::vector<uint32_t> popIndex(wantOrder ? n * V : 0);
    bool anyIgnore = false;
    for (size_t k = 0; k < n; ++k) anyIgnore |= ignores[slot[k]] && !ignores[slot[k]]->empty();
    std::vector<uint32_t> ptr, links;
    if (anyIgnore) {
      const auto& lid = m.linkIndex;
      ptr.assign(n + 1, 0);
      for (size_t k = 0; k < n; ++k) {
        if (const LinkSet* ign = ignores[slot[k]]) {
          for (auto const& link : *ign) {
            // match by link identity (LinkPtrEqual), not pointer
            for (auto const& cand : linksFromNode(link->firstNodeName())) {
              if (*cand == *link) {
                auto f = lid.find(cand.get());
                if (f != lid.end()) links.push_back(f->second);
                break;
              }
            }
          }
        }
        ptr[k + 1] = (uint32_t)links.size();
      }
      if (links.empty()) links.push_back(0);
    }
    if (wantOrder) {
      SpfEngineHandle::check(openr_spf_solve_order(engine_->ctx(), ids.data(), (uint32_t)n, flags,
                                                   anyIgnore ? ptr.data() : nullptr, anyIgnore ? links.data() : nullptr,
                                                   dist.data(), nh.data(), nb, tight.data(), popIndex.data()),
                             "openr_spf_solve_order");
    } else if (anyIgnore) {
      SpfEngineHandle::check(openr_spf_solve_ignore(engine_->ctx(), ids.data(), (uint32_t)n, flags, ptr.data(),
                                                    links.data(), dist.data(), nh.data(), nb, tight.data()),
                             "openr_spf_solve_ignore");
    } else {
      SpfEngineHandle::check(
          openr_spf_solve(engine_->ctx(), ids.data(), (uint32_t)n, flags, dist.data(), nh.data(), nb, tight.data()),
          "openr_spf_solve");
    }
    // materialise SpfResult: nextHops from the bitsets, pathLinks from tight edges
    // ordered by the predecessor's settle order ((dist, name), or the exact kernel's pop
    // index) then row position. Sources are independent: one host worker each.
    const unsigned workers = parallelWorkers(n, 8);
    std::vector<std::vector<uint32_t>> nbrsW(workers, std::vector<uint32_t>(V ? V : 1)), orderW(workers);
    parallelFor(n, 8, workers, [&](unsigned w, size_t k) {
      auto& nbrs = nbrsW[w];
      auto& order = orderW[w];
      const uint32_t src = ids[k];
      uint32_t nn = 0;
      SpfEngineHandle::check(openr_spf_neighbor_map(engine_->ctx(), src, nbrs.data(), (uint32_t)nbrs.size(), &nn),
                             "openr_spf_neighbor_map");
      const uint64_t* d = dist.data() + k * V;
      const uint8_t* h = nh.data() + k * (size_t)V * nb;
      const uint64_t* t = tight.data() + k * (size_t)std::max<uint32_t>(tw, 1);
      SpfResult& res = out[slot[k]];
      res.reserve(V);
      const uint32_t* pop = wantOrder ? popIndex.data() + k * V : nullptr;
      for (uint32_t v = 0; v < V; ++v) {
        // reached: popped (a wrapped sum can equal UINT64_MAX), else a finite distance
        if (pop ? pop[v] == UINT32_MAX : d[v] == UINT64_MAX) continue;
        NodeSpfResult r(d[v]);
        const uint8_t* hv = h + (size_t)v * nb;
        for (uint32_t i = 0; i < nn; ++i)
          if ((hv[i >> 3] >> (i & 7)) & 1u) r.addNextHop(m.names[nbrs[i]]);
        res.emplace(m.names[v], std::move(r));
      }
      order.clear();
      for (uint32_t e = 0; e < E; ++e)
        if ((t[e >> 6] >> (e & 63)) & 1ull) order.push_back(e);
      std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        const uint32_t ux = m.edgeOwner[x], uy = m.edgeOwner[y];
        if (pop) return pop[ux] != pop[uy] ? pop[ux] < pop[uy] : x < y;
        if (d[ux] != d[uy]) return d[ux] < d[uy];
        if (m.nameRank[ux] != m.nameRank[uy]) return m.nameRank[ux] < m.nameRank[uy];
        return x < y;
      });
      for (uint32_t e : order) {
        const uint32_t u = m.edgeOwner[e], v = m.col[e];
        res.at(m.names[v]).addPath(m.links[m.linkId[e]], m.names[u]);
      }
    });
  }
  *msOut = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return out;
}

LinkState::SpfResult LinkState::runSpf(const std::string& src, bool useLinkMetric, const LinkSet& linksToIgnore) const {
  double ms = 0;
  auto v = runSpfBatch({src}, useLinkMetric, {&linksToIgnore}, &ms);
  SpfCounters::get().addSpfRun(ms);  // decision.spf_runs counts logical SPFs (LinkState.cpp:815, :880)
  return std::move(v[0]);
}

}  // namespace openr
