// LinkState.h — C++ host mirror of openr::LinkState with the SPF on the GPU engine.
//
// Public surface and semantics follow /root/reference/openr/decision/LinkState.h
// (HoldableValue :36-58, Link :82-175, LinkState :177-469) so that Decision's callers
// (SpfSolver, Decision.cpp) compile against it unchanged. What differs is below the
// surface: LinkState::runSpf (reference LinkState.cpp:808-882) is a call through the
// C-ABI in include/openr_spf.h on a CSR mirror of linkMap_, and results are
// materialised from the engine's dense outputs (distances, next-hop bitsets,
// tight-edge mask). There is no CPU Dijkstra here.
//
// Thrift types: this standalone build carries minimal structs with the fields of
// openr/if/Lsdb.thrift:71-129 (Adjacency, AdjacencyDatabase) and Network.thrift
// BinaryAddress. In the real tree the generated types replace them.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <tuple>
#include <utility>
#include <vector>

namespace openr {
// folly::hash::hash_128_to_64 (CityHash Hash128to64), folly rev 1540c39c.
inline uint64_t hash_128_to_64(uint64_t upper, uint64_t lower) {
  const uint64_t kMul = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * kMul;
  a ^= (a >> 47);
  uint64_t b = (upper ^ a) * kMul;
  b ^= (b >> 47);
  b *= kMul;
  return b;
}
}  // namespace openr

namespace std {
// folly provides these for the reference (folly/hash/Hash.h): hash_combine of the
// element hashes. Link::hash, and with it linksFromNode() iteration order, depend on it.
template <class A, class B>
struct hash<pair<A, B>> {
  size_t operator()(const pair<A, B>& p) const {
    return openr::hash_128_to_64(std::hash<A>()(p.first), std::hash<B>()(p.second));
  }
};
template <class... T>
struct hash<tuple<T...>> {
  size_t operator()(const tuple<T...>& t) const {
    size_t h = 0;
    bool first = true;
    std::apply(
        [&](const auto&... e) {
          ((h = first ? (first = false, std::hash<std::decay_t<decltype(e)>>()(e))
                      : openr::hash_128_to_64(h, std::hash<std::decay_t<decltype(e)>>()(e))),
           ...);
        },
        t);
    return h;
  }
};
}  // namespace std

namespace openr {

using LinkStateMetric = uint64_t;

namespace thrift {
struct BinaryAddress {
  std::string addr;
  std::optional<std::string> ifName;
  bool operator==(const BinaryAddress& o) const { return addr == o.addr && ifName == o.ifName; }
  bool operator!=(const BinaryAddress& o) const { return !(*this == o); }
};

struct Adjacency {
  std::string otherNodeName;
  std::string ifName;
  BinaryAddress nextHopV6;
  BinaryAddress nextHopV4;
  int32_t metric = 0;
  int32_t adjLabel = 0;
  bool isOverloaded = false;
  int32_t rtt = 0;
  int64_t timestamp = 0;
  int64_t weight = 1;
  std::string otherIfName;
};

// Lsdb.thrift:24-32
struct PerfEvent {
  std::string nodeName;
  std::string eventDescr;
  int64_t unixTs = 0;
};
struct PerfEvents {
  std::vector<PerfEvent> events;
};

struct AdjacencyDatabase {
  std::string thisNodeName;
  bool isOverloaded = false;
  std::vector<Adjacency> adjacencies;
  int32_t nodeLabel = 0;
  std::optional<PerfEvents> perfEvents;
  std::string area;
};
}  // namespace thrift

// fb303-style counters of the SPF path: decision.spf_runs (COUNT) and decision.spf_ms
// (AVG), as recorded by the reference at LinkState.cpp:815 and :880.
// Thread-safe: route builds of many nodes run on host worker threads (SpfSolver::buildRouteDbs).
struct SpfCounters {
  static SpfCounters& get();
  void addSpfRun(double ms, uint64_t runs = 1);
  void reset();
  uint64_t spfRuns() const;
  double spfMsAvg() const;

 private:
  mutable std::mutex mu_;
  uint64_t runs_ = 0, samples_ = 0;
  double msSum_ = 0.0;
};

// A flag that copies / moves by value (so structs holding it stay movable)
struct RelaxedFlag {
  std::atomic<int> v{0};
  RelaxedFlag() = default;
  RelaxedFlag(const RelaxedFlag& o) : v(o.v.load(std::memory_order_relaxed)) {}
  RelaxedFlag& operator=(const RelaxedFlag& o) {
    v.store(o.v.load(std::memory_order_relaxed), std::memory_order_relaxed);
    return *this;
  }
};

// A mutex that copies / moves as a fresh one (caches of a copyable object)
struct CacheMutex {
  mutable std::mutex m;
  CacheMutex() = default;
  CacheMutex(const CacheMutex&) {}
  CacheMutex& operator=(const CacheMutex&) { return *this; }
};

template <class T>
class HoldableValue {
 public:
  explicit HoldableValue(T val);
  void operator=(T val);
  const T& value() const;
  bool hasHold() const;
  // return true if the call changed value()
  bool decrementTtl();
  bool updateValue(T val, LinkStateMetric holdUpTtl, LinkStateMetric holdDownTtl);

 private:
  bool isChangeBringingUp(T val) const;
  T val_;
  std::optional<T> heldVal_;
  LinkStateMetric holdTtl_{0};
};

class Link {
 public:
  Link(const std::string& area, const std::string& nodeName1, const std::string& if1,
       const std::string& nodeName2, const std::string& if2);
  Link(const std::string& area, const std::string& nodeName1, const thrift::Adjacency& adj1,
       const std::string& nodeName2, const thrift::Adjacency& adj2);

 private:
  // one end of the link, as advertised by that end's node
  struct End {
    std::string node, iface;
    HoldableValue<LinkStateMetric> metric{1};
    HoldableValue<bool> overload{false};
    int32_t adjLabel{0};
    thrift::BinaryAddress nhV4, nhV6;
  };
  const std::string area_;
  End ends_[2];
  LinkStateMetric holdUpTtl_{0};
  const std::pair<std::pair<std::string, std::string>, std::pair<std::string, std::string>> orderedNames_;

  int sideOf(const std::string& nodeName) const;  // throws std::invalid_argument

 public:
  const size_t hash{0};

  void setHoldUpTtl(LinkStateMetric ttl);
  bool isUp() const;
  bool decrementHolds();
  bool hasHolds() const;
  const std::string& getArea() const { return area_; }
  const std::string& getOtherNodeName(const std::string& nodeName) const;
  const std::string& firstNodeName() const;
  const std::string& secondNodeName() const;
  const std::string& getIfaceFromNode(const std::string& nodeName) const;
  LinkStateMetric getMetricFromNode(const std::string& nodeName) const;
  int32_t getAdjLabelFromNode(const std::string& nodeName) const;
  bool getOverloadFromNode(const std::string& nodeName) const;
  const thrift::BinaryAddress& getNhV4FromNode(const std::string& nodeName) const;
  const thrift::BinaryAddress& getNhV6FromNode(const std::string& nodeName) const;
  void setNhV4FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV4);
  void setNhV6FromNode(const std::string& nodeName, const thrift::BinaryAddress& nhV6);
  bool setMetricFromNode(const std::string& nodeName, LinkStateMetric d, LinkStateMetric holdUpTtl,
                         LinkStateMetric holdDownTtl);
  void setAdjLabelFromNode(const std::string& nodeName, int32_t adjLabel);
  bool setOverloadFromNode(const std::string& nodeName, bool overload, LinkStateMetric holdUpTtl,
                           LinkStateMetric holdDownTtl);
  bool operator<(const Link& other) const;
  bool operator==(const Link& other) const;
  std::string toString() const;
  std::string directionalToString(const std::string& fromNode) const;
};

class SpfEngineHandle;  // RAII owner of an openr_spf_ctx (LinkState.cpp)

class LinkState {
 public:
  explicit LinkState(const std::string& area);

  struct LinkPtrHash {
    size_t operator()(const std::shared_ptr<Link>& l) const;
  };
  struct LinkPtrLess {
    bool operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const;
  };
  struct LinkPtrEqual {
    bool operator()(const std::shared_ptr<Link>& lhs, const std::shared_ptr<Link>& rhs) const;
  };
  using LinkSet = std::unordered_set<std::shared_ptr<Link>, LinkPtrHash, LinkPtrEqual>;

  class NodeSpfResult {
   public:
    class PathLink {
     public:
      PathLink(std::shared_ptr<Link> const& l, std::string const& n) : link(l), prevNode(n) {}
      std::shared_ptr<Link> const link;
      std::string const prevNode;
    };
    explicit NodeSpfResult(LinkStateMetric m) : metric_(m) {}
    void reset(LinkStateMetric newMetric) {
      metric_ = newMetric;
      pathLinks_.clear();
      nextHops_.clear();
    }
    std::vector<PathLink> const& pathLinks() const { return pathLinks_; }
    std::unordered_set<std::string> const& nextHops() const { return nextHops_; }
    LinkStateMetric metric() const { return metric_; }
    void addPath(std::shared_ptr<Link> const& link, std::string const& prevNode) {
      pathLinks_.emplace_back(link, prevNode);
    }
    void addNextHops(std::unordered_set<std::string> const& toInsert) {
      nextHops_.insert(toInsert.begin(), toInsert.end());
    }
    void addNextHop(std::string const& toInsert) { nextHops_.insert(toInsert); }

   private:
    LinkStateMetric metric_{std::numeric_limits<LinkStateMetric>::max()};
    std::vector<PathLink> pathLinks_;
    std::unordered_set<std::string> nextHops_;
  };

  using SpfResult = std::unordered_map<std::string, NodeSpfResult>;
  using Path = std::vector<std::shared_ptr<Link>>;

  // memoized per (node, useLinkMetric) until the next topology change
  SpfResult const& getSpfResult(const std::string& nodeName, bool useLinkMetric = true) const;

  // Batched prefetch (new): one engine launch fills the memo for every node in
  // `nodes` (e.g. me + neighbours for LFA, or all nodes for all-sources route build).
  // A prefetched result counts as an SPF run (decision.spf_runs / spf_ms) when it is first
  // read, where the reference's memo miss would have run it: counters do not depend on
  // what was prefetched, nor on how many threads read.
  void prefetchSpfResults(const std::vector<std::string>& nodes, bool useLinkMetric = true) const;

  // While a MemoFreeze is alive the SPF memos are read-only: several threads may read
  // results the prefetch covered (getSpfResult / getKthPaths), and a read the prefetch did
  // not cover throws std::logic_error instead of solving and inserting concurrently.
  class MemoFreeze {
   public:
    explicit MemoFreeze(const LinkState& ls) : ls_(ls) { ls_.frozen_.v.fetch_add(1); }
    ~MemoFreeze() { ls_.frozen_.v.fetch_sub(1); }
    MemoFreeze(const MemoFreeze&) = delete;
    MemoFreeze& operator=(const MemoFreeze&) = delete;

   private:
    const LinkState& ls_;
  };

  std::vector<LinkState::Path> const& getKthPaths(const std::string& src, const std::string& dest,
                                                  size_t k) const;

  // Batched KSP2 prefetch (new): getKthPaths(src, d, 1) and (src, d, 2) for every d in
  // `dests`, traced on the device in one openr_spf_ksp2 launch instead of one ignore-set
  // SPF per destination. Results are staged, not memoised: a later getKthPaths(src, d, k)
  // takes its staged paths and records the logical SPF run the reference would have made
  // then, so memo contents and decision.spf_runs match the call-by-call sequence however
  // many destinations were prefetched. Graphs the device tracer refuses (a metric outside
  // [1, 2^31-1], too many links) and pairs whose paths overflow the token rows are left to
  // getKthPaths' own path.
  void prefetchKthPaths(const std::string& src, const std::vector<std::string>& dests) const;

  // Route-build form of getKthPaths (round 5): the k-th paths of (src, dest) as a token row
  // of the current mirror's edge ids, [n_paths, (len, e_1 .. e_len) ..] with e_1 leaving
  // src, for a pair prefetchKthPaths staged. It has exactly the memo and counter effects of
  // getKthPaths(src, dest, k) (k = 1, 2) without building Path vectors of shared_ptr<Link>;
  // a later getKthPaths of the pair materialises the paths as a memo hit. Null when the
  // pair is not staged (the caller takes getKthPaths).
  const uint32_t* kthPathTokens(const std::string& src, const std::string& dest, size_t k) const;
  // true when kthPathTokens(src, d, 1 and 2) serves every d in `dests` (a pure test)
  bool kthPathTokensStaged(const std::string& src, const std::vector<const std::string*>& dests) const;
  // nodeLabel of each mirror node id (its adjacency database's; kNoNodeLabel without one)
  static constexpr int64_t kNoNodeLabel = INT64_MIN;
  const std::vector<int64_t>& nodeLabelsById() const;

  class LinkStateChange {
   public:
    LinkStateChange() = default;
    LinkStateChange(bool topo, bool link, bool node)
        : topologyChanged(topo), linkAttributesChanged(link), nodeLabelChanged(node) {}
    bool operator==(LinkStateChange const& other) const {
      return topologyChanged == other.topologyChanged && linkAttributesChanged == other.linkAttributesChanged &&
             nodeLabelChanged == other.nodeLabelChanged;
    }
    bool topologyChanged{false};
    bool linkAttributesChanged{false};
    bool nodeLabelChanged{false};
  };

  LinkStateChange decrementHolds();
  LinkStateChange updateAdjacencyDatabase(thrift::AdjacencyDatabase const& adjacencyDb,
                                          LinkStateMetric holdUpTtl = 0, LinkStateMetric holdDownTtl = 0);
  // same, taking ownership of a database the caller no longer needs (bulk loads: no copy)
  LinkStateChange updateAdjacencyDatabase(thrift::AdjacencyDatabase&& adjacencyDb, LinkStateMetric holdUpTtl = 0,
                                          LinkStateMetric holdDownTtl = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& nodeName);

  std::optional<LinkStateMetric> getMetricFromAToB(std::string const& a, std::string const& b,
                                                   bool useLinkMetric = true) const;
  std::optional<LinkStateMetric> getHopsFromAToB(std::string const& a, std::string const& b) const {
    return getMetricFromAToB(a, b, false);
  }
  LinkStateMetric getMaxHopsToNode(const std::string& nodeName) const;
  const std::string& getArea() const { return area_; }
  bool hasNode(const std::string& nodeName) const { return adjacencyDatabases_.count(nodeName) != 0; }
  const LinkSet& linksFromNode(const std::string& nodeName) const;
  bool isNodeOverloaded(const std::string& nodeName) const;
  bool hasHolds() const;
  size_t numLinks() const { return allLinks_.size(); }
  size_t numNodes() const { return linkMap_.size(); }
  // adjacency databases that carry a node label (new: lets a route build skip the
  // node-label pass, and the SPFs it would read, when there are none)
  size_t labeledNodeCount() const { return labeledNodes_; }
  // The adjacency databases with a node label, in getAdjacencyDatabases() iteration order
  // (the order buildRouteDb visits them, which decides label collisions), with each node's
  // id on the current mirror: the node-label route pass walks this list instead of hashing
  // every name per build. Rebuilt after an adjacency database update or a mirror rebuild.
  struct LabeledNode {
    int32_t label;
    const std::string* name;  // the adjacency database's thisNodeName
    uint32_t id;              // csrMirror().id of the node (UINT32_MAX: not on the mirror)
  };
  const std::vector<LabeledNode>& labeledNodes() const;
  std::unordered_map<std::string, thrift::AdjacencyDatabase> const& getAdjacencyDatabases() const {
    return adjacencyDatabases_;
  }
  static bool pathAInPathB(Path const& a, Path const& b);

  // --- engine mirror (introspection for tests and benchmarks) ---------------
  struct CsrMirror {
    std::vector<std::string> names;  // sorted: id == rank under std::string operator<
    std::unordered_map<std::string, uint32_t> id;
    std::vector<uint32_t> rowPtr, col, linkId;
    std::vector<uint64_t> metric;
    std::vector<uint8_t> edgeUp, overloaded;
    std::vector<uint32_t> nameRank;
    std::vector<std::shared_ptr<Link>> links;  // link id -> Link
    std::vector<uint32_t> linkEdges;           // link id -> its two directed edge ids (2 per link)
    std::vector<uint32_t> edgeOwner;
    std::unordered_map<const Link*, uint32_t> linkIndex;  // Link -> link id (ignore sets)
    bool metricsPositive = true;  // every usable metric in [1, 2^31-1]: fast kernels
    uint64_t generation = 0;      // process-wide id of this mirror build (kept by a retired snapshot)
  };
  const CsrMirror& csrMirror() const;
  // process-wide id of the mirror csrMirror() last built (tests: a rebuild changes it)
  uint64_t mirrorGeneration() const { return mirrorGeneration_; }

  // Dense view of a memoised SPF (route build fast path, round 3): the same result
  // getSpfResult(node, useLinkMetric) holds — reached nodes, metrics, next hops — read from
  // the memo's dense rows without materialising the SpfResult map. Counts the SPF run like
  // getSpfResult (first read of the memo entry). The view resolves its row on every access,
  // so later SPF reads and prefetches (which grow the dense rows) leave it valid; like the
  // reference's SpfResult reference, it is invalidated by the next adjacency / overload
  // update of the LinkState (updateAdjacencyDatabase, deleteAdjacencyDatabase, decrementHolds).
  class SpfView {
   public:
    bool reached(const std::string& node) const;
    // metric of a reached node (std::out_of_range otherwise, like SpfResult::at)
    LinkStateMetric metric(const std::string& node) const;
    // next hops of a reached node (std::out_of_range otherwise)
    std::vector<std::string> nextHops(const std::string& node) const;
    // f(next-hop name, distance to that next hop) for each next hop of a reached node
    // (std::out_of_range otherwise): nextHops + metric(nh) without building names
    template <class F>
    void forEachNextHop(const std::string& node, F&& f) const;
    // Dense internals for id-based readers (the route build's fast path): mirror() is null
    // when the entry is map-backed; ids index mirror()->names. dist(v) = the metric of v
    // (UINT64_MAX: not reached), nhRow()[v * nhBytes() ..] its next-hop bits, bit i = node
    // nhNeighbours()[i].
    const CsrMirror* mirror() const { return map_ ? nullptr : m_; }
    inline uint64_t dist(uint32_t v) const;
    const uint8_t* nhRow() const { return nh(0); }
    uint32_t nhBytes() const;
    const std::vector<uint32_t>& nhNeighbours() const;

   private:
    friend class LinkState;
    // the materialised SpfResult when the memo entry has no dense row (unknown source,
    // zero / wrapped metrics): then every call reads it
    const SpfResult* map_ = nullptr;
    const CsrMirror* m_ = nullptr;
    const void* rows_ = nullptr;  // the DenseRows holding row_ (resolved per access)
    uint32_t row_ = 0;
    std::shared_ptr<const void> keep_;  // a retired row snapshot the view reads (see RowSnapshot)
    const uint8_t* nh(uint32_t v) const;
    int32_t id(const std::string& node) const;
  };
  SpfView getSpfView(const std::string& nodeName, bool useLinkMetric = true) const;

  // Incremental-update introspection (tests / benchmarks): attribute-only topology changes
  // patch the engine's resident graph (openr_spf_patch_graph) and refresh the memo's dense
  // rows (openr_spf_refresh) instead of re-uploading the graph and re-solving every row.
  struct UpdateStats {
    uint64_t graphUploads = 0;  // openr_spf_set_graph calls
    uint64_t patches = 0;       // openr_spf_patch_graph calls
    uint64_t refreshes = 0;     // openr_spf_refresh calls
    uint64_t rowsRefreshed = 0; // rows those refreshes re-solved
    uint64_t rowsKept = 0;      // dense rows carried across a change (not re-solved)
    uint64_t rowsRetired = 0;   // dense rows a mirror rebuild kept in snapshots for live memo entries
  };
  const UpdateStats& updateStats() const { return ustats_; }
  size_t denseRows(bool useLinkMetric = true) const { return dense_[useLinkMetric ? 1 : 0].src.size(); }

 private:
  const std::string area_;
  // memo entry: the result, and whether its logical SPF run has been counted (a prefetched
  // entry is counted on its first read, with its share of the batch's time)
  // A once-flag that copies as a fresh flag (memo entries stay copyable)
  struct LazyOnce {
    std::unique_ptr<std::once_flag> f = std::make_unique<std::once_flag>();
    LazyOnce() = default;
    LazyOnce(const LazyOnce&) : f(std::make_unique<std::once_flag>()) {}
    LazyOnce& operator=(const LazyOnce&) {
      f = std::make_unique<std::once_flag>();
      return *this;
    }
  };
  struct RowSnapshot;
  struct MemoEntry {
    SpfResult res;
    RelaxedFlag counted;
    double ms = 0;
    uint32_t row = UINT32_MAX;  // dense row of the result (materialised into res on first read), or none
    // the mirror + rows `row` indexes when a rebuild of the mirror retired them (null: the
    // live mirror_ / dense_)
    std::shared_ptr<const RowSnapshot> snap;
    LazyOnce once;
  };
  // Dense memo rows per useLinkMetric (round 3): the results the memo holds as the engine
  // writes them — distance and next-hop bitset per (source, node) — host-resident. They
  // outlive attribute-only topology changes (refreshed in place after the engine graph is
  // patched) and are materialised into SpfResult maps only when read.
  // Distances are kept as u32 (UINT32_MAX = not reached) while every finite one fits, else
  // as u64 (round 4: G100's 10 000 rows in 500 instead of 900 MB); the engine's u64 rows
  // pass through a bounded staging buffer.
  struct DenseRows {
    uint32_t nb = 1;
    uint32_t V = 0;
    std::unordered_map<uint32_t, uint32_t> slot;  // node id -> row
    std::vector<uint32_t> src;                     // row -> node id
    bool wide = false;                             // distances in dist64 (else dist32)
    std::vector<uint32_t> dist32;                  // rows x V
    std::vector<uint64_t> dist64;                  // rows x V
    std::vector<uint8_t> nh;                       // rows x V x nb
    std::vector<std::vector<uint32_t>> nbrs;       // row -> node id of next-hop bit i
    bool stale = false;                            // rows predate a patch: refresh before any read
    void clear() { *this = DenseRows{}; }
    uint64_t dist(size_t row, uint32_t v) const {
      const size_t i = row * V + v;
      if (wide) return dist64[i];
      const uint32_t x = dist32[i];
      return x == UINT32_MAX ? UINT64_MAX : (uint64_t)x;
    }
    // rows [r0, r0 + n) from engine u64 rows (widens every row first when one does not fit)
    void store(size_t r0, size_t n, const uint64_t* rows);
    // rows [r0, r0 + n) as engine u64 rows
    void load(size_t r0, size_t n, uint64_t* rows) const;
    void resizeRows(size_t rows);
  };
  mutable DenseRows dense_[2];
  // A structural change that the reference does not count as a topology change (a node's
  // first adjacency database, a link that is added or removed while not up) keeps the memo
  // (LinkState.cpp:714-717 clear it only on topologyChanged) but rebuilds the mirror, whose
  // node ids the dense rows are indexed by. The memo entries that point at rows then move,
  // with those rows and the mirror they were solved on, into a shared snapshot.
  struct RowSnapshot {
    CsrMirror mirror;
    DenseRows rows[2];
  };
  void retireDenseRows();
  mutable UpdateStats ustats_;
  bool denseEligible(bool useLinkMetric) const;
  void refreshDense(bool useLinkMetric, double* ms) const;
  const SpfResult& materialize(const MemoEntry& e, bool useLinkMetric) const;
  // attribute-only change: patch the mirror and the engine's graph in place
  void applyAttrPatch(const std::vector<std::shared_ptr<Link>>& links, const std::vector<std::string>& nodes);
  std::vector<std::shared_ptr<Link>> attrLinks_;  // links / nodes an update changed (attributes only)
  std::vector<std::string> attrNodes_;
  mutable std::unordered_map<std::pair<std::string, bool>, MemoEntry> spfResults_;
  mutable RelaxedFlag frozen_;  // MemoFreeze depth
  void throwIfFrozen(const char* what, const std::string& key) const;
  mutable std::unordered_map<std::tuple<std::string, std::string, size_t>, std::vector<LinkState::Path>>
      kthPathResults_;
  size_t labeledNodes_ = 0;  // adjacency databases with nodeLabel != 0
  struct StagedKsp2 {
    std::vector<Path> k1, k2;
    double ms = 0;  // this pair's share of the launch (decision.spf_ms)
  };
  mutable std::unordered_map<std::pair<std::string, std::string>, StagedKsp2> kthStaged_;
  // Device-traced k = 1 / 2 paths of one source as edge-id token rows of mirror_ (round 5):
  // what prefetchKthPaths stages, per destination id. `memo` bit k-1: the (src, d, k) entry
  // exists in the reference's kthPathResults_ (read, counted). A mirror rebuild converts the
  // rows into kthStaged_ / kthPathResults_ first (their edge ids die with the mirror).
  struct KspRows {
    uint32_t src = UINT32_MAX;
    double ms = 0;                  // per pair share of the launch (decision.spf_ms)
    std::vector<uint32_t> off;      // per dst id: offset of its k = 1 row in tok (k = 2 row follows), or UINT32_MAX
    std::vector<uint8_t> memo;
    std::vector<uint32_t> tok;
    bool spfRead = false;           // getSpfResult(src) read through this object (k = 1 counting)
  };
  mutable std::unordered_map<std::string, KspRows> kspRows_;
  // prefetchKthPaths' engine token buffers: page-locked (openr_spf_host_alloc), reused
  // across calls; a copy of the LinkState starts without one
  struct KspScratch {
    uint32_t* p = nullptr;
    size_t cap = 0;
    KspScratch() = default;
    KspScratch(const KspScratch&) {}
    KspScratch& operator=(const KspScratch&) { return *this; }
    KspScratch(KspScratch&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr, o.cap = 0; }
    KspScratch& operator=(KspScratch&& o) noexcept {
      std::swap(p, o.p);
      std::swap(cap, o.cap);
      return *this;
    }
    ~KspScratch();
    uint32_t* get(size_t n);
  };
  mutable KspScratch kspScratch_;
  static size_t tokenRowLength(const uint32_t* row);
  void decodeTokens(const uint32_t* row, std::vector<Path>& out) const;  // mirror_'s edge ids -> Links
  void convertKspRows() const;  // kspRows_ -> kthStaged_ / kthPathResults_ (mirror_ still valid)
  // id-indexed caches read by concurrent route builds (buildRouteDbs workers): the first
  // reader after a change rebuilds under the lock; no update runs during a build
  CacheMutex cacheMu_;
  // labeledList_ points into this object's adjacencyDatabases_: a copy starts empty with
  // stamps that never match, so it rebuilds against its own databases (a move keeps the
  // map's nodes, and the pointers with them)
  struct LabeledListCache {
    std::vector<LabeledNode> list;
    uint64_t gen = 0, adjVer = ~0ull;
    LabeledListCache() = default;
    LabeledListCache(const LabeledListCache&) {}
    LabeledListCache& operator=(const LabeledListCache&) {
      list.clear();
      gen = 0;
      adjVer = ~0ull;
      return *this;
    }
    LabeledListCache(LabeledListCache&&) noexcept = default;
    LabeledListCache& operator=(LabeledListCache&&) noexcept = default;
  };
  mutable LabeledListCache labeledList_;
  mutable std::vector<int64_t> nodeLabelsById_;
  mutable uint64_t nodeLabelsGen_ = 0, nodeLabelsAdjVer_ = 0;
  uint64_t adjDbVersion_ = 0;  // bumped by every adjacency database update / delete
  void clearMemos() const {
    spfResults_.clear();
    kthPathResults_.clear();
    kthStaged_.clear();
    kspRows_.clear();
  }
  void ensureEngineGraph() const;

  std::optional<Path> traceOnePath(std::string const& src, std::string const& dest, SpfResult const& result,
                                   LinkSet& linksToIgnore) const;
  void addLink(std::shared_ptr<Link> link);
  void removeLink(std::shared_ptr<Link> link);
  void removeNode(const std::string& nodeName);
  bool updateNodeOverloaded(const std::string& nodeName, bool isOverloaded, LinkStateMetric holdUpTtl,
                            LinkStateMetric holdDownTtl);
  // one logical SPF (counted in decision.spf_runs)
  SpfResult runSpf(const std::string& src, bool useLinkMetric, const LinkSet& linksToIgnore = {}) const;
  // a batch of SPFs, NOT counted (callers count when the reference would); *ms = wall time
  std::vector<SpfResult> runSpfBatch(const std::vector<std::string>& srcs, bool useLinkMetric,
                                     const std::vector<const LinkSet*>& ignores, double* ms) const;
  std::shared_ptr<Link> maybeMakeLink(const std::string& nodeName, const thrift::Adjacency& adj) const;
  std::vector<std::shared_ptr<Link>> getOrderedLinkSet(const thrift::AdjacencyDatabase& adjDb) const;
  std::vector<std::shared_ptr<Link>> orderedLinksFromNode(const std::string& nodeName) const;
  void markMirrorDirty() {
    convertKspRows();   // edge ids change with the rebuilt mirror
    retireDenseRows();  // node ids change with the rebuilt mirror
    mirrorDirty_ = true;
    dense_[0].clear();
    dense_[1].clear();
  }

  std::unordered_map<std::string, LinkSet> linkMap_;
  LinkSet allLinks_;
  std::unordered_map<std::string, HoldableValue<bool>> nodeOverloads_;
  std::unordered_map<std::string, thrift::AdjacencyDatabase> adjacencyDatabases_;
  // per node: ifName -> positions in its adjacency list (increasing), so maybeMakeLink
  // finds the reverse adjacency without scanning the other node's whole list
  std::unordered_map<std::string, std::unordered_map<std::string, std::vector<uint32_t>>> ifIndex_;
  void indexAdjacencies(const std::string& nodeName);

  mutable CsrMirror mirror_;
  mutable bool mirrorDirty_ = true;
  mutable uint64_t mirrorGeneration_ = 0;
  mutable std::shared_ptr<SpfEngineHandle> engine_;
};

template <class F>
void LinkState::SpfView::forEachNextHop(const std::string& node, F&& f) const {
  if (map_) {
    for (auto const& nh : map_->at(node).nextHops()) f(nh, map_->at(nh).metric());
    return;
  }
  const int32_t v = id(node);
  if (v < 0) throw std::out_of_range("SpfView::forEachNextHop: " + node + " not reached");
  const DenseRows& d = *static_cast<const DenseRows*>(rows_);
  const uint8_t* hv = nh((uint32_t)v);
  const std::vector<uint32_t>& nbrs = d.nbrs[row_];
  for (uint32_t i = 0; i < nbrs.size(); ++i)
    if ((hv[i >> 3] >> (i & 7)) & 1u) f(m_->names[nbrs[i]], d.dist(row_, nbrs[i]));
}

inline uint64_t LinkState::SpfView::dist(uint32_t v) const {
  return static_cast<const DenseRows*>(rows_)->dist(row_, v);
}

}  // namespace openr

namespace std {
template <>
struct hash<openr::Link> {
  size_t operator()(openr::Link const& link) const { return link.hash; }
};
}  // namespace std
