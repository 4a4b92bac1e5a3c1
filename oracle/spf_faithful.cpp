// spf_faithful.cpp — CPU BASELINE (test / benchmark infrastructure only), "faithful cost".
//
// The dense-id oracle (spf_oracle.c) restates LinkState::runSpf's *semantics* on integer
// ids; it is ~350x cheaper per core than the reference because the reference's time goes
// to its data structures, not arithmetic (SURVEY.md §6 gprof: std::string-keyed hash
// lookups, Link::getOtherNodeName string compares, shared_ptr heap nodes, per-node
// unordered_set<std::string> next-hop copies). This file restates runSpf with THOSE data
// structure choices so bench.py can time a reference-cost CPU baseline (SURVEY.md §7.1
// step 2, §8d) without building the reference (its fbthrift / folly / fb303 deps are
// absent here). Each piece cites what it stands in for:
//   FLink                 Link (LinkState.h:82-175): node / interface names as strings,
//                         directional metric and overload, isUp(), getOtherNodeName by
//                         string compare (LinkState.cpp:163-172, 195-204, 233-236)
//   linkMap / overloads   LinkState::linkMap_ (unordered_map<string, LinkSet>) and
//                         nodeOverloads_ (LinkState.h:456-467)
//   QNode / Queue         DijkstraQNode / DijkstraQ (LinkState.h:475-535): shared_ptr
//                         heap keyed (metric, name), name -> node map, make_heap on every
//                         decrease (reMake)
//   NodeResult            NodeSpfResult (LinkState.h:203-260): metric, ordered pathLinks
//                         (shared_ptr<Link>, prevNode), unordered_set<string> nextHops
//   run_spf               LinkState::runSpf (LinkState.cpp:808-882)
// Results equal the dense oracle's (tests/test_oracle_golden.py checks it); only the
// cost model differs. Never linked into or called by the product (openr_amd/).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "spf_oracle.h"

namespace {

struct FLink {
  std::string n1, n2, if1, if2;
  uint64_t m1 = 1, m2 = 1;  // metric advertised by n1 (towards n2) / by n2
  bool up = true;
  const std::string& other(const std::string& n) const {
    if (n == n1) return n2;
    if (n == n2) return n1;
    throw std::invalid_argument(n);
  }
  uint64_t metricFrom(const std::string& n) const {
    if (n == n1) return m1;
    if (n == n2) return m2;
    throw std::invalid_argument(n);
  }
};
using LinkPtr = std::shared_ptr<FLink>;
struct LinkHash {
  size_t operator()(const LinkPtr& l) const {  // hash of the ordered ((n1, if1), (n2, if2)) ends
    std::hash<std::string> h;
    size_t x = h(l->n1) * 1000003u ^ h(l->if1);
    return x * 1000003u ^ (h(l->n2) * 31u ^ h(l->if2));
  }
};
using LinkSet = std::unordered_set<LinkPtr, LinkHash>;

struct NodeResult {
  uint64_t metric = UINT64_MAX;
  std::vector<std::pair<LinkPtr, std::string>> pathLinks;
  std::unordered_set<std::string> nextHops;
};

struct QNode {
  std::string name;
  NodeResult result;
};
using QNodePtr = std::shared_ptr<QNode>;

struct Queue {  // DijkstraQ: min-heap on (metric, name)
  std::vector<QNodePtr> heap;
  std::unordered_map<std::string, QNodePtr> byName;
  static bool greater(const QNodePtr& a, const QNodePtr& b) {
    if (a->result.metric != b->result.metric) return a->result.metric > b->result.metric;
    return a->name > b->name;
  }
  QNodePtr get(const std::string& n) {
    auto it = byName.find(n);
    return it == byName.end() ? nullptr : it->second;
  }
  void insert(const std::string& n, uint64_t metric) {
    auto q = std::make_shared<QNode>();
    q->name = n;
    q->result.metric = metric;
    heap.push_back(q);
    byName.emplace(n, q);
    std::push_heap(heap.begin(), heap.end(), greater);
  }
  QNodePtr extractMin() {
    if (heap.empty()) return nullptr;
    std::pop_heap(heap.begin(), heap.end(), greater);
    auto q = heap.back();
    heap.pop_back();
    byName.erase(q->name);
    return q;
  }
  void reMake() { std::make_heap(heap.begin(), heap.end(), greater); }
};

struct Replica {  // one LinkState (per thread)
  std::unordered_map<std::string, LinkSet> linkMap;
  std::unordered_map<std::string, bool> overloads;

  Replica(const oracle_graph* g, const std::vector<std::string>& names) {
    std::vector<LinkPtr> byId(g->num_links);
    for (uint32_t u = 0; u < g->num_nodes; ++u) overloads[names[u]] = g->node_overloaded[u] != 0;
    for (uint32_t u = 0; u < g->num_nodes; ++u) {
      linkMap[names[u]];
      for (uint32_t e = g->row_ptr[u]; e < g->row_ptr[u + 1]; ++e) {
        const uint32_t l = g->link_id[e], v = g->col[e];
        auto& lp = byId[l];
        if (!lp) {
          lp = std::make_shared<FLink>();
          lp->n1 = names[u];
          lp->n2 = names[v];
          lp->if1 = "if" + std::to_string(l) + "a";
          lp->if2 = "if" + std::to_string(l) + "b";
          lp->m1 = g->metric[e];
          lp->up = g->edge_up[e] != 0;
        } else {
          lp->m2 = g->metric[e];
        }
        linkMap[names[u]].insert(lp);
      }
    }
  }

  // LinkState::runSpf (LinkState.cpp:808-882)
  std::unordered_map<std::string, NodeResult> runSpf(const std::string& src, bool useLinkMetric) const {
    std::unordered_map<std::string, NodeResult> result;
    Queue q;
    q.insert(src, 0);
    while (auto node = q.extractMin()) {
      auto& rec = result.emplace(node->name, std::move(node->result)).first->second;
      const auto ov = overloads.find(node->name);
      if (node->name != src && ov != overloads.end() && ov->second) continue;  // sink
      const auto lm = linkMap.find(node->name);
      if (lm == linkMap.end()) continue;
      for (const auto& link : lm->second) {
        const auto& other = link->other(node->name);
        if (!link->up || result.count(other)) continue;
        const uint64_t metric = useLinkMetric ? link->metricFrom(node->name) : 1u;
        auto otherNode = q.get(other);
        if (!otherNode) {
          q.insert(other, rec.metric + metric);
          otherNode = q.get(other);
        }
        if (otherNode->result.metric >= rec.metric + metric) {
          if (otherNode->result.metric > rec.metric + metric) {
            otherNode->result.metric = rec.metric + metric;
            otherNode->result.pathLinks.clear();
            otherNode->result.nextHops.clear();
            q.reMake();
          }
          otherNode->result.pathLinks.emplace_back(link, node->name);
          for (const auto& nh : rec.nextHops) otherNode->result.nextHops.insert(nh);  // addNextHops
          if (otherNode->result.nextHops.empty()) otherNode->result.nextHops.insert(other);
        }
      }
    }
    return result;
  }
};

}  // namespace

extern "C" {

/* runSpf(sources[i]) for i < n on `nthreads` threads (one LinkState replica each, built
 * before the clock starts), reference data structures. Node names are
 * name_pool[name_off[v] .. name_off[v+1]). Optional outputs: dist [n][V] (UINT64_MAX for
 * nodes absent from the SpfResult) and nh [n][V][nh_bytes] (bit i = the source's i-th
 * distinct neighbour in row order). *out_seconds = wall time of the solves alone.
 * Returns 0, or -1 on a bad argument. */
int faithful_all_sources(const oracle_graph* g, const char* name_pool, const uint64_t* name_off,
                         const uint32_t* sources, uint32_t n, int use_link_metric, int nthreads, uint64_t* dist,
                         uint8_t* nh, uint32_t nh_bytes, double* out_seconds) {
  if (!g || !name_pool || !name_off || (n && !sources)) return -1;
  const uint32_t V = g->num_nodes;
  for (uint32_t i = 0; i < n; ++i)
    if (sources[i] >= V) return -1;
  std::vector<std::string> names(V);
  for (uint32_t v = 0; v < V; ++v) names[v].assign(name_pool + name_off[v], name_off[v + 1] - name_off[v]);
  nthreads = std::max(1, std::min(nthreads, 256));
  std::vector<std::unique_ptr<Replica>> reps(nthreads);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back([&, t] { reps[t] = std::make_unique<Replica>(g, names); });
    for (auto& x : th) x.join();
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      for (uint32_t i = (uint32_t)t; i < n; i += (uint32_t)nthreads) {
        const uint32_t s = sources[i];
        auto res = reps[t]->runSpf(names[s], use_link_metric != 0);
        if (!dist && !nh) continue;
        std::unordered_map<std::string, uint32_t> bit;  // distinct neighbours of s in row order
        for (uint32_t e = g->row_ptr[s]; e < g->row_ptr[s + 1]; ++e)
          bit.emplace(names[g->col[e]], (uint32_t)bit.size());
        for (uint32_t v = 0; v < V; ++v) {
          auto it = res.find(names[v]);
          if (dist) dist[(size_t)i * V + v] = it == res.end() ? UINT64_MAX : it->second.metric;
          if (nh) {
            uint8_t* o = nh + ((size_t)i * V + v) * nh_bytes;
            std::memset(o, 0, nh_bytes);
            if (it != res.end())
              for (const auto& h : it->second.nextHops) {
                const uint32_t b = bit.at(h);
                if (b / 8 < nh_bytes) o[b / 8] |= (uint8_t)(1u << (b % 8));
              }
          }
        }
      }
    });
  }
  for (auto& x : th) x.join();
  if (out_seconds) *out_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // extern "C"
