// adjdb_capi.cpp — extern "C" wrapper of AdjDbCodec (include/openr_adjdb.h).
#include <cerrno>
#include <chrono>
#include <unordered_map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/openr_adjdb.h"
#include "../../../include/openr_routes.h"
#include "AdjDbCodec.h"
#include "Decision.h"
#include "HostParallel.h"

struct openr_adjdb_batch {
  std::vector<openr::thrift::AdjacencyDatabase> dbs;
};

struct openr_adjdb_graph {
  // the area's LinkState, held in the areaLinkStates map SpfSolver consumes
  std::unordered_map<std::string, openr::LinkState> als;
  openr::LinkState* linkState = nullptr;
  const openr::LinkState::CsrMirror* mirror = nullptr;
  std::unique_ptr<openr::PrefixState> prefixes;  // openr_routes_build: fd00::<id>/128 per node
  std::vector<openr::thrift::IpPrefix> prefixList;
};

namespace {
thread_local std::string g_error;

int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

template <class F>
int guarded(F&& f) {
  try {
    g_error.clear();
    return f();
  } catch (const openr::CompactProtocolError& e) {
    return fail(OPENR_ADJDB_EBADMSG, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(OPENR_ADJDB_EINVAL, e.what());
  } catch (const std::exception& e) {
    return fail(OPENR_ADJDB_EINTERNAL, e.what());
  } catch (...) {
    return fail(OPENR_ADJDB_EINTERNAL, "unknown exception");
  }
}
}  // namespace

#ifndef OPENR_DECISION_BUILD_ID
#define OPENR_DECISION_BUILD_ID "unknown"
#endif

extern "C" {

const char* openr_decision_build_id(void) { return OPENR_DECISION_BUILD_ID; }

const char* openr_adjdb_last_error(void) { return g_error.c_str(); }

int openr_adjdb_decode(const uint8_t* data, const uint64_t* offsets, uint32_t n, uint32_t n_threads,
                       openr_adjdb_batch** out) {
  if (!out || !offsets || (n && !data)) return fail(OPENR_ADJDB_EINVAL, "null argument");
  *out = nullptr;
  return guarded([&] {
    std::vector<std::string_view> values(n);
    for (uint32_t i = 0; i < n; ++i) {
      if (offsets[i + 1] < offsets[i]) return fail(OPENR_ADJDB_EINVAL, "offsets not monotone at " + std::to_string(i));
      values[i] = std::string_view(reinterpret_cast<const char*>(data) + offsets[i], offsets[i + 1] - offsets[i]);
    }
    auto b = std::make_unique<openr_adjdb_batch>();
    b->dbs = openr::serializer::readAdjacencyDatabases(values, n_threads);
    *out = b.release();
    return 0;
  });
}

void openr_adjdb_free(openr_adjdb_batch* batch) { delete batch; }

int openr_adjdb_info(const openr_adjdb_batch* b, openr_adjdb_info_t* out) {
  if (!b || !out) return fail(OPENR_ADJDB_EINVAL, "null argument");
  openr_adjdb_info_t info{};
  info.n_dbs = (uint32_t)b->dbs.size();
  for (const auto& db : b->dbs) {
    info.n_adjs += db.adjacencies.size();
    info.string_bytes += db.thisNodeName.size() + db.area.size();
    for (const auto& a : db.adjacencies) {
      info.string_bytes += a.otherNodeName.size() + a.ifName.size() + a.otherIfName.size() + a.nextHopV6.addr.size() +
                           a.nextHopV4.addr.size();
    }
    if (db.perfEvents) info.n_perf_events += db.perfEvents->events.size();
  }
  info.n_strings = 2ull * info.n_dbs + 5ull * info.n_adjs;
  *out = info;
  return 0;
}

int openr_adjdb_export(const openr_adjdb_batch* b, const openr_adjdb_columns* c) {
  if (!b || !c) return fail(OPENR_ADJDB_EINVAL, "null argument");
  const void* ptrs[] = {c->str_pool, c->str_off,      c->node_name,   c->area,   c->node_overloaded, c->node_label,
                        c->adj_begin, c->other_node,  c->if_name,     c->other_if_name, c->nh_v6, c->nh_v4,
                        c->metric,   c->adj_label,    c->adj_overloaded, c->rtt,  c->timestamp, c->weight};
  for (const void* p : ptrs)
    if (!p) return fail(OPENR_ADJDB_EINVAL, "null column pointer");
  uint64_t pos = 0;
  uint32_t s = 0;
  c->str_off[0] = 0;
  auto put = [&](const std::string& str) {
    std::memcpy(c->str_pool + pos, str.data(), str.size());
    pos += str.size();
    c->str_off[s + 1] = pos;
    return s++;
  };
  uint64_t k = 0;
  for (size_t i = 0; i < b->dbs.size(); ++i) {
    const auto& db = b->dbs[i];
    c->node_name[i] = put(db.thisNodeName);
    c->area[i] = put(db.area);
    c->node_overloaded[i] = db.isOverloaded ? 1 : 0;
    c->node_label[i] = db.nodeLabel;
    c->adj_begin[i] = k;
    for (const auto& a : db.adjacencies) {
      c->other_node[k] = put(a.otherNodeName);
      c->if_name[k] = put(a.ifName);
      c->other_if_name[k] = put(a.otherIfName);
      c->nh_v6[k] = put(a.nextHopV6.addr);
      c->nh_v4[k] = put(a.nextHopV4.addr);
      c->metric[k] = a.metric;
      c->adj_label[k] = a.adjLabel;
      c->adj_overloaded[k] = a.isOverloaded ? 1 : 0;
      c->rtt[k] = a.rtt;
      c->timestamp[k] = a.timestamp;
      c->weight[k] = a.weight;
      ++k;
    }
  }
  c->adj_begin[b->dbs.size()] = k;
  return 0;
}

int openr_adjdb_batch_from_columns(const openr_adjdb_columns* c, uint32_t n_dbs, openr_adjdb_batch** out) {
  if (!c || !out) return fail(OPENR_ADJDB_EINVAL, "null argument");
  *out = nullptr;
  return guarded([&] {
    auto str = [&](uint32_t k) { return std::string(c->str_pool + c->str_off[k], c->str_off[k + 1] - c->str_off[k]); };
    auto b = std::make_unique<openr_adjdb_batch>();
    b->dbs.resize(n_dbs);
    for (uint32_t i = 0; i < n_dbs; ++i) {
      auto& db = b->dbs[i];
      db.thisNodeName = str(c->node_name[i]);
      db.area = str(c->area[i]);
      db.isOverloaded = c->node_overloaded[i] != 0;
      db.nodeLabel = c->node_label[i];
      if (c->adj_begin[i + 1] < c->adj_begin[i]) return fail(OPENR_ADJDB_EINVAL, "adj_begin not monotone");
      db.adjacencies.resize(c->adj_begin[i + 1] - c->adj_begin[i]);
      for (uint64_t k = c->adj_begin[i], j = 0; k < c->adj_begin[i + 1]; ++k, ++j) {
        auto& a = db.adjacencies[j];
        a.otherNodeName = str(c->other_node[k]);
        a.ifName = str(c->if_name[k]);
        a.otherIfName = str(c->other_if_name[k]);
        a.nextHopV6.addr = str(c->nh_v6[k]);
        a.nextHopV4.addr = str(c->nh_v4[k]);
        a.metric = c->metric[k];
        a.adjLabel = c->adj_label[k];
        a.isOverloaded = c->adj_overloaded[k] != 0;
        a.rtt = c->rtt[k];
        a.timestamp = c->timestamp[k];
        a.weight = c->weight[k];
      }
    }
    *out = b.release();
    return 0;
  });
}

int openr_adjdb_encode_all(const openr_adjdb_batch* b, uint8_t* data, uint64_t cap, uint64_t* offsets,
                           uint64_t* total) {
  if (!b || !total) return fail(OPENR_ADJDB_EINVAL, "null argument");
  return guarded([&] {
    std::vector<std::string> enc(b->dbs.size());
    uint64_t sum = 0;
    for (size_t i = 0; i < b->dbs.size(); ++i) {
      enc[i] = openr::serializer::writeAdjacencyDatabase(b->dbs[i]);
      sum += enc[i].size();
    }
    *total = sum;
    if (!data) return 0;
    if (!offsets) return fail(OPENR_ADJDB_EINVAL, "null offsets");
    if (cap < sum) return fail(OPENR_ADJDB_ENOSPC, "buffer too small");
    uint64_t pos = 0;
    offsets[0] = 0;
    for (size_t i = 0; i < enc.size(); ++i) {
      std::memcpy(data + pos, enc[i].data(), enc[i].size());
      pos += enc[i].size();
      offsets[i + 1] = pos;
    }
    return 0;
  });
}

int openr_adjdb_encode(const openr_adjdb_batch* b, uint32_t index, uint8_t* out, uint64_t cap, uint64_t* out_len) {
  if (!b || !out_len) return fail(OPENR_ADJDB_EINVAL, "null argument");
  if (index >= b->dbs.size()) return fail(OPENR_ADJDB_EINVAL, "index out of range");
  return guarded([&] {
    const std::string s = openr::serializer::writeAdjacencyDatabase(b->dbs[index]);
    *out_len = s.size();
    if (!out || cap < s.size()) return out ? fail(OPENR_ADJDB_ENOSPC, "buffer too small") : 0;
    std::memcpy(out, s.data(), s.size());
    return 0;
  });
}

int openr_adjdb_build_graph(const openr_adjdb_batch* b, const char* area, openr_adjdb_graph** out) {
  if (!b || !area || !out) return fail(OPENR_ADJDB_EINVAL, "null argument");
  *out = nullptr;
  return guarded([&] {
    auto g = std::make_unique<openr_adjdb_graph>();
    g->linkState = &g->als.emplace(area, openr::LinkState(area)).first->second;
    for (const auto& db : b->dbs) {
      openr::thrift::AdjacencyDatabase stamped = db;
      stamped.area = area;
      g->linkState->updateAdjacencyDatabase(std::move(stamped), 0, 0);
    }
    g->mirror = &g->linkState->csrMirror();
    *out = g.release();
    return 0;
  });
}

void openr_adjdb_graph_free(openr_adjdb_graph* g) { delete g; }

int openr_adjdb_graph_info(const openr_adjdb_graph* g, openr_adjdb_graph_info_t* out) {
  if (!g || !out) return fail(OPENR_ADJDB_EINVAL, "null argument");
  const auto& m = *g->mirror;
  out->num_nodes = (uint32_t)m.names.size();
  out->num_dir_edges = (uint32_t)m.col.size();
  out->num_links = (uint32_t)m.links.size();
  out->name_bytes = 0;
  for (const auto& n : m.names) out->name_bytes += n.size();
  return 0;
}

int openr_adjdb_graph_export(const openr_adjdb_graph* g, uint32_t* row_ptr, uint32_t* col, uint64_t* metric,
                             uint32_t* link_id, uint8_t* edge_up, uint8_t* node_overloaded, uint32_t* name_rank,
                             char* name_pool, uint64_t* name_off) {
  if (!g || !row_ptr || !col || !metric || !link_id || !edge_up || !node_overloaded || !name_rank || !name_pool ||
      !name_off)
    return fail(OPENR_ADJDB_EINVAL, "null argument");
  const auto& m = *g->mirror;
  const size_t V = m.names.size(), E = m.col.size();
  std::memcpy(row_ptr, m.rowPtr.data(), (V + 1) * sizeof(uint32_t));
  if (E) {
    std::memcpy(col, m.col.data(), E * sizeof(uint32_t));
    std::memcpy(metric, m.metric.data(), E * sizeof(uint64_t));
    std::memcpy(link_id, m.linkId.data(), E * sizeof(uint32_t));
    std::memcpy(edge_up, m.edgeUp.data(), E);
  }
  if (V) {
    std::memcpy(node_overloaded, m.overloaded.data(), V);
    std::memcpy(name_rank, m.nameRank.data(), V * sizeof(uint32_t));
  }
  uint64_t pos = 0;
  name_off[0] = 0;
  for (size_t i = 0; i < V; ++i) {
    std::memcpy(name_pool + pos, m.names[i].data(), m.names[i].size());
    pos += m.names[i].size();
    name_off[i + 1] = pos;
  }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// openr_routes_build (include/openr_routes.h)
// ---------------------------------------------------------------------------
namespace {
uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 33);
}
// 8 bytes per step (the route tally hashes every next hop of 100 M routes on G100: a byte
// at a time that was ~8 % of the route-build wall time)
uint64_t hashStr(uint64_t h, const std::string& s) {
  const char* p = s.data();
  size_t n = s.size();
  for (; n >= 8; p += 8, n -= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    h = (h ^ w) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  uint64_t w = 0;
  std::memcpy(&w, p, n);
  return mix64(h ^ w ^ ((uint64_t)s.size() << 56));
}
}  // namespace

extern "C" int openr_routes_build(openr_adjdb_graph* g, const uint32_t* node_ids, uint32_t n, uint32_t flags,
                                  int32_t default_weight, const int32_t* neighbor_weight,
                                  openr_routes_stats_t* out) {
  if (!g || !out || (n && !node_ids)) return fail(OPENR_ADJDB_EINVAL, "null argument");
  const auto& m = *g->mirror;
  const uint32_t V = (uint32_t)m.names.size();
  for (uint32_t i = 0; i < n; ++i)
    if (node_ids[i] >= V) return fail(OPENR_ADJDB_EINVAL, "node id " + std::to_string(node_ids[i]) + " out of range");
  return guarded([&] {
    using clock = std::chrono::steady_clock;
    if (!g->prefixes) {  // one loopback prefix per node, originated once per graph
      g->prefixes = std::make_unique<openr::PrefixState>();
      const std::string area = g->linkState->getArea();
      for (uint32_t v = 0; v < V; ++v) {
        char buf[48];
        std::snprintf(buf, sizeof(buf), "fd00::%x", v);
        openr::thrift::PrefixEntry e;
        e.prefix = openr::thrift::IpPrefix{buf, 128};
        g->prefixList.push_back(e.prefix);
        g->prefixes->updatePrefix(m.names[v], area, e);
      }
    }
    *out = openr_routes_stats_t{};
    if (!n) return 0;
    std::vector<std::string> nodes;
    nodes.reserve(n);
    for (uint32_t i = 0; i < n; ++i) nodes.push_back(m.names[node_ids[i]]);
    openr::SpfSolver solver(nodes[0], (flags & OPENR_ROUTES_V4) != 0, (flags & OPENR_ROUTES_LFA) != 0);
    std::unique_ptr<openr::RibPolicy> policy;
    if (flags & OPENR_ROUTES_UCMP) {  // RibPolicy set_weight over every route (Decision.cpp applies it per rebuild)
      openr::RibPolicyStatement st;
      st.name = "ucmp";
      st.prefixes = std::set<openr::thrift::IpPrefix>(g->prefixList.begin(), g->prefixList.end());
      st.defaultWeight = default_weight;
      if (neighbor_weight)
        for (uint32_t v = 0; v < V; ++v)
          if (neighbor_weight[v] > 0) st.neighborToWeight[m.names[v]] = neighbor_weight[v];
      policy = std::make_unique<openr::RibPolicy>(std::vector<openr::RibPolicyStatement>{st});
    }
    // per node: build, policy, checksum, free — on the worker that built it (streaming
    // buildRouteDbs), while the DB is cache-hot
    std::vector<openr_routes_stats_t> per(n, openr_routes_stats_t{});
    const auto t0 = clock::now();
    solver.buildRouteDbs(nodes, g->als, *g->prefixes, [&](size_t i, std::optional<openr::DecisionRouteDb>& db) {
      if (!db) return;
      auto& o = per[i];
      if (policy) {
        const auto p0 = clock::now();
        policy->applyPolicy(db->unicastRoutes);
        o.ms_policy = std::chrono::duration<double, std::milli>(clock::now() - p0).count();
      }
      const uint64_t hn = hashStr(0xcbf29ce484222325ULL, nodes[i]);
      o.unicast_routes = db->unicastRoutes.size();
      o.mpls_routes = db->mplsRoutes.size();
      for (auto const& [p, route] : db->unicastRoutes) {
        const uint64_t hp = hashStr(hn, p.addr) ^ (uint64_t)p.prefixLength;
        for (auto const& nh : route.nexthops) {
          ++o.nexthops;
          o.weighted_nexthops += nh.weight > 1;
          uint64_t h = hashStr(hp, nh.address.addr);
          h = hashStr(h, nh.address.ifName.value_or(""));
          h = hashStr(h, nh.neighborNodeName.value_or(""));
          h = mix64(h ^ ((uint64_t)(uint32_t)nh.metric << 32) ^ (uint32_t)nh.weight);
          o.checksum += h;  // order-independent
        }
      }
    });
    const double ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    double policyMs = 0;
    for (auto const& o : per) {
      out->unicast_routes += o.unicast_routes;
      out->mpls_routes += o.mpls_routes;
      out->nexthops += o.nexthops;
      out->weighted_nexthops += o.weighted_nexthops;
      out->checksum += o.checksum;
      policyMs += o.ms_policy;
    }
    // the policy's share of the wall time: its thread time over the workers that ran
    const unsigned workers = openr::parallelWorkers(n, 1);
    out->ms_policy = policyMs / workers;
    out->ms_build = ms - out->ms_policy;
    return 0;
  });
}
