// cpu_engine_stub.cpp — TEST INFRASTRUCTURE ONLY: the openr_spf C-ABI (include/openr_spf.h)
// answered by the CPU oracle (oracle/spf_oracle.c), so the HOST side of the drop-in
// (LinkState memo, SpfSolver route builds, RibPolicy) can be profiled with gprof in a
// container without a GPU (tests/cpp/host_profile.cpp). It is linked only into that
// profiling binary, never into libopenr_spf.so / libopenr_decision.so, and nothing in the
// product loads it: the product has no CPU path (openr_spf_create fails with ENODEV).
// Only the entry points LinkState calls are served; the rest return ENOTSUP.
#include <cstdlib>
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/openr_spf.h"
#include "../../oracle/spf_oracle.h"

struct openr_spf_ctx {
  std::vector<uint32_t> row, col, lid, rank;
  std::vector<uint64_t> metric;
  std::vector<uint8_t> up, ovl;
  uint32_t V = 0, E = 0, L = 0;
  bool has = false;
  openr_spf_stats_t stats{};
  oracle_graph og() const {
    return oracle_graph{V, E, L, row.data(), col.data(), metric.data(), lid.data(), up.data(), ovl.data(), rank.data()};
  }
};

namespace {
thread_local std::string g_err;
int fail(int code, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
uint32_t nhBits(const openr_spf_ctx* c) {
  uint32_t mx = 1;
  const oracle_graph g = c->og();
  for (uint32_t u = 0; u < c->V; ++u) mx = std::max(mx, oracle_num_distinct_neighbors(&g, u));
  return mx;
}
// rows [n] on hardware threads
template <typename F>
void parallelRows(uint32_t n, F f) {
  const unsigned T = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (uint32_t i = t; i < n; i += T) f(i);
    });
  for (auto& x : th) x.join();
}
}  // namespace

extern "C" {
int openr_spf_abi_version(void) { return OPENR_SPF_ABI_VERSION; }
int openr_spf_host_alloc(size_t bytes, void** out) {
  *out = std::malloc(bytes ? bytes : 1);
  return *out ? 0 : OPENR_SPF_ENOMEM;
}
void openr_spf_host_free(void* p) { std::free(p); }
const char* openr_spf_build_id(void) { return "cpu-stub (test infrastructure)"; }
const char* openr_spf_last_error(void) { return g_err.c_str(); }
const char* openr_spf_last_kernels(void) { return "cpu_stub"; }
void openr_spf_limits(openr_spf_limits_t* out) {
  out->max_nodes = 1u << 30;
  out->max_nh_bits = 1u << 16;
}
int openr_spf_create(const int*, int, openr_spf_ctx** out) {
  *out = new openr_spf_ctx();
  return OPENR_SPF_OK;
}
void openr_spf_destroy(openr_spf_ctx* ctx) { delete ctx; }
int openr_spf_set_graph(openr_spf_ctx* c, const openr_spf_graph* g) {
  c->V = g->num_nodes;
  c->E = g->num_dir_edges;
  c->L = g->num_links;
  c->row.assign(g->row_ptr, g->row_ptr + c->V + 1);
  c->col.assign(g->col, g->col + c->E);
  c->metric.assign(g->metric, g->metric + c->E);
  c->lid.assign(g->link_id, g->link_id + c->E);
  c->up.assign(g->edge_up, g->edge_up + c->E);
  c->ovl.assign(g->node_overloaded, g->node_overloaded + c->V);
  c->rank.assign(g->name_rank, g->name_rank + c->V);
  c->has = true;
  return OPENR_SPF_OK;
}
int openr_spf_nh_bytes(const openr_spf_ctx* c, uint32_t* out) {
  *out = (nhBits(c) + 7) / 8;
  return OPENR_SPF_OK;
}
int openr_spf_neighbor_map(const openr_spf_ctx* c, uint32_t src, uint32_t* out, uint32_t cap, uint32_t* count) {
  uint32_t k = 0;
  for (uint32_t e = c->row[src]; e < c->row[src + 1]; ++e) {
    bool seen = false;
    for (uint32_t i = 0; i < k && !seen; ++i) seen = out[i] == c->col[e];
    if (!seen) {
      if (k >= cap) return fail(OPENR_SPF_EINVAL, "capacity");
      out[k++] = c->col[e];
    }
  }
  *count = k;
  return OPENR_SPF_OK;
}
static int solveRows(openr_spf_ctx* c, const uint32_t* sources, uint32_t n, uint32_t flags, const uint32_t* ip,
                     const uint32_t* il, uint64_t* dist, uint8_t* nh, uint32_t nb, uint64_t* tight, uint32_t* order) {
  const oracle_graph g = c->og();
  const uint32_t words = (c->E + 63) / 64;
  parallelRows(n, [&](uint32_t i) {
    std::vector<uint64_t> ign;
    if (ip) {
      ign.assign((c->L + 63) / 64, 0);
      for (uint32_t k = ip[i]; k < ip[i + 1]; ++k) ign[il[k] >> 6] |= 1ull << (il[k] & 63);
    }
    std::vector<uint32_t> plp(c->V + 1), ple(c->E + 1), ord(c->V);
    const int64_t cnt =
        oracle_run_spf(&g, sources[i], (flags & OPENR_SPF_USE_LINK_METRIC) != 0, ip ? ign.data() : nullptr,
                       dist + (size_t)i * c->V, nh ? nh + (size_t)i * c->V * nb : nullptr, nb, ord.data(),
                       tight ? plp.data() : nullptr, tight ? ple.data() : nullptr);
    if (tight) {
      uint64_t* t = tight + (size_t)i * words;
      std::fill(t, t + words, 0ull);
      for (uint32_t k = 0; k < plp[c->V]; ++k) t[ple[k] >> 6] |= 1ull << (ple[k] & 63);
    }
    if (order) {
      uint32_t* o = order + (size_t)i * c->V;
      std::fill(o, o + c->V, UINT32_MAX);
      for (int64_t k = 0; k < cnt; ++k) o[ord[k]] = (uint32_t)k;
    }
  });
  c->stats.spf_runs += n;
  c->stats.batches += 1;
  return OPENR_SPF_OK;
}
int openr_spf_solve(openr_spf_ctx* c, const uint32_t* s, uint32_t n, uint32_t flags, uint64_t* dist, uint8_t* nh,
                    uint32_t nb, uint64_t* tight) {
  return solveRows(c, s, n, flags, nullptr, nullptr, dist, nh, nb, tight, nullptr);
}
int openr_spf_solve_ignore(openr_spf_ctx* c, const uint32_t* s, uint32_t n, uint32_t flags, const uint32_t* ip,
                           const uint32_t* il, uint64_t* dist, uint8_t* nh, uint32_t nb, uint64_t* tight) {
  return solveRows(c, s, n, flags, ip, il, dist, nh, nb, tight, nullptr);
}
int openr_spf_solve_order(openr_spf_ctx* c, const uint32_t* s, uint32_t n, uint32_t flags, const uint32_t* ip,
                          const uint32_t* il, uint64_t* dist, uint8_t* nh, uint32_t nb, uint64_t* tight,
                          uint32_t* order) {
  return solveRows(c, s, n, flags, ip, il, dist, nh, nb, tight, order);
}
int openr_spf_solve_device(openr_spf_ctx*, int, const uint32_t*, uint32_t, uint32_t, const uint32_t*, const uint32_t*,
                           uint64_t*, uint8_t*, uint32_t, uint64_t*, void*) {
  return fail(OPENR_SPF_ENOTSUP, "cpu stub: no device form");
}
int openr_spf_take_status(openr_spf_ctx*, int, uint32_t* s) {
  *s = 0;
  return OPENR_SPF_OK;
}
int openr_spf_whatif(openr_spf_ctx*, const uint32_t*, uint32_t, const uint32_t*, uint32_t, uint32_t, uint32_t*,
                     uint64_t*) {
  return fail(OPENR_SPF_ENOTSUP, "cpu stub");
}
int openr_spf_whatif_device(openr_spf_ctx*, int, const uint32_t*, uint32_t, const uint32_t*, uint32_t, uint32_t,
                            uint32_t*, void*, uint64_t*) {
  return fail(OPENR_SPF_ENOTSUP, "cpu stub");
}
int openr_spf_ksp2(openr_spf_ctx* c, const uint32_t* src, const uint32_t* dst, uint32_t n, uint32_t cap,
                   uint32_t* t1, uint32_t* t2) {
  const oracle_graph g = c->og();
  return oracle_ksp2_batch(&g, src, dst, n, cap, t1, t2, 16) == 0 ? OPENR_SPF_OK : fail(OPENR_SPF_E2BIG, "ksp2");
}
int openr_spf_ksp2_device(openr_spf_ctx*, int, const uint32_t*, uint32_t, const uint32_t*, const uint32_t*, uint32_t,
                          uint32_t, uint32_t*, uint32_t*, void*) {
  return fail(OPENR_SPF_ENOTSUP, "cpu stub");
}
int openr_spf_patch_graph(openr_spf_ctx* c, const openr_spf_patch* p) {
  for (uint32_t i = 0; i < p->n_edges; ++i) c->metric[p->edge_ids[i]] = p->metric[i];
  for (uint32_t i = 0; i < p->n_links; ++i)
    for (uint32_t e = 0; e < c->E; ++e)
      if (c->lid[e] == p->link_ids[i]) c->up[e] = p->link_up[i];
  for (uint32_t i = 0; i < p->n_nodes; ++i) c->ovl[p->node_ids[i]] = p->node_overloaded[i];
  return OPENR_SPF_OK;
}
int openr_spf_refresh(openr_spf_ctx* c, const uint32_t* s, uint32_t n, uint32_t flags, uint64_t* dist, uint8_t* nh,
                      uint32_t nb, uint64_t* tight, uint32_t* out) {
  if (out) *out = n;
  return solveRows(c, s, n, flags, nullptr, nullptr, dist, nh, nb, tight, nullptr);
}
int openr_spf_refresh_device(openr_spf_ctx*, int, const uint32_t*, uint32_t, uint32_t, uint64_t*, uint8_t*, uint32_t,
                             uint64_t*, void*, uint32_t*) {
  return fail(OPENR_SPF_ENOTSUP, "cpu stub");
}
int openr_spf_get_stats(const openr_spf_ctx* c, openr_spf_stats_t* out) {
  *out = c->stats;
  return OPENR_SPF_OK;
}
}  // extern "C"
