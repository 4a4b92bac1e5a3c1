// spf_capi.hip — host side of the C-ABI declared in include/openr_spf.h.
//
// Owns the per-device CSR replicas (one DevGraph per GPU of the context), picks the
// kernel for a solve (uniform-cost BFS or settle-safe buckets), splits a batch of
// sources across the context's devices and moves results. There is deliberately no
// CPU path: every solve runs on the GPU or fails with an error code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/openr_spf.h"
#include "spf_kernels.h"

using namespace openr_spf;

namespace {

thread_local std::string g_last_error;
thread_local std::string g_launch_trace;  // "kernel;kernel;..." of the last solve call

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(OPENR_SPF_EIO, "%s failed: %s", #expr, hipGetErrorString(_e));       \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Device {
  int ordinal = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;
  DevGraph g;
  // scratch for host-buffer solves
  DevBuf<uint32_t> src, ign_ptr, ign_links;
  DevBuf<uint64_t> dist, tight;
  DevBuf<uint8_t> nh;
  DevBuf<uint32_t> ovf;  // re-run list of the BFS ring variants ([n * slices])
  // small multi-class batches: the classes run concurrently, one stream each (forked from
  // and joined back into the caller's stream), each with its own re-run list
  DevBuf<uint32_t> slicetmp;  // code-family sliced class: [n][nsl][V] next-hop chunks
  DevBuf<uint32_t> work;  // dynamic-scheduling counters (kWorkSlots)
  DevBuf<uint32_t> status;  // sticky OPENR_SPF_STATUS_* bits of device-form calls
  DevBuf<uint32_t> perm, part;  // source-class partition of a batch
  // what-if sweep: base SPF rows, the affected-unit work list, chunk result rows
  DevBuf<uint64_t> base_dist, base_tight, wdist;
  DevBuf<uint8_t> base_nh, wnh;
  DevBuf<uint32_t> wsrc, wlink, wunit, wcount, wiota, win_links, win_src, wchanged;
  DevBuf<uint32_t> wchanged_t;  // grouped repair: results source-major, transposed into the caller's rows
  DevBuf<uint16_t> base_tin;  // what-if base SPF: tight in-degree rows (rounds plan)
  size_t wiota_n = 0;  // wiota[0, wiota_n) holds 0, 1, 2, ... (kept across calls)
  // KSP2: base rows, chunk rows, per-chunk ignore slots / sources / pointers, status
  DevBuf<uint64_t> kbase, krows;
  DevBuf<uint16_t> krows16;  // KSP2 second SPFs on the code family: u16 level rows
  uint32_t ktag = 0;         // tagged krows16: tag of the last chunk (0 = rows zeroed)
  size_t ktag_rows = 0;      // entries of krows16 zeroed for tagging
  DevBuf<uint32_t> kign, kend, ksrc, kptr, kstatus, kin_src, kin_row, kin_dst, ktok1, ktok2, kq;
  DevBuf<uint32_t> kretry;  // KSP small-tier overflows: [0,1] counts (k = 1, k = 2), lists after
  DevBuf<uint32_t> kkeep, kpart;  // KSP pairs that need a second SPF; its count as a class partition
  DevBuf<uint32_t> ktloff;  // KSP2 k = 1: per base row, pathLinks list offsets [V + 1]
  DevBuf<uint2> ktlent;     // ... and entries [E] (launch_ksp_path_lists)
  // what-if delta output of the host form (openr_spf_whatif_delta): per-unit pool offsets,
  // the pool (node, distance, next-hop bytes) and its cursor
  DevBuf<uint32_t> dl_off, dl_node;
  DevBuf<unsigned long long> dl_dist, dl_used, dl_tsum;
  DevBuf<uint8_t> dl_nh;
  // ... and the host form's device-side CSR before it is copied out
  DevBuf<unsigned long long> dlo_ptr, dlo_dist;
  DevBuf<uint32_t> dlo_node;
  DevBuf<uint8_t> dlo_nh;
  // incremental updates: patch records, the last patch's delta edges, refresh work list,
  // host-form refresh rows
  DevBuf<PatchRec> precs;
  DevBuf<DeltaEdge> delta;
  DevBuf<uint32_t> alist, asrc, acount, alist2, asrc2;  // refresh: listed rows (first / exact stage)
  // exact-order kernel: per-solve slots when a slot does not fit LDS; pop-order rows
  DevBuf<uint8_t> exscratch;
  DevBuf<uint32_t> order;
};

// Launch counters live zeroed: each kernel's last workgroup resets what it used.
hipError_t reserve_counters(Device& d) {
  if (d.work.p) return hipSuccess;
  hipError_t e = d.work.reserve(kWorkSlots);
  if (e == hipSuccess) e = hipMemset(d.work.p, 0, kWorkSlots * sizeof(uint32_t));
  return e;
}

void free_graph(DevGraph& g) {
  void* ptrs[] = {g.row, g.row2, g.row2t, g.ovl_bits, g.ellt,    g.ellv,  g.adj,  g.w,    g.win, g.rev,
                   g.lid, g.nbr,  g.ovl,   g.cls,      g.cls_lvl, g.ledge, g.rank, g.erec, g.w64, g.elld, g.erecs};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  g = DevGraph{};
}

}  // namespace

namespace openr_spf {
void note_launch(const char* kernel) {
  if (g_launch_trace.size() < 4096) {
    g_launch_trace += kernel;
    g_launch_trace += ';';
  }
}
void clear_launch_trace() { g_launch_trace.clear(); }
}  // namespace openr_spf

struct openr_spf_ctx {
  std::vector<Device> devs;
  bool has_graph = false;
  uint32_t V = 0, E = 0, L = 0;
  std::vector<uint32_t> row_ptr, col;
  uint32_t nh_bits = 0;         // max distinct degree
  uint32_t w_min = 0, w_max = 0;
  bool metric_ok = true;        // every usable metric in [1, 2^31-1]
  uint32_t group_lanes = 4;
  int family = kFamCode;        // BFS kernel family picked for this graph (FrontierEstimate)
  uint32_t est_depth = 0;       // sampled BFS hop depth (general-metric kernel choice)
  uint32_t cls_mask[kNumFamilies] = {0, 0};  // source classes present among the nodes, per family
  uint32_t nsl[kNumFamilies] = {1, 1};       // next-hop slices of each family's sliced class
  uint32_t nsl_max() const { return std::max(nsl[0], nsl[1]); }
  openr_spf_stats_t stats{};
  // host copy of the mutable attributes and of the device arrays derived from them, so
  // openr_spf_patch_graph can recompute and re-upload single elements
  std::vector<uint64_t> metric;
  std::vector<uint8_t> edge_up, ovl;
  std::vector<uint32_t> adj, w, win, rev, lid, owner, ovl_bits;
  std::vector<uint2> ledge, row2t;
  std::vector<uint4> erec, ellt;
  std::vector<uint32_t> erec_pos;  // directed edge -> its position in DevGraph::erecs
  // delta edges of the most recent patch (openr_spf_refresh); invalid after set_graph
  std::vector<DeltaEdge> delta;
  bool delta_valid = false;
  // the rows before or after the last patch came from a graph with zero / wrapped
  // metrics: the delta filter's tight-edge reasoning does not hold, refresh every row
  bool delta_all = false;
  // no refresh since the last patch: the next patch merges into delta (rows may still be
  // those of the graph before the earlier patch), keeping each edge's oldest state
  bool refreshed = true;
  std::unordered_map<uint32_t, uint32_t> delta_index;  // directed edge -> delta slot
  // metrics of the usable edges as a multiset (w_min / w_max after a patch without an O(E)
  // scan) and the number of usable edges whose metric is 0 or above 2^31-1
  std::map<uint32_t, uint32_t> wcount;
  uint64_t n_bad_metric = 0;
  // per-patch marks (stamp == patch_epoch: set during this patch), so a patch costs
  // O(touched edges) rather than O(E)
  std::vector<uint32_t> seen_e, dirty_e, dirty_v;
  uint32_t patch_epoch = 0;
  void count_metric(uint32_t e, int dir) {  // e's contribution while it is usable
    if (adj[e] & kEdgeDown) return;
    const uint64_t m = metric[e];
    if (m == 0 || m > 0x7FFFFFFFull) {
      n_bad_metric += dir > 0 ? 1 : (uint64_t)-1;
      return;
    }
    if (dir > 0) ++wcount[(uint32_t)m];
    else if (auto it = wcount.find((uint32_t)m); it != wcount.end() && --it->second == 0) wcount.erase(it);
  }
};

namespace {

constexpr uint32_t kDeepGraphLevels = 24;
constexpr uint32_t kRoundsMaxDepth = 48;  // hop depth below which general metrics use the rounds kernel

struct Plan {
  bool exact = false;   // spf_exact.hip: the reference's heap process (metrics / sizes outside the fast kernels)
  bool use_metric = true;
  bool bfs = true;
  bool rounds = false;  // general metrics: distance rounds + Kahn (shallow graphs), else fringe
  int family = kFamCode;
  uint64_t cost = 1;
  uint32_t delta = 1;
  bool dist64 = false;
  int nh_mode = kNhByte;
};

// Tuning / test override (benchmarks and parity tests only): OPENR_SPF_BFS_FAMILY=code|lvl.
int family_override(int dflt) {
  const char* e = std::getenv("OPENR_SPF_BFS_FAMILY");
  if (!e) return dflt;
  if (!std::strcmp(e, "code")) return kFamCode;
  if (!std::strcmp(e, "lvl")) return kFamLvl;
  return dflt;
}

// Frontier shape of a graph, sampled on the host at set_graph (O(samples * (V + E))):
// BFS from evenly spaced sources plus the widest row, overloaded nodes as sinks
// (LinkState.cpp:831-838). depth picks the kernel family — the lvl kernels win on deep
// graphs (grid G100: ~150 levels of ~70 nodes; 1.07 vs 1.92 ms), the code kernels on
// shallow ones (fabric: 5 levels; 1.44 vs 1.95 ms) — and width2 (max |level L| +
// |level L+1|) sizes the frontier ring (width1 = max |level L|: the lean pass's halves).
struct FrontierEstimate {
  uint32_t depth = 0, width2 = 0, width1 = 0;
  int family() const { return depth >= kDeepGraphLevels ? kFamLvl : kFamCode; }
};

FrontierEstimate estimate_frontier(uint32_t V, const uint32_t* row_ptr, const uint32_t* adj, const uint8_t* ovl) {
  FrontierEstimate est;
  if (V == 0) return est;
  std::vector<uint32_t> srcs;
  const uint32_t ns = std::min<uint32_t>(V, 8u);
  for (uint32_t i = 0; i < ns; ++i) srcs.push_back((uint32_t)((uint64_t)i * V / ns));
  uint32_t widest = 0;
  for (uint32_t u = 1; u < V; ++u)
    if (row_ptr[u + 1] - row_ptr[u] > row_ptr[widest + 1] - row_ptr[widest]) widest = u;
  srcs.push_back(widest);
  std::vector<uint32_t> lvl(V), q, width;
  q.reserve(V);
  for (uint32_t src : srcs) {
    std::fill(lvl.begin(), lvl.end(), UINT32_MAX);
    q.clear();
    width.assign(1, 1);
    q.push_back(src);
    lvl[src] = 0;
    for (size_t i = 0; i < q.size(); ++i) {
      const uint32_t u = q[i];
      if (u != src && ovl[u]) continue;  // reached, never expanded
      for (uint32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
        if (adj[e] & kEdgeDown) continue;
        const uint32_t v = adj[e];
        if (lvl[v] != UINT32_MAX) continue;
        lvl[v] = lvl[u] + 1u;
        if (lvl[v] >= width.size()) width.push_back(0);
        ++width[lvl[v]];
        q.push_back(v);
      }
    }
    est.depth = std::max<uint32_t>(est.depth, (uint32_t)width.size() - 1u);
    for (size_t l = 0; l + 1 < width.size(); ++l) est.width2 = std::max<uint32_t>(est.width2, width[l] + width[l + 1]);
    for (uint32_t w : width) est.width1 = std::max(est.width1, w);
  }
  return est;
}

// Bytes of exact-order slots (global memory) a device may hold at once.
constexpr uint64_t kExactScratchBytes = uint64_t(2) << 30;

int make_plan(const openr_spf_ctx* ctx, uint32_t flags, bool has_ign, Plan* p) {
  const bool use_metric = (flags & OPENR_SPF_USE_LINK_METRIC) != 0;
  p->use_metric = use_metric;
  // Outside the fast kernels' domain the exact-order kernel replays the reference's heap
  // process instead of refusing the graph: zero or wrapped-negative usable metrics (pop
  // order history-dependent), next-hop sets wider than 256, graphs larger
  // than the LDS-resident layouts, and pop-order output requests.
  auto exact = [p, ctx]() -> int {
    // one exact-order slot per solve, addressed with u32 offsets (spf_exact.hip ex_layout)
    const uint64_t slot = exact_slot_bytes(ctx->V, ctx->E, ctx->L, ctx->nh_bits);
    if (slot > 0xFFFFFFFFull || slot > kExactScratchBytes)
      return fail(OPENR_SPF_E2BIG, "graph too large for the exact-order kernel (%llu bytes per solve)",
                  (unsigned long long)slot);
    p->exact = true;
    return OPENR_SPF_OK;
  };
  if ((flags & OPENR_SPF_EMIT_ORDER) || std::getenv("OPENR_SPF_FORCE_EXACT")) return exact();
  if (use_metric && !ctx->metric_ok) return exact();
  p->nh_mode = nh_mode_for_bits(ctx->nh_bits);
  if (p->nh_mode < 0) return exact();
  if (!use_metric || ctx->w_min == ctx->w_max) {
    p->bfs = true;
    p->cost = use_metric ? std::max<uint32_t>(ctx->w_min, 1u) : 1u;
    p->family = family_override(ctx->family);
    for (int c = 0; c < num_classes(p->family); ++c)
      if ((ctx->cls_mask[p->family] >> c) & 1u)
        if (!bfs_lds_bytes(p->family, ctx->V, ctx->L, has_ign, c)) return exact();
  } else {
    p->bfs = false;
    p->delta = ctx->w_min;
    p->dist64 = (uint64_t)ctx->V * ctx->w_max >= 0xFFFFFFFFull;
    // shallow graphs (sampled hop depth): rounds scale with hops, the fringe with distinct
    // distances (OPENR_SPF_GENERAL=fringe|rounds overrides)
    p->rounds = ctx->est_depth < kRoundsMaxDepth && ctx->devs[0].g.max_deg < 65535u;  // u16 in-degrees
    if (const char* e = std::getenv("OPENR_SPF_GENERAL")) {
      if (!std::strcmp(e, "fringe")) p->rounds = false;
      if (!std::strcmp(e, "rounds")) p->rounds = ctx->devs[0].g.max_deg < 65535u;
    }
    if (p->rounds && !rounds_lds_bytes(ctx->V, ctx->L, has_ign, p->nh_mode, p->dist64)) p->rounds = false;
    if (!fringe_lds_bytes(ctx->V, ctx->L, has_ign, p->nh_mode, p->dist64)) return exact();
  }
  return OPENR_SPF_OK;
}


// Uniform-cost solves run per source class (next-hop width): one class -> one launch;
// several -> a device-side partition of the batch, then one launch per class, the
// widest first.
hipError_t launch(const openr_spf_ctx* ctx, Device& d, const Plan& p, SolveArgs a, hipStream_t s) {
  LaunchInfo info;
  if (p.exact) {  // writes every dist / nh / tight word itself
    const uint64_t slot = exact_slot_bytes(d.g.V, d.g.E, d.g.L, ctx->nh_bits);
    uint64_t bytes = 0;
    if (slot > kMaxLds || std::getenv("OPENR_SPF_EXACT_GLOBAL")) {
      const uint64_t slots = std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)a.n, (uint64_t)d.num_cus * 8u,
                                                                        kExactScratchBytes / std::max<uint64_t>(slot, 1)}));
      bytes = slots * slot;
      hipError_t err = d.exscratch.reserve(bytes);
      if (err != hipSuccess) return err;
    }
    hipError_t err = reserve_counters(d);
    if (err != hipSuccess) return err;
    return launch_exact(d.g, a, d.g.w64, p.use_metric, ctx->nh_bits, d.exscratch.p, bytes, a.order,
                        d.work.p + kExactCtr, d.num_cus, s);
  }
  if (a.tight && !a.out_row) {
    hipError_t err = hipMemsetAsync(a.tight, 0, (size_t)a.n * ((d.g.E + 63u) / 64u) * 8u, s);
    if (err != hipSuccess) return err;
  }
  if (!p.bfs) {
    if (p.rounds) return launch_rounds(d.g, a, p.dist64, p.nh_mode, d.num_cus, s, &info);
    return launch_fringe(d.g, a, p.delta, p.dist64, p.nh_mode, d.num_cus, s, &info);
  }
  const int gl = (int)ctx->group_lanes;
  // a caller's list of the batch (KSP2 second SPFs: the pairs ksp_select_pairs kept) is
  // honoured by the single-class distance-only launch; every other launch partitions
  const uint32_t* list = a.perm;
  const uint32_t* list_part = a.part;
  a.perm = nullptr;
  a.part = nullptr;
  const int fam = p.family;
  uint32_t mask = ctx->cls_mask[fam];
  a.nsl = ctx->nsl[fam];
  a.dist_only = 0;
  if (fam == kFamCode && !a.nh && !a.tight) {  // distances only (KSP2 SPFs): 8-bit fields, no slices
    a.dist_only = 1;
    // OPENR_SPF_KSP_PULL=0: the target's pull test (2) one neighbour per wave (A/B, tests)
    if (const char* e = std::getenv("OPENR_SPF_KSP_PULL"))
      if (std::atoi(e) == 0) a.dist_only |= 2u;
    a.nsl = 1;
    mask = 1u << kCls8;
  }
  a.k0 = a.krows = 0;
  if (fam == kFamCode && ((mask >> kClsSliced) & 1u) && a.nh) {
    // slice scratch for at most a budget's worth of sliced solves at a time (the class runs
    // in chunks of krows): 512 MiB, OPENR_SPF_SLICE_ROWS (tests) forces a chunk size
    const uint64_t per_row = (uint64_t)a.nsl * d.g.V * sizeof(uint32_t);
    const uint64_t budget_rows = std::max<uint64_t>(1, (512ull << 20) / std::max<uint64_t>(per_row, 1));
    const uint32_t forced = (uint32_t)std::strtoul(std::getenv("OPENR_SPF_SLICE_ROWS") ? std::getenv("OPENR_SPF_SLICE_ROWS") : "0", nullptr, 10);
    const uint32_t rows = (uint32_t)std::min<uint64_t>(std::max(a.n, 1u), forced ? forced : budget_rows);
    hipError_t err = d.slicetmp.reserve((size_t)rows * a.nsl * d.g.V);
    if (err != hipSuccess) return err;
    a.slice_tmp = d.slicetmp.p;
    a.krows = rows;
  }
  if (__builtin_popcount(mask) == 1) {
    a.cls = (uint32_t)__builtin_ctz(mask);
    if (a.dist_only && list) {  // part[cls] = listed count, part[kMaxClasses + cls] = 0
      a.perm = list;
      a.part = list_part;
    }
    return launch_bfs(fam, d.g, a, p.cost, gl, d.num_cus, s, &info);
  }
  hipError_t err = d.perm.reserve(std::max<uint32_t>(a.n, 1u));
  if (err == hipSuccess) err = d.part.reserve(3u * kMaxClasses);
  if (err == hipSuccess) err = launch_partition(a.sources, a.n, fam == kFamLvl ? d.g.cls_lvl : d.g.cls, d.g.V, d.part.p,
                                                 d.perm.p, s);
  if (err != hipSuccess) return err;
  a.perm = d.perm.p;
  a.part = d.part.p;
  // classes one after another on the caller's stream (side-by-side class streams were
  // measured slower: the fork / join cost more than the overlap saved, round 3)
  const int nc = num_classes(fam);
  for (int c = nc - 1; c >= 0; --c) {
    if (!((mask >> c) & 1u)) continue;
    a.cls = (uint32_t)c;
    err = launch_bfs(fam, d.g, a, p.cost, gl, d.num_cus, s, &info);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

int check_solve_args(const openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint64_t* dist,
                     uint8_t* nh, uint32_t nh_bytes) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (n && (!sources || !dist)) return fail(OPENR_SPF_EINVAL, "null sources or dist");
  const uint32_t need = std::max<uint32_t>(1u, (ctx->nh_bits + 7u) / 8u);
  if (nh && nh_bytes < need) return fail(OPENR_SPF_EINVAL, "nh_bytes %u < required %u", nh_bytes, need);
  return OPENR_SPF_OK;
}

int solve_host(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags,
               const uint32_t* ignore_ptr, const uint32_t* ignore_links, uint64_t* dist, uint8_t* nh,
               uint32_t nh_bytes, uint64_t* tight, uint32_t* order = nullptr) {
  clear_launch_trace();
  if (order) flags |= OPENR_SPF_EMIT_ORDER;
  int rc = check_solve_args(ctx, sources, n, dist, nh, nh_bytes);
  if (rc) return rc;
  for (uint32_t i = 0; i < n; ++i)
    if (sources[i] >= ctx->V) return fail(OPENR_SPF_EINVAL, "source %u out of range (V=%u)", sources[i], ctx->V);
  if (ignore_ptr) {
    if (ignore_ptr[0] != 0) return fail(OPENR_SPF_EINVAL, "ignore_ptr[0] must be 0");
    for (uint32_t i = 0; i < n; ++i)
      if (ignore_ptr[i + 1] < ignore_ptr[i]) return fail(OPENR_SPF_EINVAL, "ignore_ptr not monotone");
    if (ignore_ptr[n] && !ignore_links) return fail(OPENR_SPF_EINVAL, "null ignore_links");
  }
  Plan plan;
  rc = make_plan(ctx, flags, ignore_ptr != nullptr, &plan);
  if (rc) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t V = ctx->V, tw = (ctx->E + 63u) / 64u;
  const uint32_t nd = (uint32_t)ctx->devs.size();
  const uint32_t per = (n + nd - 1) / std::max<uint32_t>(nd, 1);
  std::vector<uint32_t> rebased;
  for (uint32_t di = 0; di < nd; ++di) {
    Device& d = ctx->devs[di];
    const uint32_t b = std::min(n, di * per), e = std::min(n, b + per), m = e - b;
    if (!m) continue;
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(d.src.reserve(m));
    HIP_TRY(d.dist.reserve((size_t)m * V));
    if (nh) HIP_TRY(d.nh.reserve((size_t)m * V * nh_bytes));
    if (tight) HIP_TRY(d.tight.reserve((size_t)m * tw));
    if (order) HIP_TRY(d.order.reserve((size_t)m * V));
    HIP_TRY(hipMemcpyAsync(d.src.p, sources + b, m * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    SolveArgs a{};
    a.sources = d.src.p;
    a.n = m;
    if (ignore_ptr) {
      const uint32_t lb = ignore_ptr[b], le = ignore_ptr[e];
      rebased.resize(m + 1);
      for (uint32_t i = 0; i <= m; ++i) rebased[i] = ignore_ptr[b + i] - lb;
      HIP_TRY(d.ign_ptr.reserve(m + 1));
      HIP_TRY(d.ign_links.reserve(std::max<uint32_t>(le - lb, 1u)));
      HIP_TRY(hipMemcpy(d.ign_ptr.p, rebased.data(), (m + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
      if (le > lb)
        HIP_TRY(hipMemcpyAsync(d.ign_links.p, ignore_links + lb, (le - lb) * sizeof(uint32_t),
                               hipMemcpyHostToDevice, d.stream));
      a.ign_ptr = d.ign_ptr.p;
      a.ign_links = d.ign_links.p;
    }
    a.dist = d.dist.p;
    a.nh = nh ? d.nh.p : nullptr;
    a.nh_bytes = nh_bytes;
    a.tight = tight ? d.tight.p : nullptr;
    a.order = order ? d.order.p : nullptr;
    a.nh_bits = ctx->nh_bits;
    HIP_TRY(d.ovf.reserve((size_t)m * ctx->nsl_max()));
    a.ovf_list = d.ovf.p;
    HIP_TRY(reserve_counters(d));
    a.work = d.work.p;
    HIP_TRY(hipEventRecord(d.ev_begin, d.stream));
    HIP_TRY(launch(ctx, d, plan, a, d.stream));
    HIP_TRY(hipEventRecord(d.ev_end, d.stream));
    HIP_TRY(hipMemcpyAsync(dist + (size_t)b * V, d.dist.p, (size_t)m * V * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, d.stream));
    if (nh)
      HIP_TRY(hipMemcpyAsync(nh + (size_t)b * V * nh_bytes, d.nh.p, (size_t)m * V * nh_bytes,
                             hipMemcpyDeviceToHost, d.stream));
    if (tight)
      HIP_TRY(hipMemcpyAsync(tight + (size_t)b * tw, d.tight.p, (size_t)m * tw * sizeof(uint64_t),
                             hipMemcpyDeviceToHost, d.stream));
    if (order)
      HIP_TRY(hipMemcpyAsync(order + (size_t)b * V, d.order.p, (size_t)m * V * sizeof(uint32_t),
                             hipMemcpyDeviceToHost, d.stream));
  }
  double kms = 0.0;
  for (uint32_t di = 0; di < nd; ++di) {
    Device& d = ctx->devs[di];
    const uint32_t b = std::min(n, di * per), e = std::min(n, b + per);
    if (e <= b) continue;
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(hipStreamSynchronize(d.stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, d.ev_begin, d.ev_end));
    kms = std::max(kms, (double)ms);
  }
  ctx->stats.spf_runs += n;
  ctx->stats.batches += 1;
  ctx->stats.last_kernel_ms = kms;
  ctx->stats.last_batch_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return OPENR_SPF_OK;
}

// Identity array 0, 1, ..., n-1 in d.wiota (one-link ignore sets: solve k ignores exactly
// links[k]); built once and kept while it is long enough.
hipError_t ensure_iota(Device& d, size_t n, hipStream_t s) {
  if (n <= d.wiota_n) return hipSuccess;
  if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  d.wiota_n = 0;
  hipError_t e = d.wiota.reserve(n);
  if (e == hipSuccess) e = launch_iota(d.wiota.p, (uint32_t)n, d.num_cus, s);
  if (e == hipSuccess) d.wiota_n = n;
  return e;
}

// Bytes of chunk result rows a what-if sweep may hold on a device at once.
constexpr size_t kWhatifChunkBytes = size_t(1) << 30;

// Per-link-failure what-if sweep on one device (spf_sweep.hip has the unit semantics):
// base SPF with tight edges -> filter of the affected units -> chunks of single-link
// ignore-set solves through the ordinary launcher -> row comparison against the base.
// Reads the affected-unit count back (one stream sync) to size the chunks.
hipError_t whatif_on_device(openr_spf_ctx* ctx, Device& d, const Plan& base_plan, const Plan& ign_plan,
                            const uint32_t* d_links, uint32_t n_links, const uint32_t* d_sources, uint32_t n_src,
                            uint32_t* d_changed, hipStream_t s, uint32_t* solved, bool use_link_metric,
                            const WhatifDelta& dl = WhatifDelta{}) {
  const uint32_t V = ctx->V, tw = (ctx->E + 63u) / 64u;
  const uint32_t nb = std::max<uint32_t>(1u, (ctx->nh_bits + 7u) / 8u);
  *solved = 0;
  if (!n_src || !n_links) return hipSuccess;
  hipError_t err;
#define OPENR_TRY(x)              \
  do {                            \
    err = (x);                    \
    if (err != hipSuccess) return err; \
  } while (0)
  OPENR_TRY(d.base_dist.reserve((size_t)n_src * V));
  OPENR_TRY(d.base_nh.reserve((size_t)n_src * V * nb));
  OPENR_TRY(d.base_tight.reserve((size_t)n_src * tw));
  OPENR_TRY(reserve_counters(d));
  SolveArgs a{};
  a.sources = d_sources;
  a.n = n_src;
  a.dist = d.base_dist.p;
  a.nh = d.base_nh.p;
  a.nh_bytes = nb;
  a.tight = d.base_tight.p;
  a.nh_bits = ctx->nh_bits;
  OPENR_TRY(d.ovf.reserve((size_t)n_src * ctx->nsl_max()));
  a.ovf_list = d.ovf.p;
  a.work = d.work.p;
  // the rounds kernel also leaves each base row's tight in-degrees for the seeded re-solves
  const bool base_tin = base_plan.rounds && !base_plan.exact && !base_plan.bfs;
  if (base_tin) {
    OPENR_TRY(d.base_tin.reserve((size_t)n_src * V));
    a.tin_out = d.base_tin.p;
  }
  OPENR_TRY(launch(ctx, d, base_plan, a, s));
  // re-solve the `count` units listed in wsrc / wlink / wunit (ignore set = the unit's
  // link) and compare each row with its source's base row
  auto resolve_units = [&](uint32_t count, uint32_t base) -> hipError_t {
    hipError_t e2;
    const size_t row = (size_t)V * (8u + nb);
    const uint32_t chunk = (uint32_t)std::min<size_t>(count, std::max<size_t>(1, kWhatifChunkBytes / row));
    if ((e2 = d.wdist.reserve((size_t)chunk * V)) != hipSuccess) return e2;
    if ((e2 = d.wnh.reserve((size_t)chunk * V * nb)) != hipSuccess) return e2;
    if ((e2 = ensure_iota(d, (size_t)chunk + 1u, s)) != hipSuccess) return e2;
    if ((e2 = d.ovf.reserve((size_t)chunk * ctx->nsl_max())) != hipSuccess) return e2;
    for (uint32_t off0 = 0; off0 < count; off0 += chunk) {
      const uint32_t m = std::min(chunk, count - off0), off = base + off0;
      SolveArgs b{};
      b.sources = d.wsrc.p + off;
      b.n = m;
      b.ign_ptr = d.wiota.p;  // solve k ignores exactly wlink[off + k]
      b.ign_links = d.wlink.p + off;
      b.dist = d.wdist.p;
      b.nh = d.wnh.p;
      b.nh_bytes = nb;
      b.nh_bits = ctx->nh_bits;
      b.ovf_list = d.ovf.p;
      b.work = d.work.p;
      // the rounds kernel starts each unit from its source's base rows (only the nodes the
      // failed link pushes back are re-solved); other kernels solve from scratch
      b.seed_dist = d.base_dist.p;
      b.seed_tight = d.base_tight.p;
      b.seed_unit = d.wunit.p + off;
      b.seed_nsrc = n_src;
      b.seed_tin = base_tin ? d.base_tin.p : nullptr;
      // ... and compares each solve with the base rows itself (no rows through HBM)
      const bool fused = ign_plan.rounds && !ign_plan.exact && !ign_plan.bfs;
      if (fused) {
        b.seed_nh = d.base_nh.p;
        b.seed_changed = d_changed;
        b.delta = dl;
      }
      if ((e2 = launch(ctx, d, ign_plan, b, s)) != hipSuccess) return e2;
      if (!fused && (e2 = launch_rows_compare(m, V, nb, d.wdist.p, d.wnh.p, d.base_dist.p, d.base_nh.p, d.wunit.p + off, n_src,
                                    d_changed, dl, d.num_cus, s)) != hipSuccess)
        return e2;
    }
    return hipSuccess;
  };
  const char* mode = std::getenv("OPENR_SPF_WHATIF");
  const bool dist64 = use_link_metric && (uint64_t)V * ctx->w_max >= 0xFFFFFFFFull;
  // exact-order plans (metrics / widths outside the fast kernels): filter + re-solve; with
  // zero or wrapped metrics the pop order depends on every relaxation, so every unit whose
  // link is up is re-solved (no tight-edge filter)
  const bool exact = base_plan.exact || ign_plan.exact;
  if (!exact && (!mode || !std::strcmp(mode, "group"))) {
    // default: grouped repair (base rows staged once per (source, link chunk), fused filter)
    // (a unit with more dirty nodes than a wave's slots is re-solved after the launch)
    if (whatif_group_lds_bytes(V, ctx->E, nb, dist64, d.g.max_deg)) {
      const size_t units = (size_t)n_links * n_src;
      OPENR_TRY(d.wcount.reserve(3));
      OPENR_TRY(d.wsrc.reserve(units));
      OPENR_TRY(d.wlink.reserve(units));
      OPENR_TRY(d.wunit.reserve(units));
      OPENR_TRY(d.wchanged_t.reserve(units));
      OPENR_TRY(hipEventRecord(d.ev_begin, s));  // the repair kernel's own time -> stats.last_kernel_ms
      OPENR_TRY(launch_whatif_group(d.g, d_links, n_links, d_sources, n_src, d.base_dist.p, d.base_nh.p,
                                    d.base_tight.p, base_tin ? d.base_tin.p : nullptr, nb, !use_link_metric, dist64, ctx->w_max, ctx->nh_bits,
                                    d_changed, d.wchanged_t.p, d.wcount.p, d.wsrc.p, d.wlink.p, d.wunit.p,
                                    d.work.p + kIncrCtr, dl, d.num_cus, s));
      OPENR_TRY(hipEventRecord(d.ev_end, s));
      // Units past the slots are large (WAN: ~6 500 of 1.02 M affected units, ~150 dirty
      // nodes on average): re-solved, each starting from its source's base rows (the
      // rounds kernel's seeded start). On the rounds plan one launch covers them, its
      // count read on the device (wcount[1]): no host round trip between the kernels.
      const bool fused = ign_plan.rounds && !ign_plan.exact && !ign_plan.bfs;
      if (fused) {
        OPENR_TRY(ensure_iota(d, units + 1u, s));
        SolveArgs b{};
        b.sources = d.wsrc.p;
        b.n = (uint32_t)std::min<size_t>(units, 0xFFFFFFFEu);
        b.n_dev = d.wcount.p + 1;
        // two waves per solve: WAN re-solves (6 835 units, 256-thread base SPF) 64 / 128 / 256
        // threads: span 1.02 / 0.83 / 1.00 ms (more solves resident, rounds still split)
        b.n_block = 128u;
        b.ign_ptr = d.wiota.p;  // solve k ignores exactly wlink[k]
        b.ign_links = d.wlink.p;
        b.nh_bytes = nb;
        b.nh_bits = ctx->nh_bits;
        b.work = d.work.p;
        b.seed_dist = d.base_dist.p;
        b.seed_tight = d.base_tight.p;
        b.seed_unit = d.wunit.p;
        b.seed_nsrc = n_src;
        b.seed_tin = base_tin ? d.base_tin.p : nullptr;
        b.seed_nh = d.base_nh.p;
        b.seed_changed = d_changed;
        b.delta = dl;
        if (prof_enabled()) {
          OPENR_TRY(hipMallocAsync(reinterpret_cast<void**>(&b.prof_solve), 10 * units * sizeof(unsigned long long), s));
          OPENR_TRY(hipMemsetAsync(b.prof_solve, 0, 10 * units * sizeof(unsigned long long), s));
        }
        OPENR_TRY(launch(ctx, d, ign_plan, b, s));
        if (b.prof_solve) {  // tuning aid: the re-solves' phases (100 MHz wall clock) and the tail
          uint32_t nres = 0;
          OPENR_TRY(hipMemcpyAsync(&nres, d.wcount.p + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
          OPENR_TRY(hipStreamSynchronize(s));
          std::vector<unsigned long long> h(10 * (size_t)nres);
          OPENR_TRY(hipMemcpy(h.data(), b.prof_solve, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
          OPENR_TRY(hipFreeAsync(b.prof_solve, s));
          if (nres) {
            unsigned long long t0 = ~0ull, t1 = 0;
            double ph[7] = {0}, na = 0, rd = 0, rk = 0, tot = 0;
            for (uint32_t k = 0; k < nres; ++k) {
              const unsigned long long* x = &h[10 * (size_t)k];
              t0 = std::min(t0, x[0]);
              t1 = std::max(t1, x[7]);
              for (int q = 0; q < 7; ++q) ph[q] += (double)(x[q + 1] - x[q]) / 100.0;
              tot += (double)(x[7] - x[0]) / 100.0;
              na += (double)x[8];
              rd += (double)(x[9] & 0xFFFFFFFFull);
              rk += (double)(x[9] >> 32);
            }
            std::fprintf(stderr,
                         "[whatif resolve] n=%u span=%.1fus mean solve %.1fus: seed-a %.1f seed-A %.1f seed-c %.1f "
                         "dist %.1f indeg %.1f kahn %.1f compare %.1f | |A| %.1f, rounds: A+c+dist %.1f, kahn %.1f, "
                         "concurrency %.0f\n",
                         nres, (t1 - t0) / 100.0, tot / nres, ph[0] / nres, ph[1] / nres, ph[2] / nres, ph[3] / nres,
                         ph[4] / nres, ph[5] / nres, ph[6] / nres, na / nres, rd / nres, rk / nres,
                         tot / ((t1 - t0) / 100.0));
            // duration spread, its correlation with |A|, and the solves running over the span
            std::vector<double> dur(nres), asz(nres);
            for (uint32_t k = 0; k < nres; ++k) {
              dur[k] = (double)(h[10 * (size_t)k + 7] - h[10 * (size_t)k]) / 100.0;
              asz[k] = (double)h[10 * (size_t)k + 8];
            }
            std::vector<double> srt = dur;
            std::sort(srt.begin(), srt.end());
            const double md = tot / nres, ma = na / nres;
            double sxy = 0, sxx = 0, syy = 0;
            for (uint32_t k = 0; k < nres; ++k) {
              sxy += (dur[k] - md) * (asz[k] - ma);
              sxx += (dur[k] - md) * (dur[k] - md);
              syy += (asz[k] - ma) * (asz[k] - ma);
            }
            std::fprintf(stderr, "  duration p10 %.1f p50 %.1f p90 %.1f max %.1f us; corr(duration, |A|) %.2f; running at",
                         srt[nres / 10], srt[nres / 2], srt[nres * 9 / 10], srt.back(),
                         sxx > 0 && syy > 0 ? sxy / std::sqrt(sxx * syy) : 0.0);
            for (int q : {10, 25, 50, 75, 90, 95}) {
              const unsigned long long tq = t0 + (t1 - t0) * q / 100;
              uint32_t live = 0;
              for (uint32_t k = 0; k < nres; ++k) live += (h[10 * (size_t)k] <= tq && h[10 * (size_t)k + 7] > tq) ? 1u : 0u;
              std::fprintf(stderr, " %d%%:%u", q, live);
            }
            std::fprintf(stderr, "\n");
          }
        }
      }
      uint32_t cnt[2] = {0, 0};  // affected units, units past the slots
      OPENR_TRY(hipMemcpyAsync(cnt, d.wcount.p, sizeof(cnt), hipMemcpyDeviceToHost, s));
      OPENR_TRY(hipStreamSynchronize(s));
      float ms = 0.f;
      OPENR_TRY(hipEventElapsedTime(&ms, d.ev_begin, d.ev_end));
      ctx->stats.last_kernel_ms = ms;
      if (!fused && cnt[1]) OPENR_TRY(resolve_units(cnt[1], 0));
      *solved = cnt[0];
      return hipSuccess;
    }
  }
  const size_t units = (size_t)n_links * n_src;
  OPENR_TRY(d.wsrc.reserve(units));
  OPENR_TRY(d.wlink.reserve(units));
  OPENR_TRY(d.wunit.reserve(units));
  OPENR_TRY(d.wcount.reserve(1));
  const uint64_t* filter_tight = (exact && !ctx->metric_ok && use_link_metric) ? nullptr : d.base_tight.p;
  OPENR_TRY(launch_whatif_filter(d.g, d_links, n_links, d_sources, n_src, filter_tight, d_changed, d.wsrc.p,
                                 d.wlink.p, d.wunit.p, d.wcount.p, d.num_cus, s));
  uint32_t count = 0;
  OPENR_TRY(hipMemcpyAsync(&count, d.wcount.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  OPENR_TRY(hipStreamSynchronize(s));
  *solved = count;
  if (!count) return hipSuccess;
  // OPENR_SPF_WHATIF=incr: one wavefront per affected unit repairs it from the base rows it
  // re-reads (A set, distances inside A, dirty next hops); =solve re-solves every unit
  if (!exact && !dl.node && !(mode && !std::strcmp(mode, "solve")) && whatif_incr_lds_bytes(V, nb, dist64)) {
    return launch_whatif_incr(d.g, d.wsrc.p, d.wlink.p, d.wunit.p, count, n_src, d.base_dist.p, d.base_nh.p, nb,
                              !use_link_metric, dist64, d_changed, d.work.p + kIncrCtr, d.num_cus, s);
  }
  return resolve_units(count, 0);
#undef OPENR_TRY
  return hipSuccess;
}

// Bytes of second-SPF distance rows a KSP2 batch may hold on a device at once.
constexpr size_t kKspChunkBytes = size_t(8) << 30;  // second-SPF rows + ignore slots per chunk

// getKthPaths(src, dest, 1) and (.., 2) for a batch of pairs on one device: the base SPF
// of every listed source (the reference's memoized getSpfResult), then per chunk of
// pairs: k = 1 trace on the base rows (its links become the pair's ignore set), the
// second SPF with that ignore set (runSpf(src, true, ignore)), the k = 2 trace.
// Sets *overflow when a pair's paths exceed tok_cap tokens or kKspMaxDepth hops.
hipError_t ksp2_on_device(openr_spf_ctx* ctx, Device& d, const Plan& base_plan, const Plan& ign_plan,
                          const uint32_t* d_sources, uint32_t n_src, const uint32_t* d_prow, const uint32_t* d_pdst,
                          uint32_t n_pairs, uint32_t tok_cap, uint32_t* d_tok1, uint32_t* d_tok2, hipStream_t s,
                          bool* overflow) {
  const uint32_t V = ctx->V;
  *overflow = false;
  if (!n_pairs) return hipSuccess;
  hipError_t err;
#define OPENR_TRY(x)                   \
  do {                                 \
    err = (x);                         \
    if (err != hipSuccess) return err; \
  } while (0)
  OPENR_TRY(reserve_counters(d));
  OPENR_TRY(d.kbase.reserve((size_t)n_src * V));
  OPENR_TRY(d.kstatus.reserve(1));
  OPENR_TRY(hipMemsetAsync(d.kstatus.p, 0, sizeof(uint32_t), s));
  SolveArgs a{};
  a.sources = d_sources;
  a.n = n_src;
  a.dist = d.kbase.p;
  a.nh_bits = ctx->nh_bits;
  OPENR_TRY(d.ovf.reserve((size_t)n_src * ctx->nsl_max()));
  a.ovf_list = d.ovf.p;
  a.work = d.work.p;
  OPENR_TRY(launch(ctx, d, base_plan, a, s));
  // uniform cost: the base rows' pathLinks as lists, read by the k = 1 trace's frames
  // (a list read instead of a record row plus its tails' distances); up to 16 GiB
  const uint32_t* tl_off = nullptr;
  const uint2* tl_ent = nullptr;
  if (base_plan.bfs && base_plan.cost && ksp_path_lists_ok(d.g) &&
      (size_t)n_src * d.g.E * sizeof(uint2) <= (size_t(16) << 30)) {
    if (d.ktloff.reserve((size_t)n_src * (V + 1u)) == hipSuccess &&
        d.ktlent.reserve((size_t)n_src * d.g.E) == hipSuccess) {
      OPENR_TRY(launch_ksp_path_lists(d.g, d_sources, n_src, d.kbase.p, d.ktloff.p, d.ktlent.p, d.num_cus, s));
      tl_off = d.ktloff.p;
      tl_ent = d.ktlent.p;
    } else {
      (void)hipGetLastError();  // no room: the trace gathers from the records
    }
  }
  // the k = 2 trace also reads them where its pair's row keeps the base distance (same
  // uniform cost in both solves); OPENR_SPF_KSP_TL2=0: record rows only (A/B, tests)
  const char* tl2_env = std::getenv("OPENR_SPF_KSP_TL2");
  const uint32_t* tl2_off = tl_off && ign_plan.bfs && ign_plan.cost == base_plan.cost &&
                                    !(tl2_env && std::atoi(tl2_env) == 0)
                                ? tl_off
                                : nullptr;
  const uint32_t ign_cap = tok_cap;  // the k = 1 paths' links fit their tokens (slot; ends in kend)
  // the second SPF as a repair of the base rows (launch_ksp_repair): needs the k = 2 lists'
  // conditions, tagged rows, and a level mask no real level reaches; OPENR_SPF_KSP_REPAIR=0:
  // the forward, target-bounded solve (A/B, tests)
  // uniform-cost second SPFs on the code family are distance-only: u16 level rows, tagged
  // (SolveArgs::lvl_tag: a solve writes only the nodes it settles — it stops at the pair's
  // target — and the trace reads other entries as unreached) when levels leave >= 2 tag bits
  const bool rows16 = ign_plan.bfs && ign_plan.family == kFamCode;
  uint32_t lshift = 1;
  while ((1u << lshift) < V) ++lshift;  // levels < V <= 2^lshift
  const uint32_t tag_max = lshift <= 14u ? (1u << (16u - lshift)) - 1u : 0u;
  const char* tag_env = std::getenv("OPENR_SPF_KSP_TAG");  // 0: untagged rows, unreached fill (A/B)
  const bool tagged = rows16 && tag_max && !(tag_env && std::atoi(tag_env) == 0);
  const size_t row_bytes = (size_t)V * (rows16 ? 2u : 8u);
  // pairs whose k = 2 answer is empty by construction skip the second SPF and the k = 2
  // trace (ksp_select_pairs); the code family's single-class distance-only launch takes
  // the kept list. OPENR_SPF_KSP_SKIP=0: every pair solved and traced (A/B, tests).
  const char* skip_env = std::getenv("OPENR_SPF_KSP_SKIP");
  const bool skip = rows16 && !(skip_env && std::atoi(skip_env) == 0);
  const char* rep_env = std::getenv("OPENR_SPF_KSP_REPAIR");
  const bool repair = tagged && tl_off && ign_plan.bfs && ign_plan.cost == base_plan.cost && (1u << lshift) > V && ksp_repair_lds_bytes(V, d.g.L) != 0u &&
                      !(rep_env && std::atoi(rep_env) == 0);
  // pairs per chunk from a byte budget for the chunk's rows and ignore slots: 8 GiB of the
  // 288 GB, capped at half the device memory free at the call, and halved again
  // when a reservation still fails. Fabric, 512 sources x all destinations, ms per step by
  // budget: 2 GiB (~150 k pairs) 254.3, 4 GiB 248.3, 8 GiB 246.8, 16 GiB 246.4; by pairs:
  // 65 536 271.6, 32 768 297.0, 16 384 351.0, 8 192 470.8. Per-chunk launches and kernel
  // tails dominate, not the rows' cache locality. (Two pipeline lanes alternating chunks
  // over two streams measured slower, 264.7 vs 254.2 ms: each chunk's kernels already fill
  // the GPU; removed in round 4.)
  size_t chunk_budget = kKspChunkBytes;
  {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
      chunk_budget = std::min(chunk_budget, std::max<size_t>(free_b / 2u, size_t(64) << 20));
  }
  uint32_t chunk =
      (uint32_t)std::min<size_t>(n_pairs, std::max<size_t>(1, chunk_budget / (row_bytes + 4u * ign_cap)));
  if (const char* e = std::getenv("OPENR_SPF_KSP_CHUNK"))  // pairs per chunk (tests: many chunks, tag wrap)
    if (std::atoi(e) > 0) chunk = std::min<uint32_t>(chunk, (uint32_t)std::atoi(e));
  auto reserve_chunk = [&](uint32_t c) -> hipError_t {
    hipError_t e2;
    if ((e2 = d.kptr.reserve((size_t)c + 1u)) != hipSuccess) return e2;
    if (rows16) {
      if ((e2 = d.krows16.reserve((size_t)c * V)) != hipSuccess) return e2;
    } else if ((e2 = d.krows.reserve((size_t)c * V)) != hipSuccess) {
      return e2;
    }
    if ((e2 = d.kign.reserve((size_t)c * ign_cap)) != hipSuccess) return e2;
    if ((e2 = d.kend.reserve(c)) != hipSuccess) return e2;
    if ((e2 = d.kq.reserve((size_t)ksp_max_grid(d.g, d.num_cus) * (V + (V + 31u) / 32u))) != hipSuccess) return e2;
    if ((e2 = d.ksrc.reserve(c)) != hipSuccess) return e2;
    if ((e2 = d.ovf.reserve((size_t)c * ctx->nsl_max())) != hipSuccess) return e2;
    if (skip && (e2 = d.kkeep.reserve(c)) != hipSuccess) return e2;
    if ((e2 = d.kpart.reserve(4u * kMaxClasses)) != hipSuccess) return e2;
    return d.kretry.reserve(8u + 4u * (size_t)c);
  };
  for (;;) {
    err = reserve_chunk(chunk);
    if (err != hipErrorOutOfMemory || chunk == 1) break;
    (void)hipGetLastError();  // clear the failed allocation
    chunk = (chunk + 1u) / 2u;
  }
  if (err != hipSuccess) return err;
  OPENR_TRY(launch_strided_iota(d.kptr.p, chunk + 1u, ign_cap, d.num_cus, s));
  if (tagged && d.ktag_rows < (size_t)chunk * V) {  // fresh or grown buffer: no valid tag in it
    OPENR_TRY(hipMemsetAsync(d.krows16.p, 0, (size_t)chunk * V * sizeof(uint16_t), s));
    d.ktag_rows = (size_t)chunk * V;
    d.ktag = 0;
  }
  // OPENR_SPF_PROF=1: per-kind trace counters printed to stderr (tuning only)
  const uint32_t nst = ksp_stats_count();
  unsigned long long* kst = nullptr;
  if (prof_enabled()) {
    OPENR_TRY(hipMallocAsync(reinterpret_cast<void**>(&kst), 2 * nst * sizeof(unsigned long long), s));
    OPENR_TRY(hipMemsetAsync(kst, 0, 2 * nst * sizeof(unsigned long long), s));
  }
  for (uint32_t first = 0; first < n_pairs; first += chunk) {
    const uint32_t m = std::min(chunk, n_pairs - first);
    hipStream_t ls = s;
    uint32_t* rcount = d.kretry.p;  // [0] k = 1, [1] k = 2; [2..5] work counters of the 4 launches
    uint32_t* wctr = d.kretry.p + 2;
    uint32_t* rlist1 = d.kretry.p + 8;
    uint32_t* rlist2 = rlist1 + chunk;
    uint32_t* rlist3 = rlist2 + chunk;  // repaired second SPFs handed to the forward solve
    uint32_t* rmode = rlist3 + chunk;   // per pair: 0 repaired row, 1 forward row
    uint32_t* rpart3 = d.kpart.p + 2u * kMaxClasses;  // rlist3's count as the kCls8 partition
    OPENR_TRY(hipMemsetAsync(rcount, 0, 8u * sizeof(uint32_t), ls));
    // small tier (occupancy), then the full tier over the pairs it could not hold
    OPENR_TRY(launch_ksp_trace(1, d.g, d_sources, d_prow, d_pdst, first, m, d.kbase.p, d.kign.p, d.kend.p, ign_cap,
                               d_tok1, tok_cap, d.kstatus.p, d.kq.p, d.num_cus, ls, kst, nullptr, nullptr, rlist1,
                               rcount, wctr, nullptr, base_plan.bfs ? base_plan.cost : 0u, 0u, tl_off, tl_ent,
                               d.kbase.p));
    OPENR_TRY(launch_ksp_trace(1, d.g, d_sources, d_prow, d_pdst, first, m, d.kbase.p, d.kign.p, d.kend.p, ign_cap,
                               d_tok1, tok_cap, d.kstatus.p, d.kq.p, d.num_cus, ls, kst, rlist1, rcount, nullptr,
                               nullptr, wctr + 1, nullptr, base_plan.bfs ? base_plan.cost : 0u, 0u, tl_off, tl_ent,
                               d.kbase.p));
    const uint32_t* keep = nullptr;  // chunk-local pairs left for the second SPF (skip)
    const uint32_t* keep_count = nullptr;
    if (skip || repair) OPENR_TRY(hipMemsetAsync(d.kpart.p, 0, 4u * kMaxClasses * sizeof(uint32_t), ls));
    if (skip) {
      OPENR_TRY(launch_ksp_select_pairs(d.g, d_sources, d_prow, d_pdst, first, m, d_tok1, d_tok2, tok_cap, d.ksrc.p,
                                        d.kkeep.p, d.kpart.p + kCls8, d.num_cus, ls));
      keep = d.kkeep.p;
      keep_count = d.kpart.p + kCls8;
    } else {
      OPENR_TRY(launch_gather_sources(d_sources, d_prow, first, m, d.ksrc.p, d.num_cus, ls));
    }
    SolveArgs b{};
    b.sources = d.ksrc.p;
    b.n = m;
    b.perm = keep;  // launch(): the distance-only class runs over keep[0 .. *keep_count)
    b.part = skip ? d.kpart.p : nullptr;
    b.ign_ptr = d.kptr.p;  // pair k ignores kign[k * ign_cap, kend[k])
    b.ign_end = d.kend.p;
    b.ign_links = d.kign.p;
    b.dist = rows16 ? nullptr : d.krows.p;
    b.lvl16 = rows16 ? d.krows16.p : nullptr;
    uint32_t& tag = d.ktag;  // the tag of the last chunk written into this lane's rows (0: rows all zero)
    if (tagged) {
      if (tag == tag_max) {  // every tag used since the rows were zeroed: zero them again
        OPENR_TRY(hipMemsetAsync(d.krows16.p, 0, d.ktag_rows * sizeof(uint16_t), ls));
        tag = 0;
      }
      b.lvl_tag = ++tag;
      b.lvl_shift = lshift;
    }
    b.nh_bits = ctx->nh_bits;
    b.ovf_list = d.ovf.p;
    b.work = d.work.p;
    b.target = d_pdst + first;  // the k = 2 trace reads nodes no farther than dest
    if (repair) {
      OPENR_TRY(launch_ksp_repair(d.g, b.sources, d_prow + first, b.target, keep, keep_count, m, b.ign_ptr, b.ign_end,
                                  b.ign_links, d.kbase.p, tl_off, base_plan.cost, b.lvl16, b.lvl_tag << b.lvl_shift,
                                  (1u << b.lvl_shift) - 1u, rmode, rlist3, rpart3 + kCls8, d.kretry.p + 6,
                                  d.num_cus, ls));
      b.perm = rlist3;  // the pairs it handed back: the forward solve
      b.part = rpart3;
    }
    OPENR_TRY(launch(ctx, d, ign_plan, b, ls));
    const uint64_t* r2 = rows16 ? nullptr : d.krows.p;
    const uint16_t* r16 = rows16 ? d.krows16.p : nullptr;
    OPENR_TRY(launch_ksp_trace(2, d.g, d_sources, d_prow, d_pdst, first, m, r2, d.kign.p, d.kend.p, ign_cap, d_tok2,
                               tok_cap, d.kstatus.p, d.kq.p, d.num_cus, ls, kst ? kst + nst : nullptr, keep, keep_count,
                               rlist2, rcount + 1, wctr + 2, r16, ign_plan.bfs ? ign_plan.cost : 0u,
                               tagged ? (b.lvl_tag << 8 | lshift) : 0u, tl2_off, tl_ent, d.kbase.p,
                               repair ? rmode : nullptr));
    OPENR_TRY(launch_ksp_trace(2, d.g, d_sources, d_prow, d_pdst, first, m, r2, d.kign.p, d.kend.p, ign_cap, d_tok2,
                               tok_cap, d.kstatus.p, d.kq.p, d.num_cus, ls, kst ? kst + nst : nullptr, rlist2,
                               rcount + 1, nullptr, nullptr, wctr + 3, r16, ign_plan.bfs ? ign_plan.cost : 0u,
                               tagged ? (b.lvl_tag << 8 | lshift) : 0u, tl2_off, tl_ent, d.kbase.p,
                               repair ? rmode : nullptr));
  }
  if (kst) {
    std::vector<unsigned long long> h(2 * nst);
    OPENR_TRY(hipMemcpyAsync(h.data(), kst, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    OPENR_TRY(hipStreamSynchronize(s));
    OPENR_TRY(hipFree(kst));
    for (int k = 0; k < 2; ++k) {
      std::fprintf(stderr, "ksp_stats k=%d", k + 1);
      for (uint32_t i = 0; i < nst; ++i) std::fprintf(stderr, " %llu", h[k * nst + i]);
      std::fprintf(stderr, "\n");
    }
  }
  uint32_t status = 0;
  OPENR_TRY(hipMemcpyAsync(&status, d.kstatus.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  OPENR_TRY(hipStreamSynchronize(s));
  *overflow = status != 0;
#undef OPENR_TRY
  return hipSuccess;
}

int whatif_plans(openr_spf_ctx* ctx, uint32_t flags, Plan* base_plan, Plan* ign_plan) {
  int rc = make_plan(ctx, flags, false, base_plan);
  if (rc) return rc;
  return make_plan(ctx, flags, true, ign_plan);
}

// openr_spf_whatif_delta[_device] on one device: the sweep with the delta into library
// scratch (per-unit slots, WhatifDelta), the exclusive scan of changed into d_ptr, then
// (when the total fits `cap`) every unit's entries gathered into the caller's CSR arrays.
// Synchronizes s. *total = sum(changed); OPENR_SPF_E2BIG when it exceeds cap.
int whatif_delta_on_device(openr_spf_ctx* ctx, Device& d, const uint32_t* d_links, uint32_t n_links,
                           const uint32_t* d_sources, uint32_t n_src, uint32_t flags, uint32_t* d_changed,
                           uint64_t* d_ptr, uint32_t* d_node, unsigned long long* d_dist, uint8_t* d_nh, uint64_t cap,
                           uint32_t nhb, hipStream_t s, uint64_t* total, uint64_t* solved_out) {
  const uint32_t nb = std::max<uint32_t>(1u, (ctx->nh_bits + 7u) / 8u);
  if (nhb < nb) return fail(OPENR_SPF_EINVAL, "nh_bytes %u below the graph's next-hop width %u", nhb, nb);
  Plan bp, ip;
  int rc = whatif_plans(ctx, flags, &bp, &ip);
  if (rc) return rc;
  const size_t units = (size_t)n_links * n_src;
  *total = 0;
  *solved_out = 0;
  unsigned long long* ptr = reinterpret_cast<unsigned long long*>(d_ptr);
  if (!units) {
    HIP_TRY(hipMemsetAsync(ptr, 0, sizeof(unsigned long long), s));
    HIP_TRY(hipStreamSynchronize(s));
    return OPENR_SPF_OK;
  }
  // scratch pool: room for the caller's cap twice over (gaps of the waves' slot blocks,
  // grp_repair) plus one block per resident wave, at most 2^32 - 1 slots
  const uint64_t want = std::min<uint64_t>(2u * cap + (uint64_t)d.num_cus * 32u * 256u + 1024u, 0xFFFFFFFFull);
  HIP_TRY(d.dl_off.reserve(units));
  HIP_TRY(d.dl_node.reserve(want));
  HIP_TRY(d.dl_dist.reserve(want));
  HIP_TRY(d.dl_nh.reserve(want * nhb));
  HIP_TRY(d.dl_used.reserve(1));
  HIP_TRY(d.dl_tsum.reserve(units / 4096u + 1u));
  HIP_TRY(hipMemsetAsync(d.dl_used.p, 0, sizeof(unsigned long long), s));
  WhatifDelta dl;
  dl.off = d.dl_off.p;
  dl.node = d.dl_node.p;
  dl.dist = d.dl_dist.p;
  dl.nh = d.dl_nh.p;
  dl.cap = (uint32_t)want;
  dl.nhb = nhb;
  dl.used = d.dl_used.p;
  uint32_t solved = 0;
  HIP_TRY(whatif_on_device(ctx, d, bp, ip, d_links, n_links, d_sources, n_src, d_changed, s, &solved,
                           (flags & OPENR_SPF_USE_LINK_METRIC) != 0, dl));
  HIP_TRY(launch_delta_scan(d_changed, units, d.dl_tsum.p, ptr, s));
  unsigned long long tu[2] = {0, 0};  // total entries, pool slots used
  HIP_TRY(hipMemcpyAsync(&tu[0], ptr + units, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&tu[1], d.dl_used.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *total = tu[0];
  *solved_out = (uint64_t)solved + n_src;
  ctx->stats.spf_runs += *solved_out;
  ctx->stats.batches += 1;
  if (tu[1] > want)
    return fail(OPENR_SPF_E2BIG, "delta needs %llu entries (%llu pool slots; scratch %llu for cap %llu)", tu[0], tu[1],
                (unsigned long long)want, (unsigned long long)cap);
  if (tu[0] > cap) return fail(OPENR_SPF_E2BIG, "delta needs %llu entries, cap %llu", tu[0], (unsigned long long)cap);
  HIP_TRY(launch_delta_gather(d_changed, units, d.dl_off.p, ptr, dl, d_node, d_dist, d_nh, d.num_cus, s));
  HIP_TRY(hipStreamSynchronize(s));
  return OPENR_SPF_OK;
}


}  // namespace

extern "C" {

int openr_spf_abi_version(void) { return OPENR_SPF_ABI_VERSION; }

const char* openr_spf_last_error(void) { return g_last_error.c_str(); }

int openr_spf_host_alloc(size_t bytes, void** out) {
  if (!out) return fail(OPENR_SPF_EINVAL, "openr_spf_host_alloc: null out");
  *out = nullptr;
  const hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return fail(OPENR_SPF_ENOMEM, "openr_spf_host_alloc: %s", hipGetErrorString(e));
  }
  return OPENR_SPF_OK;
}

void openr_spf_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

const char* openr_spf_last_kernels(void) { return g_launch_trace.c_str(); }

void openr_spf_limits(openr_spf_limits_t* out) {
  if (!out) return;
  // Largest V whose LDS-resident BFS state (<= 8 next-hop bits, no ignore set) fits a CU.
  uint32_t lo = 1, hi = 65535;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) / 2;
    if (bfs_lds_bytes(kFamCode, mid, 0, false, kCls8)) lo = mid;
    else hi = mid - 1;
  }
  out->max_nodes = lo;
  out->max_nh_bits = 65535;  // wider than 256: the exact-order kernel
}

int openr_spf_create(const int* device_ids, int n_devices, openr_spf_ctx** out) {
  if (!out) return fail(OPENR_SPF_EINVAL, "null out");
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0)
    return fail(OPENR_SPF_ENODEV, "no HIP device available (%s); the engine has no CPU path",
                e == hipSuccess ? "count=0" : hipGetErrorString(e));
  std::vector<int> ids;
  if (!device_ids || n_devices <= 0) {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    ids.push_back(cur);
  } else {
    for (int i = 0; i < n_devices; ++i) {
      if (device_ids[i] < 0 || device_ids[i] >= count)
        return fail(OPENR_SPF_EINVAL, "device id %d out of range (count=%d)", device_ids[i], count);
      ids.push_back(device_ids[i]);
    }
  }
  auto* ctx = new (std::nothrow) openr_spf_ctx();
  if (!ctx) return fail(OPENR_SPF_ENOMEM, "out of host memory");
  for (int id : ids) {
    Device d;
    d.ordinal = id;
    hipDeviceProp_t prop;
    if (hipSetDevice(id) != hipSuccess || hipGetDeviceProperties(&prop, id) != hipSuccess ||
        hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&d.ev_begin) != hipSuccess || hipEventCreate(&d.ev_end) != hipSuccess) {
      openr_spf_destroy(ctx);
      return fail(OPENR_SPF_ENODEV, "failed to initialise HIP device %d", id);
    }
    d.num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    ctx->devs.push_back(d);
  }
  *out = ctx;
  return OPENR_SPF_OK;
}

void openr_spf_destroy(openr_spf_ctx* ctx) {
  if (!ctx) return;
  for (Device& d : ctx->devs) {
    (void)hipSetDevice(d.ordinal);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    free_graph(d.g);
    d.src.release();
    d.ign_ptr.release();
    d.ign_links.release();
    d.dist.release();
    d.tight.release();
    d.nh.release();
    d.ovf.release();
    d.slicetmp.release();
    d.work.release();
    d.status.release();
    d.perm.release();
    d.part.release();
    d.kkeep.release();
    d.ktloff.release();
    d.ktlent.release();
    d.kpart.release();
    d.dl_off.release();
    d.dl_node.release();
    d.dl_dist.release();
    d.dl_used.release();
    d.dl_nh.release();
    d.dl_tsum.release();
    d.dlo_ptr.release();
    d.dlo_dist.release();
    d.dlo_node.release();
    d.dlo_nh.release();
    void* sweep[] = {d.base_dist.p, d.base_tight.p, d.wdist.p, d.base_nh.p, d.wnh.p, d.wsrc.p, d.wlink.p,
                     d.wunit.p,     d.wcount.p,     d.wiota.p, d.base_tin.p, d.win_links.p, d.win_src.p, d.wchanged.p, d.wchanged_t.p,
                     d.kbase.p,     d.krows.p,      d.krows16.p, d.kign.p,  d.kend.p, d.ksrc.p,      d.kptr.p,    d.kstatus.p,
                     d.kin_src.p,   d.kin_row.p,    d.kin_dst.p, d.ktok1.p,   d.ktok2.p,   d.kq.p, d.kretry.p};
    for (void* p : sweep)
      if (p) (void)hipFree(p);
    d.exscratch.release();
    d.order.release();
    d.precs.release();
    d.delta.release();
    d.alist.release();
    d.asrc.release();
    d.alist2.release();
    d.asrc2.release();
    d.acount.release();
    if (d.ev_begin) (void)hipEventDestroy(d.ev_begin);
    if (d.ev_end) (void)hipEventDestroy(d.ev_end);
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete ctx;
}

int openr_spf_set_graph(openr_spf_ctx* ctx, const openr_spf_graph* gr) {
  if (!ctx || !gr) return fail(OPENR_SPF_EINVAL, "null argument");
  const uint32_t V = gr->num_nodes, E = gr->num_dir_edges, L = gr->num_links;
  if (!gr->row_ptr || !gr->node_overloaded || !gr->name_rank || (E && (!gr->col || !gr->metric || !gr->link_id ||
                                                                      !gr->edge_up)))
    return fail(OPENR_SPF_EINVAL, "null graph array");
  if (V >= kNodeSink || E >= kNodeSink) return fail(OPENR_SPF_E2BIG, "too many nodes or edges");
  if (gr->row_ptr[0] != 0 || gr->row_ptr[V] != E) return fail(OPENR_SPF_EINVAL, "row_ptr must span [0, E]");
  for (uint32_t u = 0; u < V; ++u)
    if (gr->row_ptr[u + 1] < gr->row_ptr[u]) return fail(OPENR_SPF_EINVAL, "row_ptr not monotone at %u", u);

  std::vector<uint32_t> adj(E), w(E), win(E), rev(E), lid(E), owner(E);
  std::vector<uint16_t> nbr(E);
  std::vector<uint8_t> ovl(V);
  // link id -> its two directed edges
  std::vector<uint32_t> first(L, UINT32_MAX), second(L, UINT32_MAX);
  std::vector<uint2> ledge(L);
  uint32_t nh_bits = 0, w_min = UINT32_MAX, w_max = 0;
  bool metric_ok = true;
  std::vector<uint32_t> seen_stamp(V, UINT32_MAX), seen_idx(V, 0);
  for (uint32_t u = 0; u < V; ++u) {
    ovl[u] = gr->node_overloaded[u] ? 1 : 0;
    uint32_t nd = 0;
    for (uint32_t e = gr->row_ptr[u]; e < gr->row_ptr[u + 1]; ++e) {
      const uint32_t v = gr->col[e], l = gr->link_id[e];
      if (v >= V) return fail(OPENR_SPF_EINVAL, "col[%u]=%u out of range", e, v);
      if (l >= L) return fail(OPENR_SPF_EINVAL, "link_id[%u]=%u out of range", e, l);
      owner[e] = u;
      if (seen_stamp[v] != u) {
        seen_stamp[v] = u;
        seen_idx[v] = nd++;
      }
      nbr[e] = (uint16_t)std::min<uint32_t>(seen_idx[v], 0xFFFFu);
      if (first[l] == UINT32_MAX) first[l] = e;
      else if (second[l] == UINT32_MAX) second[l] = e;
      else return fail(OPENR_SPF_EINVAL, "link %u appears more than twice", l);
      lid[e] = l;
      const bool up = gr->edge_up[e] != 0;
      adj[e] = v | (up ? 0u : kEdgeDown);
      const uint64_t m = gr->metric[e];
      w[e] = (uint32_t)std::min<uint64_t>(m, 0xFFFFFFFFull);
      if (up) {
        if (m == 0 || m > 0x7FFFFFFFull) metric_ok = false;
        else {
          w_min = std::min<uint32_t>(w_min, (uint32_t)m);
          w_max = std::max<uint32_t>(w_max, (uint32_t)m);
        }
      }
    }
    nh_bits = std::max(nh_bits, nd);
  }
  for (uint32_t l = 0; l < L; ++l) {
    if (first[l] == UINT32_MAX) continue;  // unused id
    const uint32_t a = first[l], b = second[l];
    if (b == UINT32_MAX) return fail(OPENR_SPF_EINVAL, "link %u has a single direction", l);
    if (gr->col[a] != owner[b] || gr->col[b] != owner[a])
      return fail(OPENR_SPF_EINVAL, "link %u directions do not mirror each other", l);
    if ((gr->edge_up[a] != 0) != (gr->edge_up[b] != 0))
      return fail(OPENR_SPF_EINVAL, "link %u edge_up differs by direction (Link::isUp is per link)", l);
    rev[a] = b;
    rev[b] = a;
    ledge[l] = make_uint2(a, b);
  }
  for (uint32_t e = 0; e < E; ++e) win[e] = w[rev[e]];
  for (uint32_t l = 0; l < L; ++l)
    if (first[l] == UINT32_MAX) ledge[l] = make_uint2(UINT32_MAX, UINT32_MAX);  // unused id: never affected
  // transit views: an overloaded node is reached but never expanded unless it is the
  // source (LinkState.cpp:831-838), so its transit row is empty / all-down
  std::vector<uint2> row2(V), row2t(V);
  std::vector<uint4> ellt(V), erec(E);
  for (uint32_t e = 0; e < E; ++e)
    erec[e] = make_uint4(adj[e] | (ovl[gr->col[e]] ? kNodeSink : 0u), win[e], lid[e], rev[e]);
  // rank-sorted copy of every row's in-edge records (KSP tracer, uniform cost)
  std::vector<uint32_t> erec_pos(E);
  {
    std::vector<uint32_t> idx;
    for (uint32_t u = 0; u < V; ++u) {
      const uint32_t b = gr->row_ptr[u], e1 = gr->row_ptr[u + 1];
      idx.resize(e1 - b);
      for (uint32_t e = b; e < e1; ++e) idx[e - b] = e;
      std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) {
        const uint32_t rx = gr->name_rank[gr->col[x]], ry = gr->name_rank[gr->col[y]];
        return rx != ry ? rx < ry : rev[x] < rev[y];
      });
      for (uint32_t i = 0; i < idx.size(); ++i) erec_pos[idx[i]] = b + i;
    }
  }
  for (uint32_t u = 0; u < V; ++u) {
    uint32_t x[4] = {kEdgeDown, kEdgeDown, kEdgeDown, kEdgeDown};
    if (!ovl[u])
      for (uint32_t j = 0; j < 4 && gr->row_ptr[u] + j < gr->row_ptr[u + 1]; ++j) x[j] = adj[gr->row_ptr[u] + j];
    else
      x[0] |= kNodeSink;
    ellt[u] = make_uint4(x[0], x[1], x[2], x[3]);
  }
  std::vector<uint32_t> ovl_bits((V + 31) / 32 + 1, 0);
  for (uint32_t u = 0; u < V; ++u) {
    row2[u] = make_uint2(gr->row_ptr[u], gr->row_ptr[u + 1]);
    row2t[u] = ovl[u] ? make_uint2(gr->row_ptr[u] | kNodeSink, gr->row_ptr[u]) : row2[u];
    if (ovl[u]) ovl_bits[u >> 5] |= 1u << (u & 31u);
  }
  // next-hop sets wider than 256 bits: only the exact-order kernel serves them (make_plan)
  // source class of every node (distinct degree -> next-hop width)
  std::vector<uint8_t> cls[kNumFamilies];
  uint32_t cls_mask[kNumFamilies] = {0, 0}, sliced_deg[kNumFamilies] = {0, 0};
  for (int f = 0; f < kNumFamilies; ++f) cls[f].resize(V);
  for (uint32_t u = 0; u < V; ++u) {
    uint32_t nd = 0;
    for (uint32_t e = gr->row_ptr[u]; e < gr->row_ptr[u + 1]; ++e) nd = std::max<uint32_t>(nd, nbr[e] + 1u);
    for (int f = 0; f < kNumFamilies; ++f) {
      const int c = std::max(0, src_class_for_degree(f, std::min<uint32_t>(nd, 256u)));
      cls[f][u] = (uint8_t)c;
      cls_mask[f] |= 1u << c;
      if (c == sliced_class(f)) sliced_deg[f] = std::max(sliced_deg[f], nd);
    }
  }
  for (int f = 0; f < kNumFamilies; ++f)
    if (!cls_mask[f]) cls_mask[f] = 1u;  // no node: class 0
  const FrontierEstimate est = estimate_frontier(V, gr->row_ptr, adj.data(), ovl.data());
  if (w_min == UINT32_MAX) w_min = w_max = 1;  // no usable edge

  for (Device& d : ctx->devs) {
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(hipStreamSynchronize(d.stream));
    free_graph(d.g);
    d.ktag_rows = 0;  // tagged KSP2 rows of another graph (another level width): zero before reuse
    DevGraph g;
    g.V = V;
    g.E = E;
    g.L = L;
    for (uint32_t u = 0; u < V; ++u) g.max_deg = std::max(g.max_deg, gr->row_ptr[u + 1] - gr->row_ptr[u]);
    g.est_width2 = est.width2;
    g.est_width1 = est.width1;
    g.est_depth = est.depth;
    auto up = [&](auto** dst, const auto* srcp, size_t count) -> hipError_t {
      using T = std::remove_pointer_t<std::remove_pointer_t<decltype(dst)>>;
      hipError_t err = hipMalloc(reinterpret_cast<void**>(dst), std::max<size_t>(count, 1) * sizeof(T));
      if (err != hipSuccess) return err;
      if (count) err = hipMemcpy(*dst, srcp, count * sizeof(T), hipMemcpyHostToDevice);
      return err;
    };
    hipError_t err = up(&g.row, gr->row_ptr, V + 1);
    if (err == hipSuccess) err = up(&g.row2, row2.data(), V);
    if (err == hipSuccess) err = up(&g.row2t, row2t.data(), V);
    if (err == hipSuccess) err = up(&g.ovl_bits, ovl_bits.data(), ovl_bits.size());
    if (err == hipSuccess) err = up(&g.ellt, ellt.data(), V);
    if (err == hipSuccess) {
      // [V] = sentinel row (lean BFS pass)
      std::vector<uint4> ellv(ellv_rows(V), make_uint4(V, V, V, V));
      for (uint32_t u = 0; u < V; ++u) ellv[u] = ellv_of(ellt[u], V);
      err = up(&g.ellv, ellv.data(), ellv.size());
      // delta rows (wave pass): every row of <= 4 edges and every column within 127 ids of
      // its row, down edges and overloaded rows included (a patch may bring them back)
      bool delta_ok = true;
      for (uint32_t u = 0; u < V && delta_ok; ++u) {
        delta_ok = gr->row_ptr[u + 1] - gr->row_ptr[u] <= 4u;
        for (uint32_t e = gr->row_ptr[u]; e < gr->row_ptr[u + 1] && delta_ok; ++e) {
          const int32_t dlt = (int32_t)gr->col[e] - (int32_t)u;
          delta_ok = dlt >= -127 && dlt <= 127;
        }
      }
      if (err == hipSuccess && delta_ok) {
        std::vector<uint32_t> elld(V);
        for (uint32_t u = 0; u < V; ++u) elld[u] = elld_of(ellv[u], u, V);
        err = up(&g.elld, elld.data(), V);
      }
    }
    if (err == hipSuccess) err = up(&g.erec, erec.data(), E);
    if (err == hipSuccess) {
      std::vector<uint4> erecs(E);
      for (uint32_t e = 0; e < E; ++e) erecs[erec_pos[e]] = erec[e];
      err = up(&g.erecs, erecs.data(), E);
    }
    if (err == hipSuccess) err = up(&g.adj, adj.data(), E);
    if (err == hipSuccess) err = up(&g.w, w.data(), E);
    if (err == hipSuccess) err = up(&g.w64, gr->metric, E);
    if (err == hipSuccess) err = up(&g.win, win.data(), E);
    if (err == hipSuccess) err = up(&g.rev, rev.data(), E);
    if (err == hipSuccess) err = up(&g.lid, lid.data(), E);
    if (err == hipSuccess) err = up(&g.nbr, nbr.data(), E);
    if (err == hipSuccess) err = up(&g.ovl, ovl.data(), V);
    if (err == hipSuccess) err = up(&g.cls, cls[kFamCode].data(), V);
    if (err == hipSuccess) err = up(&g.cls_lvl, cls[kFamLvl].data(), V);
    if (err == hipSuccess) err = up(&g.ledge, ledge.data(), L);
    if (err == hipSuccess) err = up(&g.rank, gr->name_rank, V);
    d.g = g;
    if (err != hipSuccess) {
      ctx->has_graph = false;
      return fail(OPENR_SPF_ENOMEM, "graph upload failed: %s", hipGetErrorString(err));
    }
  }
  ctx->V = V;
  ctx->E = E;
  ctx->L = L;
  ctx->row_ptr.assign(gr->row_ptr, gr->row_ptr + V + 1);
  ctx->col.assign(gr->col, gr->col + E);
  ctx->nh_bits = nh_bits;
  ctx->w_min = w_min;
  ctx->w_max = w_max;
  ctx->metric_ok = metric_ok;
  ctx->family = est.family();
  ctx->est_depth = est.depth;
  for (int f = 0; f < kNumFamilies; ++f) {
    ctx->cls_mask[f] = cls_mask[f];
    ctx->nsl[f] = std::max<uint32_t>(1u, (sliced_deg[f] + slice_bits(f) - 1u) / slice_bits(f));
  }
  // lanes per frontier node: enough that one pass of kBfsEdgesPerLane edges per lane
  // covers an average row (grid: 1 lane x 4 edges; fabric: 8 lanes x 4 edges)
  const uint32_t avg = V ? (E + V - 1) / V : 1;
  const uint32_t per_lane = (avg + 2 * kBfsEdgesPerLane - 1) / (2 * kBfsEdgesPerLane);  // fabric: G=4 measured best
  uint32_t gl = 1;
  while (gl < per_lane && gl < 64) gl <<= 1;
  ctx->group_lanes = gl;
  ctx->metric.assign(gr->metric, gr->metric + E);
  ctx->edge_up.assign(gr->edge_up, gr->edge_up + E);
  ctx->ovl = std::move(ovl);
  ctx->adj = std::move(adj);
  ctx->w = std::move(w);
  ctx->win = std::move(win);
  ctx->rev = std::move(rev);
  ctx->lid = std::move(lid);
  ctx->owner = std::move(owner);
  ctx->ovl_bits = std::move(ovl_bits);
  ctx->ledge = std::move(ledge);
  ctx->row2t = std::move(row2t);
  ctx->erec = std::move(erec);
  ctx->ellt = std::move(ellt);
  ctx->erec_pos = std::move(erec_pos);
  ctx->delta.clear();
  ctx->delta_index.clear();
  ctx->delta_valid = false;
  ctx->wcount.clear();
  ctx->n_bad_metric = 0;
  for (uint32_t e = 0; e < E; ++e) ctx->count_metric(e, +1);
  ctx->seen_e.assign(E, 0);
  ctx->dirty_e.assign(E, 0);
  ctx->dirty_v.assign(V, 0);
  ctx->patch_epoch = 0;
  ctx->has_graph = true;
  return OPENR_SPF_OK;
}

int openr_spf_patch_graph(openr_spf_ctx* ctx, const openr_spf_patch* p) {
  if (!ctx || !p) return fail(OPENR_SPF_EINVAL, "null argument");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if ((p->n_edges && (!p->edge_ids || !p->metric)) || (p->n_links && (!p->link_ids || !p->link_up)) ||
      (p->n_nodes && (!p->node_ids || !p->node_overloaded)))
    return fail(OPENR_SPF_EINVAL, "null patch array");
  const uint32_t V = ctx->V, E = ctx->E, L = ctx->L;
  for (uint32_t i = 0; i < p->n_edges; ++i)
    if (p->edge_ids[i] >= E) return fail(OPENR_SPF_EINVAL, "edge id %u out of range (E=%u)", p->edge_ids[i], E);
  for (uint32_t i = 0; i < p->n_links; ++i)
    if (p->link_ids[i] >= L || ctx->ledge[p->link_ids[i]].x == UINT32_MAX)
      return fail(OPENR_SPF_EINVAL, "link id %u is not a link of the graph", p->link_ids[i]);
  for (uint32_t i = 0; i < p->n_nodes; ++i)
    if (p->node_ids[i] >= V) return fail(OPENR_SPF_EINVAL, "node id %u out of range (V=%u)", p->node_ids[i], V);

  // per-patch marks: stamps of this patch (epoch wrap: clear the arrays once)
  if (++ctx->patch_epoch == 0) {
    std::fill(ctx->seen_e.begin(), ctx->seen_e.end(), 0u);
    std::fill(ctx->dirty_e.begin(), ctx->dirty_e.end(), 0u);
    std::fill(ctx->dirty_v.begin(), ctx->dirty_v.end(), 0u);
    ctx->patch_epoch = 1;
  }
  const uint32_t ep = ctx->patch_epoch;

  // 1) every directed edge whose (usable, weight, tail overload) may change, old state
  std::vector<uint32_t> cand;
  auto add = [&](uint32_t e) {
    if (ctx->seen_e[e] != ep) {
      ctx->seen_e[e] = ep;
      cand.push_back(e);
    }
  };
  for (uint32_t i = 0; i < p->n_edges; ++i) add(p->edge_ids[i]);
  for (uint32_t i = 0; i < p->n_links; ++i) {
    add(ctx->ledge[p->link_ids[i]].x);
    add(ctx->ledge[p->link_ids[i]].y);
  }
  for (uint32_t i = 0; i < p->n_nodes; ++i)
    for (uint32_t e = ctx->row_ptr[p->node_ids[i]]; e < ctx->row_ptr[p->node_ids[i] + 1]; ++e) add(e);
  auto state = [&](uint32_t e, uint32_t* wout) {
    *wout = ctx->w[e];
    return ((ctx->adj[e] & kEdgeDown) ? 0u : 1u) | (ctx->ovl[ctx->owner[e]] ? 2u : 0u);
  };
  std::vector<uint32_t> w0(cand.size()), f0(cand.size());
  for (size_t k = 0; k < cand.size(); ++k) {
    f0[k] = state(cand[k], &w0[k]);
    ctx->count_metric(cand[k], -1);  // re-counted with its new state below
  }

  // 2) apply to the host attributes; collect dirty device elements
  std::vector<uint32_t> de_list, dv_list;
  auto dirty_edge = [&](uint32_t e) {
    if (ctx->dirty_e[e] != ep) {
      ctx->dirty_e[e] = ep;
      de_list.push_back(e);
    }
  };
  auto dirty_node = [&](uint32_t u) {
    if (ctx->dirty_v[u] != ep) {
      ctx->dirty_v[u] = ep;
      dv_list.push_back(u);
    }
  };
  for (uint32_t i = 0; i < p->n_edges; ++i) {  // Link::setMetricFromNode (LinkState.cpp:195-204)
    const uint32_t e = p->edge_ids[i];
    ctx->metric[e] = p->metric[i];
    ctx->w[e] = (uint32_t)std::min<uint64_t>(p->metric[i], 0xFFFFFFFFull);
    ctx->win[ctx->rev[e]] = ctx->w[e];
    dirty_edge(e);
    dirty_edge(ctx->rev[e]);
  }
  for (uint32_t i = 0; i < p->n_links; ++i) {  // Link::isUp (LinkState.cpp:233-236), per link
    const uint2 ab = ctx->ledge[p->link_ids[i]];
    for (uint32_t e : {ab.x, ab.y}) {
      ctx->edge_up[e] = p->link_up[i] ? 1 : 0;
      ctx->adj[e] = ctx->col[e] | (p->link_up[i] ? 0u : kEdgeDown);
      dirty_edge(e);
      dirty_node(ctx->owner[e]);  // ellt
    }
  }
  for (uint32_t i = 0; i < p->n_nodes; ++i) {  // LinkState::updateNodeOverloaded / isNodeOverloaded
    const uint32_t x = p->node_ids[i];
    ctx->ovl[x] = p->node_overloaded[i] ? 1 : 0;
    dirty_node(x);
    for (uint32_t e = ctx->row_ptr[x]; e < ctx->row_ptr[x + 1]; ++e) dirty_edge(ctx->rev[e]);  // erec sink flag
  }
  for (uint32_t e : cand) ctx->count_metric(e, +1);
  // records in element order (as a full scan would emit them)
  std::sort(de_list.begin(), de_list.end());
  std::sort(dv_list.begin(), dv_list.end());

  // 3) recompute the dirty device elements exactly as set_graph derives them
  std::vector<PatchRec> recs;
  recs.reserve(6 * de_list.size() + 6 * dv_list.size());
  auto rec = [&](uint32_t arr, uint32_t idx, uint4 val) { recs.push_back(PatchRec{arr, idx, 0u, 0u, val}); };
  for (uint32_t e : de_list) {
    ctx->erec[e] = make_uint4(ctx->adj[e] | (ctx->ovl[ctx->col[e]] ? kNodeSink : 0u), ctx->win[e], ctx->lid[e],
                              ctx->rev[e]);
    rec(kPatchAdj, e, make_uint4(ctx->adj[e], 0, 0, 0));
    rec(kPatchW, e, make_uint4(ctx->w[e], 0, 0, 0));
    rec(kPatchW64, e, make_uint4((uint32_t)ctx->metric[e], (uint32_t)(ctx->metric[e] >> 32), 0, 0));
    rec(kPatchWin, e, make_uint4(ctx->win[e], 0, 0, 0));
    rec(kPatchErec, e, ctx->erec[e]);
    rec(kPatchErecS, ctx->erec_pos[e], ctx->erec[e]);
  }
  uint32_t last_word = UINT32_MAX;
  for (uint32_t u : dv_list) {
    const uint32_t rb = ctx->row_ptr[u], re = ctx->row_ptr[u + 1];
    uint32_t x4[4] = {kEdgeDown, kEdgeDown, kEdgeDown, kEdgeDown};
    if (!ctx->ovl[u])
      for (uint32_t j = 0; j < 4 && rb + j < re; ++j) x4[j] = ctx->adj[rb + j];
    else
      x4[0] |= kNodeSink;
    ctx->ellt[u] = make_uint4(x4[0], x4[1], x4[2], x4[3]);
    ctx->row2t[u] = ctx->ovl[u] ? make_uint2(rb | kNodeSink, rb) : make_uint2(rb, re);
    if (ctx->ovl[u]) ctx->ovl_bits[u >> 5] |= 1u << (u & 31u);
    else ctx->ovl_bits[u >> 5] &= ~(1u << (u & 31u));
    rec(kPatchEllt, u, ctx->ellt[u]);
    rec(kPatchEllv, u, ellv_of(ctx->ellt[u], V));
    rec(kPatchElld, u, make_uint4(elld_of(ellv_of(ctx->ellt[u], V), u, V), 0, 0, 0));
    rec(kPatchRow2t, u, make_uint4(ctx->row2t[u].x, ctx->row2t[u].y, 0, 0));
    rec(kPatchOvl, u, make_uint4(ctx->ovl[u], 0, 0, 0));
  }
  for (uint32_t u : dv_list) {  // sorted: each touched overload word once, after its bits
    if ((u >> 5) == last_word) continue;
    last_word = u >> 5;
    rec(kPatchOvlBits, last_word, make_uint4(ctx->ovl_bits[last_word], 0, 0, 0));
  }

  // 4) graph-wide metric facts (kernel choice / ENOTSUP) over the usable edges, from the
  //    metric multiset kept current above
  const bool metric_ok = ctx->n_bad_metric == 0;
  uint32_t w_min = 1, w_max = 1;  // no usable edge
  if (!ctx->wcount.empty()) {
    w_min = ctx->wcount.begin()->first;
    w_max = ctx->wcount.rbegin()->first;
  }

  // 5) the delta edges of this patch (openr_spf_refresh). Patches with no refresh in
  //    between accumulate: an edge keeps its state from before the first of them, so rows
  //    of that older graph are still filtered correctly; edges back at that state drop out.
  const bool merge = ctx->delta_valid && !ctx->refreshed;
  if (!merge) {
    ctx->delta.clear();
    ctx->delta_index.clear();
  }
  for (size_t k = 0; k < cand.size(); ++k) {
    uint32_t w1 = 0;
    const uint32_t f1 = state(cand[k], &w1);
    if (f1 == f0[k] && w1 == w0[k]) continue;
    const uint32_t e = cand[k];
    const uint32_t new_flags = ((f1 & 1u) ? kDeltaUp1 : 0u) | ((f1 & 2u) ? kDeltaOvl1 : 0u);
    auto it = ctx->delta_index.find(e);
    if (it != ctx->delta_index.end()) {  // changed by an earlier, unrefreshed patch too
      DeltaEdge& de = ctx->delta[it->second];
      de.w1 = w1;
      de.flags = (de.flags & (kDeltaUp0 | kDeltaOvl0)) | new_flags;
      continue;
    }
    DeltaEdge de{};
    de.u = ctx->owner[e];
    de.v = ctx->col[e];
    de.w0 = w0[k];
    de.w1 = w1;
    de.flags = ((f0[k] & 1u) ? kDeltaUp0 : 0u) | ((f0[k] & 2u) ? kDeltaOvl0 : 0u) | new_flags;
    de.pad0 = e;
    ctx->delta_index.emplace(e, (uint32_t)ctx->delta.size());
    ctx->delta.push_back(de);
  }
  if (merge) {  // drop edges whose accumulated change cancelled out
    size_t o = 0;
    for (size_t k = 0; k < ctx->delta.size(); ++k) {
      const DeltaEdge& de = ctx->delta[k];
      const bool same = de.w0 == de.w1 && ((de.flags & kDeltaUp0) != 0) == ((de.flags & kDeltaUp1) != 0) &&
                        ((de.flags & kDeltaOvl0) != 0) == ((de.flags & kDeltaOvl1) != 0);
      if (!same) ctx->delta[o++] = de;
    }
    ctx->delta.resize(o);
    ctx->delta_index.clear();
    for (size_t k = 0; k < o; ++k) ctx->delta_index.emplace(ctx->delta[k].pad0, (uint32_t)k);
  }

  // 6) upload: one record list + one scatter kernel per replica (measured: an event that
  //    later device-form calls wait on instead of this synchronize was no faster)
  for (Device& d : ctx->devs) {
    HIP_TRY(hipSetDevice(d.ordinal));
    if (recs.empty()) continue;
    HIP_TRY(d.precs.reserve(recs.size()));
    HIP_TRY(hipMemcpyAsync(d.precs.p, recs.data(), recs.size() * sizeof(PatchRec), hipMemcpyHostToDevice, d.stream));
    HIP_TRY(launch_patch_apply(d.g, d.precs.p, (uint32_t)recs.size(), d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));  // recs is host memory of this call
  }
  ctx->w_min = w_min;
  ctx->w_max = w_max;
  ctx->delta_all = (merge && ctx->delta_all) || !ctx->metric_ok || !metric_ok;
  ctx->metric_ok = metric_ok;
  ctx->delta_valid = true;
  ctx->refreshed = false;
  return OPENR_SPF_OK;
}

int openr_spf_refresh_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_sources, uint32_t n,
                             uint32_t flags, uint64_t* d_dist, uint8_t* d_nh, uint32_t nh_bytes, uint64_t* d_tight,
                             void* stream, uint32_t* out_resolved) {
  int rc = check_solve_args(ctx, d_sources, n, d_dist, d_nh, nh_bytes);
  if (rc) return rc;
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  if (!ctx->delta_valid)
    return fail(OPENR_SPF_EINVAL, "no patch since the last openr_spf_set_graph: rows must be re-solved");
  Plan plan;
  rc = make_plan(ctx, flags, false, &plan);
  if (rc) return rc;
  Device& d = ctx->devs[device_index];
  HIP_TRY(hipSetDevice(d.ordinal));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  const uint32_t nd = (uint32_t)ctx->delta.size();
  uint32_t count = 0;
  if (ctx->delta_all && n) {
    HIP_TRY(d.alist.reserve(n));
    HIP_TRY(launch_iota(d.alist.p, n, d.num_cus, s));
    count = n;
  } else if (nd && n) {
    HIP_TRY(d.delta.reserve(nd));
    HIP_TRY(d.alist.reserve(n));
    HIP_TRY(d.asrc.reserve(n));
    HIP_TRY(d.acount.reserve(2));
    HIP_TRY(hipMemcpyAsync(d.delta.p, ctx->delta.data(), nd * sizeof(DeltaEdge), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d.acount.p, 0, sizeof(uint32_t), s));
    HIP_TRY(launch_refresh_filter(d.delta.p, nd, d_sources, n, ctx->V, d_dist,
                                  (flags & OPENR_SPF_USE_LINK_METRIC) == 0, d.alist.p, d.asrc.p, d.acount.p,
                                  d.num_cus, s));
    // exact second stage (spf_update.hip) when next-hop rows are kept and no tight rows are:
    // of the listed rows, only those the change really moves are re-solved
    const char* ex = std::getenv("OPENR_SPF_REFRESH_EXACT");  // 0: first stage only (A/B)
    if (d_nh && !d_tight && nh_bytes <= 32u && !(ex && std::atoi(ex) == 0)) {
      HIP_TRY(d.alist2.reserve(n));
      HIP_TRY(d.asrc2.reserve(n));
      HIP_TRY(hipMemsetAsync(d.acount.p + 1, 0, sizeof(uint32_t), s));
      HIP_TRY(launch_refresh_exact(d.g, d.delta.p, nd, ctx->V, d_dist, d_nh, nh_bytes,
                                   (flags & OPENR_SPF_USE_LINK_METRIC) == 0, d.alist.p, d.asrc.p, d.acount.p, n,
                                   d.alist2.p, d.asrc2.p, d.acount.p + 1, d.num_cus, s));
      HIP_TRY(hipMemcpyAsync(&count, d.acount.p + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      std::swap(d.alist, d.alist2);  // the exact list is the one re-solved
      std::swap(d.asrc, d.asrc2);
    } else {
      HIP_TRY(hipMemcpyAsync(&count, d.acount.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));  // the affected-row count sizes the re-solve
    }
  }
  if (count) {
    if (d_tight) HIP_TRY(launch_zero_rows(d_tight, (ctx->E + 63u) / 64u, d.alist.p, count, d.num_cus, s));
    SolveArgs a{};
    a.sources = ctx->delta_all ? d_sources : d.asrc.p;
    a.n = count;
    a.out_row = d.alist.p;
    a.dist = d_dist;
    a.nh = d_nh;
    a.nh_bytes = nh_bytes;
    a.tight = d_tight;
    a.nh_bits = ctx->nh_bits;
    HIP_TRY(d.ovf.reserve((size_t)count * ctx->nsl_max()));
    a.ovf_list = d.ovf.p;
    HIP_TRY(reserve_counters(d));
    a.work = d.work.p;
    HIP_TRY(launch(ctx, d, plan, a, s));
    ctx->stats.spf_runs += count;
    ctx->stats.batches += 1;
  }
  if (out_resolved) *out_resolved = count;
  ctx->refreshed = true;  // the next patch starts a new delta
  return OPENR_SPF_OK;
}

int openr_spf_refresh(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags, uint64_t* dist,
                      uint8_t* nh, uint32_t nh_bytes, uint64_t* tight, uint32_t* out_resolved) {
  int rc = check_solve_args(ctx, sources, n, dist, nh, nh_bytes);
  if (rc) return rc;
  for (uint32_t i = 0; i < n; ++i)
    if (sources[i] >= ctx->V) return fail(OPENR_SPF_EINVAL, "source %u out of range (V=%u)", sources[i], ctx->V);
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t V = ctx->V, tw = (ctx->E + 63u) / 64u;
  const uint32_t ndev = (uint32_t)ctx->devs.size();
  const uint32_t per = (n + ndev - 1) / std::max<uint32_t>(ndev, 1);
  uint32_t total = 0;
  for (uint32_t di = 0; di < ndev; ++di) {
    Device& d = ctx->devs[di];
    const uint32_t b = std::min(n, di * per), e = std::min(n, b + per), m = e - b;
    if (!m) continue;
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(d.src.reserve(m));
    HIP_TRY(d.dist.reserve((size_t)m * V));
    if (nh) HIP_TRY(d.nh.reserve((size_t)m * V * nh_bytes));
    if (tight) HIP_TRY(d.tight.reserve((size_t)m * tw));
    HIP_TRY(hipMemcpyAsync(d.src.p, sources + b, m * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.dist.p, dist + (size_t)b * V, (size_t)m * V * 8u, hipMemcpyHostToDevice, d.stream));
    if (nh)
      HIP_TRY(hipMemcpyAsync(d.nh.p, nh + (size_t)b * V * nh_bytes, (size_t)m * V * nh_bytes, hipMemcpyHostToDevice,
                             d.stream));
    if (tight)
      HIP_TRY(hipMemcpyAsync(d.tight.p, tight + (size_t)b * tw, (size_t)m * tw * 8u, hipMemcpyHostToDevice,
                             d.stream));
    uint32_t c = 0;
    rc = openr_spf_refresh_device(ctx, (int)di, d.src.p, m, flags, d.dist.p, nh ? d.nh.p : nullptr, nh_bytes,
                                  tight ? d.tight.p : nullptr, nullptr, &c);
    if (rc) return rc;
    total += c;
    HIP_TRY(hipMemcpyAsync(dist + (size_t)b * V, d.dist.p, (size_t)m * V * 8u, hipMemcpyDeviceToHost, d.stream));
    if (nh)
      HIP_TRY(hipMemcpyAsync(nh + (size_t)b * V * nh_bytes, d.nh.p, (size_t)m * V * nh_bytes, hipMemcpyDeviceToHost,
                             d.stream));
    if (tight)
      HIP_TRY(hipMemcpyAsync(tight + (size_t)b * tw, d.tight.p, (size_t)m * tw * 8u, hipMemcpyDeviceToHost,
                             d.stream));
  }
  for (Device& d : ctx->devs) {
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(hipStreamSynchronize(d.stream));
  }
  ctx->stats.last_batch_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (out_resolved) *out_resolved = total;
  return OPENR_SPF_OK;
}

int openr_spf_nh_bytes(const openr_spf_ctx* ctx, uint32_t* out) {
  if (!ctx || !out) return fail(OPENR_SPF_EINVAL, "null argument");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set");
  *out = std::max<uint32_t>(1u, (ctx->nh_bits + 7u) / 8u);
  return OPENR_SPF_OK;
}

int openr_spf_neighbor_map(const openr_spf_ctx* ctx, uint32_t src, uint32_t* out_nbrs, uint32_t capacity,
                           uint32_t* out_count) {
  if (!ctx || !out_count) return fail(OPENR_SPF_EINVAL, "null argument");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set");
  if (src >= ctx->V) return fail(OPENR_SPF_EINVAL, "source out of range");
  uint32_t n = 0;
  for (uint32_t e = ctx->row_ptr[src]; e < ctx->row_ptr[src + 1]; ++e) {
    const uint32_t v = ctx->col[e];
    bool dup = false;
    for (uint32_t f = ctx->row_ptr[src]; f < e && !dup; ++f) dup = ctx->col[f] == v;
    if (dup) continue;
    if (out_nbrs && n < capacity) out_nbrs[n] = v;
    ++n;
  }
  *out_count = n;
  if (out_nbrs && n > capacity) return fail(OPENR_SPF_EINVAL, "capacity %u < %u neighbours", capacity, n);
  return OPENR_SPF_OK;
}

int openr_spf_solve(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags, uint64_t* dist,
                    uint8_t* nh, uint32_t nh_bytes, uint64_t* tight) {
  return solve_host(ctx, sources, n, flags, nullptr, nullptr, dist, nh, nh_bytes, tight);
}

int openr_spf_solve_order(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags,
                          const uint32_t* ignore_ptr, const uint32_t* ignore_links, uint64_t* dist, uint8_t* nh,
                          uint32_t nh_bytes, uint64_t* tight, uint32_t* order) {
  if (n && !order) return fail(OPENR_SPF_EINVAL, "null order");
  return solve_host(ctx, sources, n, flags, ignore_ptr, ignore_links, dist, nh, nh_bytes, tight, order);
}

int openr_spf_solve_ignore(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags,
                           const uint32_t* ignore_ptr, const uint32_t* ignore_links, uint64_t* dist,
                           uint8_t* nh, uint32_t nh_bytes, uint64_t* tight) {
  if (!ignore_ptr) return fail(OPENR_SPF_EINVAL, "null ignore_ptr");
  return solve_host(ctx, sources, n, flags, ignore_ptr, ignore_links, dist, nh, nh_bytes, tight);
}

int openr_spf_solve_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_sources, uint32_t n,
                           uint32_t flags, const uint32_t* d_ignore_ptr, const uint32_t* d_ignore_links,
                           uint64_t* d_dist, uint8_t* d_nh, uint32_t nh_bytes, uint64_t* d_tight, void* stream) {
  clear_launch_trace();
  int rc = check_solve_args(ctx, d_sources, n, d_dist, d_nh, nh_bytes);
  if (rc) return rc;
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  Plan plan;
  rc = make_plan(ctx, flags, d_ignore_ptr != nullptr, &plan);
  if (rc) return rc;
  Device& d = ctx->devs[device_index];
  HIP_TRY(hipSetDevice(d.ordinal));
  SolveArgs a{};
  a.sources = d_sources;
  a.n = n;
  a.ign_ptr = d_ignore_ptr;
  a.ign_links = d_ignore_links;
  a.dist = d_dist;
  a.nh = d_nh;
  a.nh_bytes = nh_bytes;
  a.tight = d_tight;
  a.nh_bits = ctx->nh_bits;
  if (flags & (OPENR_SPF_EMIT_LEVELS8 | OPENR_SPF_EMIT_LEVELS16)) {
    // level rows (the compact strong-scaling exchange): level-family uniform-cost solves
    if ((flags & OPENR_SPF_EMIT_LEVELS8) && (flags & OPENR_SPF_EMIT_LEVELS16))
      return fail(OPENR_SPF_EINVAL, "EMIT_LEVELS8 and EMIT_LEVELS16 together");
    if (plan.exact || !plan.bfs || plan.family != kFamLvl || d_tight || d_ignore_ptr)
      return fail(OPENR_SPF_ENOTSUP, "level rows need a uniform-cost graph on the level BFS family, no ignore sets "
                                     "and no tight output");
    if (!d.status.p) {
      HIP_TRY(d.status.reserve(1));
      HIP_TRY(hipMemset(d.status.p, 0, sizeof(uint32_t)));
    }
    a.lvl_rows = reinterpret_cast<uint8_t*>(d_dist);
    a.lvl_bytes = (flags & OPENR_SPF_EMIT_LEVELS8) ? 1u : 2u;
    a.status = d.status.p;
    a.dist = nullptr;
  }
  HIP_TRY(d.ovf.reserve((size_t)n * ctx->nsl_max()));
  a.ovf_list = d.ovf.p;
  HIP_TRY(reserve_counters(d));
  a.work = d.work.p;
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  HIP_TRY(launch(ctx, d, plan, a, s));
  ctx->stats.spf_runs += n;
  ctx->stats.batches += 1;
  return OPENR_SPF_OK;
}

int openr_spf_take_status(openr_spf_ctx* ctx, int device_index, uint32_t* out_status) {
  if (!ctx || !out_status) return fail(OPENR_SPF_EINVAL, "null argument");
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  Device& d = ctx->devs[device_index];
  *out_status = 0;
  if (!d.status.p) return OPENR_SPF_OK;
  HIP_TRY(hipSetDevice(d.ordinal));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out_status, d.status.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(d.status.p, 0, sizeof(uint32_t)));
  return OPENR_SPF_OK;
}

int openr_spf_whatif(openr_spf_ctx* ctx, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                     uint32_t n_sources, uint32_t flags, uint32_t* changed, uint64_t* out_solved) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if ((n_links && !links) || (n_sources && !sources) || (n_links && n_sources && !changed))
    return fail(OPENR_SPF_EINVAL, "null links, sources or changed");
  for (uint32_t i = 0; i < n_sources; ++i)
    if (sources[i] >= ctx->V) return fail(OPENR_SPF_EINVAL, "source %u out of range (V=%u)", sources[i], ctx->V);
  for (uint32_t i = 0; i < n_links; ++i)
    if (links[i] >= ctx->L) return fail(OPENR_SPF_EINVAL, "link %u out of range (L=%u)", links[i], ctx->L);
  Plan bp, ip;
  int rc = whatif_plans(ctx, flags, &bp, &ip);
  if (rc) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  // links are split in contiguous blocks across the context's devices
  const uint32_t nd = (uint32_t)ctx->devs.size();
  const uint32_t per = (n_links + nd - 1) / std::max<uint32_t>(nd, 1);
  uint64_t solved_total = 0;
  for (uint32_t di = 0; di < nd; ++di) {
    Device& d = ctx->devs[di];
    const uint32_t b = std::min(n_links, di * per), e = std::min(n_links, b + per), m = e - b;
    if (!m || !n_sources) continue;
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(d.win_links.reserve(m));
    HIP_TRY(d.win_src.reserve(n_sources));
    HIP_TRY(d.wchanged.reserve((size_t)m * n_sources));
    HIP_TRY(hipMemcpyAsync(d.win_links.p, links + b, m * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.win_src.p, sources, n_sources * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    uint32_t solved = 0;
    HIP_TRY(whatif_on_device(ctx, d, bp, ip, d.win_links.p, m, d.win_src.p, n_sources, d.wchanged.p, d.stream,
                             &solved, (flags & OPENR_SPF_USE_LINK_METRIC) != 0));
    HIP_TRY(hipMemcpyAsync(changed + (size_t)b * n_sources, d.wchanged.p, (size_t)m * n_sources * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    solved_total += solved + n_sources;
  }
  ctx->stats.spf_runs += solved_total;
  ctx->stats.batches += 1;
  ctx->stats.last_batch_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (out_solved) *out_solved = solved_total;
  return OPENR_SPF_OK;
}

int openr_spf_whatif_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_links, uint32_t n_links,
                            const uint32_t* d_sources, uint32_t n_sources, uint32_t flags, uint32_t* d_changed,
                            void* stream, uint64_t* out_solved) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  if ((n_links && !d_links) || (n_sources && !d_sources) || (n_links && n_sources && !d_changed))
    return fail(OPENR_SPF_EINVAL, "null links, sources or changed");
  Plan bp, ip;
  int rc = whatif_plans(ctx, flags, &bp, &ip);
  if (rc) return rc;
  Device& d = ctx->devs[device_index];
  HIP_TRY(hipSetDevice(d.ordinal));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  uint32_t solved = 0;
  HIP_TRY(whatif_on_device(ctx, d, bp, ip, d_links, n_links, d_sources, n_sources, d_changed, s, &solved,
                           (flags & OPENR_SPF_USE_LINK_METRIC) != 0));
  const uint64_t total = n_links && n_sources ? (uint64_t)solved + n_sources : 0u;
  ctx->stats.spf_runs += total;
  ctx->stats.batches += 1;
  if (out_solved) *out_solved = total;
  return OPENR_SPF_OK;
}

int openr_spf_whatif_delta_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_links, uint32_t n_links,
                                  const uint32_t* d_sources, uint32_t n_sources, uint32_t flags, uint32_t* d_changed,
                                  uint64_t* d_ptr, uint32_t* d_node, uint64_t* d_dist, uint8_t* d_nh, uint64_t cap,
                                  uint32_t nh_bytes, void* stream, uint64_t* out_total, uint64_t* out_solved) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  if ((n_links && !d_links) || (n_sources && !d_sources) || (n_links && n_sources && !d_changed) || !d_ptr)
    return fail(OPENR_SPF_EINVAL, "null links, sources, changed or ptr");
  if (cap && (!d_node || !d_dist || !d_nh)) return fail(OPENR_SPF_EINVAL, "null delta buffer");
  Device& d = ctx->devs[device_index];
  HIP_TRY(hipSetDevice(d.ordinal));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  uint64_t total = 0, solved = 0;
  const int rc = whatif_delta_on_device(ctx, d, d_links, n_links, d_sources, n_sources, flags, d_changed, d_ptr,
                                        d_node, reinterpret_cast<unsigned long long*>(d_dist), d_nh, cap, nh_bytes,
                                        s, &total, &solved);
  if (out_total) *out_total = total;
  if (out_solved) *out_solved = solved;
  return rc;
}

int openr_spf_whatif_delta(openr_spf_ctx* ctx, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                           uint32_t n_sources, uint32_t flags, uint32_t* changed, openr_spf_whatif_delta_t* delta,
                           uint64_t* out_solved) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (!delta || !delta->ptr) return fail(OPENR_SPF_EINVAL, "null delta or delta->ptr");
  if ((n_links && !links) || (n_sources && !sources) || (n_links && n_sources && !changed))
    return fail(OPENR_SPF_EINVAL, "null links, sources or changed");
  if (delta->cap && (!delta->node || !delta->dist || !delta->nh))
    return fail(OPENR_SPF_EINVAL, "null delta->node, dist or nh");
  for (uint32_t i = 0; i < n_sources; ++i)
    if (sources[i] >= ctx->V) return fail(OPENR_SPF_EINVAL, "source %u out of range (V=%u)", sources[i], ctx->V);
  for (uint32_t i = 0; i < n_links; ++i)
    if (links[i] >= ctx->L) return fail(OPENR_SPF_EINVAL, "link %u out of range (L=%u)", links[i], ctx->L);
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t nhb = delta->nh_bytes;
  // links split in contiguous blocks across the devices (openr_spf_whatif); each device's
  // CSR is appended to the caller's at the running total
  const uint32_t nd = (uint32_t)ctx->devs.size();
  const uint32_t per = (n_links + nd - 1) / std::max<uint32_t>(nd, 1);
  uint64_t solved_total = 0, at = 0;
  bool over = false;
  delta->ptr[0] = 0;
  std::vector<uint64_t> ptr;
  std::vector<uint32_t> idx;
  for (uint32_t di = 0; di < nd; ++di) {
    Device& d = ctx->devs[di];
    const uint32_t b = std::min(n_links, di * per), e = std::min(n_links, b + per), m = e - b;
    if (!m || !n_sources) continue;
    const size_t mu = (size_t)m * n_sources;
    HIP_TRY(hipSetDevice(d.ordinal));
    HIP_TRY(d.win_links.reserve(m));
    HIP_TRY(d.win_src.reserve(n_sources));
    HIP_TRY(d.wchanged.reserve(mu));
    HIP_TRY(d.dlo_ptr.reserve(mu + 1));
    HIP_TRY(hipMemcpyAsync(d.win_links.p, links + b, m * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.win_src.p, sources, n_sources * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
    // the device's entries land in library buffers sized to the room left in the caller's
    const uint64_t room = delta->cap > at ? delta->cap - at : 0;
    HIP_TRY(d.dlo_node.reserve(std::max<uint64_t>(room, 1)));
    HIP_TRY(d.dlo_dist.reserve(std::max<uint64_t>(room, 1)));
    HIP_TRY(d.dlo_nh.reserve(std::max<uint64_t>(room * nhb, 1)));
    uint64_t total = 0, solved = 0;
    int rc = whatif_delta_on_device(ctx, d, d.win_links.p, m, d.win_src.p, n_sources, flags, d.wchanged.p,
                                    reinterpret_cast<uint64_t*>(d.dlo_ptr.p), d.dlo_node.p, d.dlo_dist.p, d.dlo_nh.p,
                                    room, nhb, d.stream, &total, &solved);
    if (rc && rc != OPENR_SPF_E2BIG) return rc;
    over |= rc == OPENR_SPF_E2BIG;
    solved_total += solved;
    ptr.resize(mu + 1);
    HIP_TRY(hipMemcpyAsync(changed + (size_t)b * n_sources, d.wchanged.p, mu * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           d.stream));
    HIP_TRY(hipMemcpyAsync(ptr.data(), d.dlo_ptr.p, (mu + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    const bool fits = !over && total <= room;
    if (fits && total) {
      HIP_TRY(hipMemcpyAsync(delta->node + at, d.dlo_node.p, total * 4u, hipMemcpyDeviceToHost, d.stream));
      HIP_TRY(hipMemcpyAsync(delta->dist + at, d.dlo_dist.p, total * 8u, hipMemcpyDeviceToHost, d.stream));
      HIP_TRY(hipMemcpyAsync(delta->nh + at * nhb, d.dlo_nh.p, total * nhb, hipMemcpyDeviceToHost, d.stream));
    }
    HIP_TRY(hipStreamSynchronize(d.stream));
    for (size_t u = 0; u < mu; ++u) {
      const size_t gu = (size_t)b * n_sources + u;
      delta->ptr[gu + 1] = at + ptr[u + 1];
      const uint32_t c = (uint32_t)(ptr[u + 1] - ptr[u]);
      if (!fits || c < 2) continue;
      // each unit's nodes ascending (the device keeps the repair's order)
      const uint64_t o = at + ptr[u];
      bool sorted = true;
      for (uint32_t k = 1; k < c && sorted; ++k) sorted = delta->node[o + k - 1] < delta->node[o + k];
      if (sorted) continue;
      idx.resize(c);
      for (uint32_t k = 0; k < c; ++k) idx[k] = k;
      std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return delta->node[o + x] < delta->node[o + y]; });
      std::vector<uint32_t> tn(c);
      std::vector<uint64_t> td(c);
      std::vector<uint8_t> th((size_t)c * nhb);
      for (uint32_t k = 0; k < c; ++k) {
        tn[k] = delta->node[o + idx[k]];
        td[k] = delta->dist[o + idx[k]];
        std::memcpy(&th[(size_t)k * nhb], delta->nh + (o + idx[k]) * nhb, nhb);
      }
      std::memcpy(delta->node + o, tn.data(), c * 4u);
      std::memcpy(delta->dist + o, td.data(), c * 8u);
      std::memcpy(delta->nh + o * nhb, th.data(), (size_t)c * nhb);
    }
    at += total;
  }
  ctx->stats.last_batch_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (out_solved) *out_solved = solved_total;
  if (over || at > delta->cap)
    return fail(OPENR_SPF_E2BIG, "delta needs %llu entries, cap %llu (ptr and changed are filled, entries are not)",
                (unsigned long long)at, (unsigned long long)delta->cap);
  return OPENR_SPF_OK;
}

int openr_spf_ksp2(openr_spf_ctx* ctx, const uint32_t* src, const uint32_t* dst, uint32_t n_pairs,
                   uint32_t tok_cap, uint32_t* tok1, uint32_t* tok2) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (n_pairs && (!src || !dst || !tok1 || !tok2)) return fail(OPENR_SPF_EINVAL, "null argument");
  if (tok_cap < 1) return fail(OPENR_SPF_EINVAL, "tok_cap must be >= 1");
  if (!ksp_lds_bytes(ctx->V, ctx->L, ctx->devs[0].g.max_deg))
    return fail(OPENR_SPF_E2BIG, "too many links (%u) for the KSP tracer", ctx->L);
  if (!ctx->metric_ok)  // the tracer walks dist[u] + w == dist[v]: ambiguous under zero metrics
    return fail(OPENR_SPF_ENOTSUP, "KSP2 needs usable metrics in [1, 2^31-1]");
  // distinct sources (the memoized SPF of each), pair -> base row
  std::vector<uint32_t> srcs, prow(n_pairs), row_of(ctx->V, UINT32_MAX);
  for (uint32_t i = 0; i < n_pairs; ++i) {
    if (src[i] >= ctx->V || dst[i] >= ctx->V) return fail(OPENR_SPF_EINVAL, "pair %u out of range", i);
    if (row_of[src[i]] == UINT32_MAX) {
      row_of[src[i]] = (uint32_t)srcs.size();
      srcs.push_back(src[i]);
    }
    prow[i] = row_of[src[i]];
  }
  Plan bp, ip;
  int rc = whatif_plans(ctx, OPENR_SPF_USE_LINK_METRIC, &bp, &ip);  // getKthPaths uses link metrics
  if (rc) return rc;
  if (!n_pairs) return OPENR_SPF_OK;
  const auto t0 = std::chrono::steady_clock::now();
  Device& d = ctx->devs[0];
  HIP_TRY(hipSetDevice(d.ordinal));
  HIP_TRY(d.kin_src.reserve(srcs.size()));
  HIP_TRY(d.kin_row.reserve(n_pairs));
  HIP_TRY(d.kin_dst.reserve(n_pairs));
  HIP_TRY(d.ktok1.reserve((size_t)n_pairs * tok_cap));
  HIP_TRY(d.ktok2.reserve((size_t)n_pairs * tok_cap));
  HIP_TRY(hipMemcpyAsync(d.kin_src.p, srcs.data(), srcs.size() * 4u, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(hipMemcpyAsync(d.kin_row.p, prow.data(), (size_t)n_pairs * 4u, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(hipMemcpyAsync(d.kin_dst.p, dst, (size_t)n_pairs * 4u, hipMemcpyHostToDevice, d.stream));
  bool overflow = false;
  HIP_TRY(ksp2_on_device(ctx, d, bp, ip, d.kin_src.p, (uint32_t)srcs.size(), d.kin_row.p, d.kin_dst.p, n_pairs,
                         tok_cap, d.ktok1.p, d.ktok2.p, d.stream, &overflow));
  HIP_TRY(hipMemcpyAsync(tok1, d.ktok1.p, (size_t)n_pairs * tok_cap * 4u, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipMemcpyAsync(tok2, d.ktok2.p, (size_t)n_pairs * tok_cap * 4u, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  ctx->stats.spf_runs += srcs.size() + n_pairs;
  ctx->stats.batches += 1;
  ctx->stats.last_batch_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (overflow)
    return fail(OPENR_SPF_E2BIG, "a pair's paths exceed tok_cap=%u tokens or %u hops (marked 0xFFFFFFFF)", tok_cap,
                kKspMaxDepth - 1u);
  return OPENR_SPF_OK;
}

int openr_spf_ksp2_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_sources, uint32_t n_sources,
                          const uint32_t* d_pair_row, const uint32_t* d_pair_dst, uint32_t n_pairs, uint32_t tok_cap,
                          uint32_t* d_tok1, uint32_t* d_tok2, void* stream) {
  if (!ctx) return fail(OPENR_SPF_EINVAL, "null context");
  if (!ctx->has_graph) return fail(OPENR_SPF_EINVAL, "no graph set (openr_spf_set_graph)");
  if (device_index < 0 || device_index >= (int)ctx->devs.size())
    return fail(OPENR_SPF_EINVAL, "device_index %d out of range", device_index);
  if (n_pairs && (!d_sources || !d_pair_row || !d_pair_dst || !d_tok1 || !d_tok2))
    return fail(OPENR_SPF_EINVAL, "null argument");
  if (tok_cap < 1) return fail(OPENR_SPF_EINVAL, "tok_cap must be >= 1");
  if (!ksp_lds_bytes(ctx->V, ctx->L, ctx->devs[0].g.max_deg))
    return fail(OPENR_SPF_E2BIG, "too many links (%u) for the KSP tracer", ctx->L);
  if (!ctx->metric_ok)  // the tracer walks dist[u] + w == dist[v]: ambiguous under zero metrics
    return fail(OPENR_SPF_ENOTSUP, "KSP2 needs usable metrics in [1, 2^31-1]");
  Plan bp, ip;
  int rc = whatif_plans(ctx, OPENR_SPF_USE_LINK_METRIC, &bp, &ip);
  if (rc) return rc;
  Device& d = ctx->devs[device_index];
  HIP_TRY(hipSetDevice(d.ordinal));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  bool overflow = false;
  HIP_TRY(ksp2_on_device(ctx, d, bp, ip, d_sources, n_sources, d_pair_row, d_pair_dst, n_pairs, tok_cap, d_tok1,
                         d_tok2, s, &overflow));
  ctx->stats.spf_runs += (uint64_t)n_sources + n_pairs;
  ctx->stats.batches += 1;
  if (overflow)
    return fail(OPENR_SPF_E2BIG, "a pair's paths exceed tok_cap=%u tokens or %u hops (marked 0xFFFFFFFF)", tok_cap,
                kKspMaxDepth - 1u);
  return OPENR_SPF_OK;
}

int openr_spf_get_stats(const openr_spf_ctx* ctx, openr_spf_stats_t* out) {
  if (!ctx || !out) return fail(OPENR_SPF_EINVAL, "null argument");
  *out = ctx->stats;
  return OPENR_SPF_OK;
}

}  // extern "C"
