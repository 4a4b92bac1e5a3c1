// spf_kernels.hip — general-metric kernel of the OpenR SPF engine and shared launch
// helpers (the uniform-cost BFS kernel is in spf_bfs.hip, the bit-parallel
// multi-source BFS in spf_msbfs.hip).
//
// Semantics restated from LinkState::runSpf (/root/reference/openr/decision/
// LinkState.cpp:808-882) in closed form for strictly positive metrics
// (SURVEY.md Appendix A.3):
//   dist  = shortest distance over usable edges, no transit through overloaded
//           nodes other than the source;
//   nh(v) = OR over tight in-edges u->v of (u == src ? {v} : nh(u)).
// The reference's heap order (metric, name) only matters for pathLinks order,
// which the host rebuilds from the tight-edge mask (include/openr_spf.h).
//
// Kernel shapes (one 256-thread workgroup = one solve, persistent over the batch):
//   bfs_kernel     uniform edge cost: level-synchronous BFS. Frontier = a slice of
//                  the BFS-order array in LDS; groups of G lanes expand one frontier
//                  node each; first-visit detection by ds_or on a visited bitmap;
//                  appends are wave-aggregated (ballot + one ds_add per wave);
//                  next-hop sets are OR-ed into LDS bitsets as edges are relaxed.
//   bucket_kernel  general positive metrics: buckets [m, m + delta), delta = the
//                  minimum usable metric, are settle-safe (no edge can land inside
//                  its own bucket), so each bucket is finalised in one step:
//                  pull next-hops over tight in-edges, push ds_min relaxations.
// No MFMA: min-plus relaxation is not a matrix contraction; the bound is the CSR
// stream and the result write (DESIGN.md "Roofline").
#include "spf_kernels.h"

#include <algorithm>
#include <cstdlib>

#include "spf_device.h"

namespace openr_spf {

namespace {
using namespace dev;


struct BucketLayout {
  uint32_t dist, settled, list, nh, ign, total;
};

__host__ __device__ inline BucketLayout bucket_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t nh_words,
                                                      uint32_t dist_bytes) {
  BucketLayout l;
  uint32_t off = 32;  // control: count, pad, 64-bit min
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.dist = take(dist_bytes * V);
  l.settled = take(4u * ((V + 31u) / 32u));
  l.list = take(2u * V);
  l.nh = take(4u * nh_words);
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.total = off;
  return l;
}

// ---------------------------------------------------------------------------
// General-metric kernel: settle-safe buckets + pull next-hops
// ---------------------------------------------------------------------------
template <typename D>
__device__ __forceinline__ D wave_min(D x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    D y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}

template <int MODE, typename D>
__global__ __launch_bounds__(kBlock) void bucket_kernel(DevGraph g, SolveArgs a, uint32_t delta, uint32_t glog,
                                                        uint32_t has_ign) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  using N = Nh<MODE>;
  constexpr D INF = (D)~(D)0;
  const uint32_t V = g.V, tid = threadIdx.x;
  const uint32_t nh_words = N::words(V);
  const BucketLayout lay = bucket_layout(V, g.L, has_ign != 0, nh_words, sizeof(D));
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;                                               // [0] list count
  D* s_min = reinterpret_cast<D*>(base + 16);                         // bucket floor
  D* dist = reinterpret_cast<D*>(base + lay.dist);
  uint32_t* settled = reinterpret_cast<uint32_t*>(base + lay.settled);
  uint16_t* list = reinterpret_cast<uint16_t*>(base + lay.list);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  const uint32_t set_words = (V + 31u) / 32u;
  const uint32_t ign_words = (g.L + 31u) / 32u;
  const uint32_t G = 1u << glog, ngroups = kBlock >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  const uint32_t tight_words = (g.E + 63u) / 64u;

  for (uint32_t sid = blockIdx.x; sid < a.n; sid += gridDim.x) {
    const uint32_t src = a.sources[sid];
    for (uint32_t v = tid; v < V; v += kBlock) dist[v] = INF;
    for (uint32_t i = tid; i < set_words; i += kBlock) settled[i] = 0;
    for (uint32_t i = tid; i < nh_words; i += kBlock) nh[i] = 0;
    if (has_ign)
      for (uint32_t i = tid; i < ign_words; i += kBlock) ign[i] = 0;
    if (tid == 0) {
      ctl[0] = 0;
      *s_min = INF;
    }
    __syncthreads();
    if (has_ign) load_ignore(ign, ign_words, a, sid, g.L);
    if (tid == 0) dist[src] = 0;
    __syncthreads();
    uint64_t* trow = a.tight ? a.tight + (size_t)sid * tight_words : nullptr;

    for (;;) {
      // (a) floor of the next bucket: min tentative distance among unsettled nodes
      D local = INF;
      for (uint32_t v = tid; v < V; v += kBlock)
        if (!test_bit(settled, v)) local = dist[v] < local ? dist[v] : local;
      local = wave_min(local);
      if (__lane_id() == 0 && local != INF) atomicMin(s_min, local);
      __syncthreads();
      const D m = *s_min;
      if (m == INF) break;
      const uint64_t hi = (uint64_t)m + delta;  // bucket [m, m + delta)
      // (b) collect the bucket (every member's distance is final)
      for (uint32_t v0 = 0; v0 < V; v0 += kBlock) {
        const uint32_t v = v0 + tid;
        const bool in = v < V && !test_bit(settled, v) && (uint64_t)dist[v] < hi;
        const uint32_t slot = wave_append(in, &ctl[0]);
        if (in) list[slot] = (uint16_t)v;
      }
      __syncthreads();
      const uint32_t cnt = ctl[0];
      // (c) per bucket member: pull next-hops over tight in-edges, push relaxations
      for (uint32_t fb = 0; fb < cnt; fb += ngroups) {
        const uint32_t idx = fb + group;
        uint32_t v = 0, beg = 0, end = 0;
        D dv = 0;
        bool expand = false;
        if (idx < cnt) {
          v = list[idx];
          dv = dist[v];
          beg = g.row[v];
          end = g.row[v + 1];
          expand = (v == src) || !g.ovl[v];
        }
        for (uint32_t e = beg + lane_g; e < end; e += G) {
          const uint32_t av = g.adj[e];
          if ((av & kEdgeDown) || (has_ign && test_bit(ign, g.lid[e]))) continue;
          const uint32_t u = av;
          // pull: in-edge u->v is tight (LinkState.cpp:857-873 closed form)
          if (v != src) {
            const D du = dist[u];
            if (du != INF && (uint64_t)du + g.win[e] == (uint64_t)dv && (u == src || !g.ovl[u])) {
              const uint32_t re = g.rev[e];
              if (u == src)
                N::or_bit(nh, v, g.nbr[re]);
              else
                N::or_from(nh, v, u);
              if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[re >> 6]), 1ull << (re & 63u));
            }
          }
          // push: relax v->u
          if (expand && !test_bit(settled, u)) {
            const D cand = dv + (D)g.w[e];
            if (cand < dist[u]) atomicMin(&dist[u], cand);
          }
        }
      }
      __syncthreads();
      for (uint32_t i = tid; i < cnt; i += kBlock) {
        const uint32_t v = list[i];
        atomicOr(&settled[v >> 5], 1u << (v & 31u));
      }
      if (tid == 0) {
        ctl[0] = 0;
        *s_min = INF;
      }
      __syncthreads();
    }

    uint64_t* drow = a.dist + (size_t)sid * V;
    for (uint32_t v = tid; v < V; v += kBlock) drow[v] = dist[v] == INF ? ~0ull : (uint64_t)dist[v];
    if (a.nh) {
      const uint32_t nb = a.nh_bytes;
      uint8_t* nrow = a.nh + (size_t)sid * V * nb;
      const uint32_t total = V * nb;
      for (uint32_t i = tid; i < total; i += kBlock) {
        const uint32_t v = i / nb, j = i - v * nb;
        nrow[i] = (uint8_t)N::byte(nh, v, j);
      }
    }
    __syncthreads();
  }
}

template <typename K>
hipError_t launch_common(K kernel, uint32_t lds, uint32_t grid, hipStream_t s, const SolveArgs& a,
                         const DevGraph& g) {
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  if (a.tight) {
    err = hipMemsetAsync(a.tight, 0, (size_t)a.n * ((g.E + 63u) / 64u) * 8u, s);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

}  // namespace

template <int MODE>
uint32_t nh_words_host(uint32_t V) {
  return Nh<MODE>::words(V);
}

uint32_t nh_words_for(int mode, uint32_t V) {
  switch (mode) {
    case kNhNibble: return nh_words_host<kNhNibble>(V);
    case kNhByte: return nh_words_host<kNhByte>(V);
    case kNhHalf: return nh_words_host<kNhHalf>(V);
    case kNhW1: return nh_words_host<kNhW1>(V);
    case kNhW2: return nh_words_host<kNhW2>(V);
    case kNhW4: return nh_words_host<kNhW4>(V);
    case kNhW8: return nh_words_host<kNhW8>(V);
  }
  return 0;
}

uint32_t blocks_for(uint32_t n, uint32_t lds, int num_cus, uint32_t block) {
  const uint32_t max_wg = 2048u / block;  // 2048 threads (32 waves) per CU
  uint32_t per_cu = lds ? kMaxLds / lds : max_wg;
  if (per_cu > max_wg) per_cu = max_wg;
  if (per_cu < 1) per_cu = 1;
  uint64_t g = (uint64_t)num_cus * per_cu;
  if (g > n) g = n;
  return (uint32_t)(g ? g : 1);
}

bool nh_mode_single(int mode) {
  return mode == kNhNibble || mode == kNhByte || mode == kNhHalf || mode == kNhW1;
}

int src_class_for_degree(int family, uint32_t d) {
  if (d > 256) return -1;
  if (family == kFamLvl) {
    if (d <= 4) return kLvl4;
    if (d <= 8) return kLvl8;
    if (d <= 16) return kLvl16;
    if (d <= 32) return kLvl32;
    return kLvlSliced;
  }
  if (d <= 5) return kCls8;
  if (d <= 13) return kCls16;
  if (d <= 24) return kCls32;
  return kClsSliced;
}

int num_classes(int family) { return family == kFamLvl ? kNumLvlClasses : kNumClasses; }
int sliced_class(int family) { return family == kFamLvl ? kLvlSliced : kClsSliced; }
uint32_t slice_bits(int family) { return family == kFamLvl ? 32u : 24u; }

uint32_t bfs_lds_bytes(int family, uint32_t V, uint32_t L, bool has_ignore, int cls) {
  return family == kFamLvl ? bfs_lvl_lds_bytes(V, L, has_ignore, cls) : bfs_code_lds_bytes(V, L, has_ignore, cls);
}

hipError_t launch_bfs(int family, const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes,
                      int num_cus, hipStream_t s, LaunchInfo* info) {
  return family == kFamLvl ? launch_bfs_lvl(g, a, cost, group_lanes, num_cus, s, info)
                           : launch_bfs_code(g, a, cost, group_lanes, num_cus, s, info);
}

namespace {
// Wave-aggregated class histogram / scatter of a source batch (one atomic per class
// per wave). part = [counts | offsets | cursors], each kMaxClasses u32, zeroed by the
// launcher.
__global__ __launch_bounds__(256) void partition_count(const uint32_t* src, uint32_t n, const uint8_t* cls,
                                                       uint32_t V, uint32_t* part) {
  for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t u = i < n ? src[i] : V;
    const uint32_t c = u < V ? cls[u] : 0u;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      const unsigned long long m = __ballot(i < n && c == k);
      if (m && __lane_id() == (uint32_t)(__ffsll((long long)m) - 1)) atomicAdd(&part[k], (uint32_t)__popcll(m));
    }
  }
}

__global__ __launch_bounds__(256) void partition_scatter(const uint32_t* src, uint32_t n, const uint8_t* cls,
                                                         uint32_t V, uint32_t* part, uint32_t* perm) {
  __shared__ uint32_t off[kMaxClasses];
  if (threadIdx.x == 0) {
    uint32_t o = 0;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      off[k] = o;
      o += part[k];
      if (blockIdx.x == 0) part[kMaxClasses + k] = off[k];
    }
  }
  __syncthreads();
  const uint32_t lane = __lane_id();
  for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t u = i < n ? src[i] : V;
    const uint32_t c = u < V ? cls[u] : 0u;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      const unsigned long long m = __ballot(i < n && c == k);
      if (!m) continue;
      const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&part[2u * kMaxClasses + k], (uint32_t)__popcll(m));
      base = __shfl(base, (int)leader);
      if (i < n && c == k) perm[off[k] + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
    }
  }
}
}  // namespace

hipError_t launch_partition(const uint32_t* d_sources, uint32_t n, const uint8_t* d_node_cls, uint32_t V,
                            uint32_t* d_part, uint32_t* d_perm, hipStream_t s) {
  hipError_t err = hipMemsetAsync(d_part, 0, 3u * kMaxClasses * sizeof(uint32_t), s);
  if (err != hipSuccess || n == 0) return err;
  const uint32_t grid = std::min<uint32_t>((n + 255u) / 256u, 1024u);
  hipLaunchKernelGGL(partition_count, dim3(grid), dim3(256), 0, s, d_sources, n, d_node_cls, V, d_part);
  err = hipGetLastError();
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(partition_scatter, dim3(grid), dim3(256), 0, s, d_sources, n, d_node_cls, V, d_part, d_perm);
  return hipGetLastError();
}

int nh_mode_for_bits(uint32_t bits) {
  if (bits <= 4) return kNhNibble;
  if (bits <= 8) return kNhByte;
  if (bits <= 16) return kNhHalf;
  if (bits <= 32) return kNhW1;
  if (bits <= 64) return kNhW2;
  if (bits <= 128) return kNhW4;
  if (bits <= 256) return kNhW8;
  return -1;
}

uint32_t nh_mode_lds_bytes(int mode, uint32_t V) { return 4u * nh_words_for(mode, V); }

uint32_t bucket_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64) {
  if (V > 65535u) return 0;
  uint32_t t = bucket_layout(V, L, has_ignore, nh_words_for(nh_mode, V), dist64 ? 8u : 4u).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_bucket(const DevGraph& g, const SolveArgs& a, uint32_t delta, bool dist64, int nh_mode,
                         int num_cus, hipStream_t s, LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  const uint32_t lds = bucket_lds_bytes(g.V, g.L, has_ign, nh_mode, dist64);
  if (!lds || delta == 0) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  const uint32_t avg = g.V ? (g.E + g.V - 1) / g.V : 1;
  uint32_t glog = 0;
  while ((1u << glog) < avg && glog < 6) ++glog;
  const uint32_t grid = blocks_for(a.n, lds, num_cus);
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = dist64 ? "bucket_kernel<u64>" : "bucket_kernel<u32>";
  }
#define OPENR_BUCKET_CASE(M)                                                                      \
  case M: {                                                                                       \
    if (dist64) {                                                                                 \
      auto k = bucket_kernel<M, unsigned long long>;                                              \
      hipError_t err = launch_common(k, lds, grid, s, a, g);                                      \
      if (err != hipSuccess) return err;                                                          \
      hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, s, g, a, delta, glog, (uint32_t)has_ign); \
    } else {                                                                                      \
      auto k = bucket_kernel<M, uint32_t>;                                                        \
      hipError_t err = launch_common(k, lds, grid, s, a, g);                                      \
      if (err != hipSuccess) return err;                                                          \
      hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, s, g, a, delta, glog, (uint32_t)has_ign); \
    }                                                                                             \
    return hipGetLastError();                                                                     \
  }
  switch (nh_mode) {
    OPENR_BUCKET_CASE(kNhNibble)
    OPENR_BUCKET_CASE(kNhByte)
    OPENR_BUCKET_CASE(kNhHalf)
    OPENR_BUCKET_CASE(kNhW1)
    OPENR_BUCKET_CASE(kNhW2)
    OPENR_BUCKET_CASE(kNhW4)
    OPENR_BUCKET_CASE(kNhW8)
  }
#undef OPENR_BUCKET_CASE
  return hipErrorInvalidValue;
}

}  // namespace openr_spf
