// spf_kernels.hip — gfx950 kernels of the OpenR SPF engine.
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

#include <cstdlib>

#include "spf_device.h"

namespace openr_spf {

namespace {
using namespace dev;


template <typename LT>
struct BfsLayout {
  uint32_t lvl, vis, nh, ring, ovl, ign, total;
};

// ring = frontier queue (power of two, wraps) in the fast path, or the full BFS-order
// array (capacity V, never wraps) in the fallback path.
template <typename LT>
__host__ __device__ inline BfsLayout<LT> bfs_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t nh_words,
                                                    uint32_t ring_cap) {
  BfsLayout<LT> l;
  uint32_t off = 16;  // control: append counters [0..2], overflow flag [3]
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.lvl = take((uint32_t)sizeof(LT) * (V + 4u));
  l.vis = take(4u * ((V + 31u) / 32u));
  l.nh = take(4u * nh_words);
  l.ring = take(2u * ring_cap);
  l.ovl = take(4u * ((V + 31u) / 32u));
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.total = off;
  return l;
}

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
// Uniform-cost kernel: level-synchronous BFS (one source per workgroup)
// ---------------------------------------------------------------------------
// LDS per solve: lvl[] (LT, all-ones = not reached), a visited bitmap, next-hop
// bitsets and the frontier queue. The source is expanded first (level 0 -> 1, next
// hops = the neighbour itself); then level L expands queue slots [head, tail):
// groups of G lanes per frontier node, K edges per lane loaded ahead (rows of degree
// <= 4 come from one 16-byte ELL load when G == 1). Edge u->v is tight iff
// lvl[v] > L (all tight preds of v sit on level L); the tight arrival ORs nh(u) into
// nh(v) and stores lvl[v] = L+1 (idempotent); ds_or_rtn on the visited bitmap elects
// the one arrival that appends v (one LDS atomic per wave per pass for the slots).
// One barrier per level; append counters are triple-buffered.
//   RING = true : LT = u8, queue = power-of-two ring; a solve whose two adjacent
//                 levels exceed the ring, or whose depth exceeds 253, sets ovf[sid].
//   RING = false: LT = u16, queue = full BFS order (capacity V).
// rerun != 0: only solves with ovf[sid] == rerun (flagged by the previous variant).
template <typename LT>
struct LvlOps;
template <>
struct LvlOps<uint8_t> {
  static constexpr uint32_t kUnset = 0xFFu;
};
template <>
struct LvlOps<uint16_t> {
  static constexpr uint32_t kUnset = 0xFFFFu;
};

template <int MODE, int K, typename LT, bool RING, bool ELL, bool GENERIC>
__global__ __launch_bounds__(kBlock) void bfs_kernel(DevGraph g, SolveArgs a, uint64_t cost, uint32_t glog,
                                                     uint32_t has_ign_rt, uint32_t ring_cap, uint32_t rerun) {
  // GENERIC = false: no ignore set and no tight-edge output (compile-time), the
  // all-sources / prefetch case; GENERIC = true handles both at run time.
  const bool has_ign = GENERIC && has_ign_rt != 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  using N = Nh<MODE>;
  using O = LvlOps<LT>;
  const uint32_t V = g.V, tid = threadIdx.x, wave = tid >> 6;
  const uint32_t nh_words = N::words(V);
  const BfsLayout<LT> lay = bfs_layout<LT>(V, g.L, has_ign != 0, nh_words, ring_cap);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  LT* lvl = reinterpret_cast<LT*>(base + lay.lvl);
  uint32_t* lvl_w = reinterpret_cast<uint32_t*>(base + lay.lvl);
  uint32_t* vis = reinterpret_cast<uint32_t*>(base + lay.vis);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint16_t* ring = reinterpret_cast<uint16_t*>(base + lay.ring);
  uint32_t* ovl = reinterpret_cast<uint32_t*>(base + lay.ovl);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  const uint32_t bit_words = (V + 31u) / 32u;
  const uint32_t lvl_words = ((uint32_t)sizeof(LT) * (V + 4u)) / 4u;
  const uint32_t ign_words = (g.L + 31u) / 32u;
  const uint32_t G = 1u << glog, ngroups = kBlock >> glog, groups_per_wave = 64u >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  const uint32_t tight_words = (g.E + 63u) / 64u;
  const uint32_t rmask = ring_cap - 1u;  // RING: ring_cap is a power of two

  for (uint32_t i = tid; i < bit_words; i += kBlock) ovl[i] = g.ovl_bits[i];

  for (uint32_t sid = blockIdx.x; sid < a.n; sid += gridDim.x) {
    if (rerun && a.ovf[sid] != rerun) continue;  // block-uniform
    const uint32_t src = a.sources[sid];
    for (uint32_t i = tid; i < lvl_words; i += kBlock) lvl_w[i] = 0xFFFFFFFFu;
    for (uint32_t i = tid; i < bit_words; i += kBlock) vis[i] = 0;
    for (uint32_t i = tid; i < nh_words; i += kBlock) nh[i] = 0;
    if (has_ign)
      for (uint32_t i = tid; i < ign_words; i += kBlock) ign[i] = 0;
    if (tid < 4) ctl[tid] = 0;
    __syncthreads();
    if (has_ign) load_ignore(ign, ign_words, a, sid, g.L);
    if (tid == 0) {
      lvl[src] = 0;
      vis[src >> 5] = 1u << (src & 31u);
    }
    __syncthreads();
    uint64_t* trow = (GENERIC && a.tight) ? a.tight + (size_t)sid * tight_words : nullptr;

    // level 0: expand the source; a directly connected node's next hop is itself
    {
      const uint2 rs = g.row2[src];
      for (uint32_t e0 = rs.x; e0 < rs.y; e0 += kBlock) {
        const uint32_t e = e0 + tid;
        bool fresh = false;
        uint32_t v = 0;
        if (e < rs.y) {
          const uint32_t av = g.adj[e];
          v = av & ~kEdgeDown;
          if (!(av & kEdgeDown) && !(has_ign && test_bit(ign, g.lid[e])) && v != src) {
            const uint32_t bit = 1u << (v & 31u);
            fresh = !(atomicOr(&vis[v >> 5], bit) & bit);
            lvl[v] = (LT)1;
            N::or_bit(nh, v, g.nbr[e]);
            if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[e >> 6]), 1ull << (e & 63u));
          }
        }
        // level-0 appends count in ctl[0]; level L >= 1 uses ctl[L % 3] (ctl[1] first)
        const uint32_t slot = 1u + wave_append(fresh, &ctl[0]);
        if (fresh) ring[slot] = (uint16_t)v;  // slot < 1 + deg(src) <= ring_cap checked by the host
      }
    }
    __syncthreads();

    uint32_t head = 1, tail = 1u + ctl[0], L = 1;
    bool overflow = false;  // block-uniform
    while (head < tail) {
      if (RING && L + 1u >= O::kUnset) {  // next level not representable in u8
        overflow = true;
        break;
      }
      uint32_t* cnt = &ctl[L % 3u];
      if (tid == 0) ctl[(L + 1u) % 3u] = 0;  // last read two barriers ago
      for (uint32_t fb = head; fb < tail; fb += ngroups) {
        if (fb + wave * groups_per_wave >= tail) continue;  // this wave has no slice (uniform)
        const uint32_t idx = fb + group;
        uint32_t u = 0, beg = 0, end = 0;
        uint4 ell = make_uint4(kEdgeDown, kEdgeDown, kEdgeDown, kEdgeDown);
        if (idx < tail) {
          u = ring[RING ? (idx & rmask) : idx];
          if (!test_bit(ovl, u)) {  // overloaded non-source nodes are sinks (LinkState.cpp:831-838)
            const uint2 r = g.row2[u];
            beg = r.x;
            end = r.y;
            if (ELL) ell = g.ell[u];
          }
        }
        const typename N::Val nhu = N::load(nh, u);  // final: u was reached a level ago
        for (uint32_t e0 = beg + lane_g; __any(e0 < end); e0 += G * K) {
          uint32_t av[K], lv[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t e = e0 + j * G;
            if (ELL && e0 == beg) {
              av[j] = j == 0 ? ell.x : j == 1 ? ell.y : j == 2 ? ell.z : ell.w;
            } else {
              av[j] = e < end ? g.adj[e] : kEdgeDown;
            }
            lv[j] = (has_ign && e < end) ? g.lid[e] : 0u;
          }
          uint32_t fresh_mask = 0;
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t e = e0 + j * G;
            const uint32_t v = av[j] & ~kEdgeDown;
            const bool ok = !(av[j] & kEdgeDown) && e < end && !(has_ign && test_bit(ign, lv[j]));
            if (ok && (uint32_t)lvl[v] > L) {
              // tight edge: first or equal-cost arrival (LinkState.cpp:857-873)
              const uint32_t bit = 1u << (v & 31u);
              fresh_mask |= (atomicOr(&vis[v >> 5], bit) & bit) ? 0u : (1u << j);
              lvl[v] = (LT)(L + 1u);
              N::or_val(nh, v, nhu);  // addNextHops(nh(u))
              if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[e >> 6]), 1ull << (e & 63u));
            }
          }
          uint32_t total;
          uint32_t slot = wave_prefix_small((uint32_t)__popc(fresh_mask), &total);
          uint32_t wbase = 0;
          if (total) {
            const int leader = __ffsll((long long)__ballot(fresh_mask != 0)) - 1;
            if ((int)__lane_id() == leader) wbase = atomicAdd(cnt, total);
            wbase = __shfl(wbase, leader);
          }
          slot += tail + wbase;
#pragma unroll
          for (int j = 0; j < K; ++j) {
            if ((fresh_mask >> j) & 1u) {
              const uint32_t v = av[j] & ~kEdgeDown;
              if (!RING) {
                ring[slot] = (uint16_t)v;
              } else if (slot - head < ring_cap) {
                ring[slot & rmask] = (uint16_t)v;
              } else {
                ctl[3] = 1;  // two adjacent levels exceed the ring
              }
              ++slot;
            }
          }
        }
      }
      __syncthreads();
      head = tail;
      tail += *cnt;
      ++L;
      if (RING && ctl[3]) {  // ring overflow; ctl[3] is uniform after the barrier
        overflow = true;
        break;
      }
    }
    if (RING && overflow) {  // re-run by the u16 / full-order variant
      if (tid == 0) a.ovf[sid] = (uint8_t)(rerun + 1u);
      __syncthreads();
      continue;
    }

    uint64_t* drow = a.dist + (size_t)sid * V;
    for (uint32_t v = tid; v < V; v += kBlock) {
      const uint32_t l = lvl[v];
      drow[v] = l != O::kUnset ? (uint64_t)l * cost : ~0ull;
    }
    if (a.nh) {
      const uint32_t nb = a.nh_bytes;
      uint8_t* nrow = a.nh + (size_t)sid * V * nb;
      if (MODE == kNhByte && nb == 1 && ((reinterpret_cast<uintptr_t>(nrow) | V) & 3u) == 0) {
        uint32_t* nrow32 = reinterpret_cast<uint32_t*>(nrow);
        for (uint32_t i = tid; i < V / 4u; i += kBlock) nrow32[i] = nh[i];
      } else {
        const uint32_t total = V * nb;
        for (uint32_t i = tid; i < total; i += kBlock) {
          const uint32_t v = i / nb, j = i - v * nb;
          nrow[i] = (uint8_t)N::byte(nh, v, j);
        }
      }
    }
    __syncthreads();
  }
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

template <int MODE>
uint32_t nh_words_host(uint32_t V) {
  return Nh<MODE>::words(V);
}

uint32_t nh_words_for(int mode, uint32_t V) {
  switch (mode) {
    case kNhByte: return nh_words_host<kNhByte>(V);
    case kNhHalf: return nh_words_host<kNhHalf>(V);
    case kNhW1: return nh_words_host<kNhW1>(V);
    case kNhW2: return nh_words_host<kNhW2>(V);
    case kNhW4: return nh_words_host<kNhW4>(V);
    case kNhW8: return nh_words_host<kNhW8>(V);
  }
  return 0;
}

uint32_t blocks_for(uint32_t n, uint32_t lds, int num_cus) {
  uint32_t per_cu = lds ? kMaxLds / lds : 8;
  if (per_cu > 8) per_cu = 8;  // 8 x 256 threads = 2048 threads per CU
  if (per_cu < 1) per_cu = 1;
  uint64_t g = (uint64_t)num_cus * per_cu;
  if (g > n) g = n;
  return (uint32_t)(g ? g : 1);
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

int nh_mode_for_bits(uint32_t bits) {
  if (bits <= 8) return kNhByte;
  if (bits <= 16) return kNhHalf;
  if (bits <= 32) return kNhW1;
  if (bits <= 64) return kNhW2;
  if (bits <= 128) return kNhW4;
  if (bits <= 256) return kNhW8;
  return -1;
}

uint32_t nh_mode_lds_bytes(int mode, uint32_t V) { return 4u * nh_words_for(mode, V); }

uint32_t bfs_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode) {
  // the full-order u16 variant must fit (it re-runs solves the fast path flags)
  if (V > 65535u) return 0;
  uint32_t t = bfs_layout<uint16_t>(V, L, has_ignore, nh_words_for(nh_mode, V), V).total;
  return t <= kMaxLds ? t : 0;
}

uint32_t bucket_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64) {
  if (V > 65535u) return 0;
  uint32_t t = bucket_layout(V, L, has_ignore, nh_words_for(nh_mode, V), dist64 ? 8u : 4u).total;
  return t <= kMaxLds ? t : 0;
}

namespace {
template <int MODE, typename LT, bool RING, bool ELL>
hipError_t launch_bfs_variant(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                              uint32_t ring_cap, uint32_t rerun, int num_cus, hipStream_t s, LaunchInfo* info) {
  constexpr int K = (int)kBfsEdgesPerLane;
  const uint32_t lds = bfs_layout<LT>(g.V, g.L, has_ign, nh_words_for(MODE, g.V), ring_cap).total;
  const uint32_t grid = blocks_for(a.n, lds, num_cus);
  const bool generic = has_ign || a.tight != nullptr;
  auto k = generic ? bfs_kernel<MODE, K, LT, RING, ELL, true> : bfs_kernel<MODE, K, LT, RING, ELL, false>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  if (info && !rerun) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = RING ? "bfs_kernel<ring,u8>" : "bfs_kernel<full,u16>";
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, s, g, a, cost, glog, (uint32_t)has_ign, ring_cap, rerun);
  return hipGetLastError();
}

// Fast path: u8 levels + a ring sized so that kBfsTargetWgs workgroups fit a CU.
// It cannot be used when its ring would be smaller than kMinRing entries; then the
// full-order u16 variant runs directly.
uint32_t fast_ring_cap(const DevGraph& g, bool has_ign, int mode) {
  if (const char* e = std::getenv("OPENR_SPF_BFS_FULL"))  // tuning: force the full-order variant
    if (e[0] == '1') return 0;
  const uint32_t fixed = bfs_layout<uint8_t>(g.V, g.L, has_ign, nh_words_for(mode, g.V), 0).total;
  const uint32_t budget = kMaxLds / kBfsTargetWgs;
  if (fixed >= budget) return 0;
  uint32_t cap = 1;
  while (cap * 2u <= (budget - fixed) / 2u && cap < 8192u) cap *= 2u;
  return (cap >= 256u && cap > g.max_deg + 1u) ? cap : 0u;
}

template <int MODE, bool ELL>
hipError_t launch_bfs_mode(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                           uint32_t first_rerun, int num_cus, hipStream_t s, LaunchInfo* info) {
  // ring/u8 variant first (or as the re-run of flagged multi-source batches); solves it
  // flags are re-run by the full-order u16 variant on the same stream
  const uint32_t cap = fast_ring_cap(g, has_ign, MODE);
  if (!cap)
    return launch_bfs_variant<MODE, uint16_t, false, ELL>(g, a, cost, glog, has_ign, g.V, first_rerun, num_cus, s,
                                                          info);
  const bool may_overflow = g.V > cap || g.V > 254u;
  hipError_t err =
      launch_bfs_variant<MODE, uint8_t, true, ELL>(g, a, cost, glog, has_ign, cap, first_rerun, num_cus, s, info);
  if (err != hipSuccess || !may_overflow) return err;
  return launch_bfs_variant<MODE, uint16_t, false, ELL>(g, a, cost, glog, has_ign, g.V, first_rerun + 1u, num_cus,
                                                        s, info);
}
}  // namespace

hipError_t launch_bfs(const DevGraph& g, const SolveArgs& a, uint64_t cost, int nh_mode, int group_lanes,
                      int num_cus, hipStream_t s, LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  if (!bfs_lds_bytes(g.V, g.L, has_ign, nh_mode)) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  if (!a.ovf) return hipErrorInvalidValue;
  hipError_t err = hipMemsetAsync(a.ovf, 0, a.n, s);
  if (err != hipSuccess) return err;
  if (a.tight) {
    err = hipMemsetAsync(a.tight, 0, (size_t)a.n * ((g.E + 63u) / 64u) * 8u, s);
    if (err != hipSuccess) return err;
  }
  uint32_t glog = 0;
  while ((1 << glog) < group_lanes && glog < 6) ++glog;
  const bool ell = glog == 0 && g.ell != nullptr;
  // bit-parallel multi-source BFS when eligible; its overflowing batches fall through
  uint32_t first_rerun = 0;
  const MsPlan ms = plan_msbfs(g, a.n, a.nh_bits, has_ign, a.tight != nullptr, num_cus);
  if (ms.use && a.scratch && a.scratch_bytes >= ms.scratch) {
    err = launch_msbfs(g, a, cost, a.nh_bits ? a.nh_bits : 1u, ms.lanes, group_lanes, ms.cap, a.scratch, ms.grid, s,
                       info);
    if (err != hipSuccess) return err;
    first_rerun = 1;
  }
#define OPENR_BFS_MODE(M)                                                                               \
  case M:                                                                                               \
    return ell ? launch_bfs_mode<M, true>(g, a, cost, glog, has_ign, first_rerun, num_cus, s, info)      \
               : launch_bfs_mode<M, false>(g, a, cost, glog, has_ign, first_rerun, num_cus, s, info);
  switch (nh_mode) {
    OPENR_BFS_MODE(kNhByte)
    OPENR_BFS_MODE(kNhHalf)
    OPENR_BFS_MODE(kNhW1)
    OPENR_BFS_MODE(kNhW2)
    OPENR_BFS_MODE(kNhW4)
    OPENR_BFS_MODE(kNhW8)
  }
#undef OPENR_BFS_MODE
  return hipErrorInvalidValue;
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
