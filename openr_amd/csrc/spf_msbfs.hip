// spf_msbfs.hip — bit-parallel multi-source BFS (uniform edge cost).
//
// One workgroup solves a batch of B sources (B = 8 or 16) at once: every node v
// carries B-bit lane masks in LDS (bit s <-> source s of the batch):
//   seen[v]    lanes that have reached v at a level <= L (snapshot during a level)
//   cur[v]     lanes for which v is on the current frontier
//   nxt[v]     lanes reaching v for the first time at level L+1 (accumulated)
//   P[j][v]    next-hop planes: bit s set <=> the s-th source's j-th distinct
//              neighbour is in nextHops(v) (j < D <= 8)
// so one level iteration relaxes an edge for all B sources with a few bitwise ops.
// Semantics are those of the per-source kernel (LinkState.cpp:808-882 closed form):
//   nh_s(v) = OR over tight preds u of (u == src_s ? {v} : nh_s(u)); with unit cost the
//   tight preds of v for lane s are exactly the frontier nodes u with s in cur[u].
// Levels reached are written as bytes to a per-workgroup global scratch [V][B] and
// turned into u64 distance rows (coalesced) at the end of the batch.
// Not used for ignore sets / tight-edge output (per-source kernels handle those);
// a batch whose frontier exceeds the LDS list, or that is deeper than 253 levels,
// flags its solves (ovf = 1) for the per-source kernels.
#include "spf_kernels.h"

#include <algorithm>
#include <cstdlib>

#include "spf_device.h"

namespace openr_spf {
namespace {
using namespace dev;

template <typename TB>
struct Lanes {
  static constexpr uint32_t B = 8u * sizeof(TB);
  static constexpr uint32_t kPer = 4u / sizeof(TB);
  static constexpr uint32_t kMask = B == 32 ? 0xFFFFFFFFu : ((1u << (B & 31u)) - 1u);
  static __host__ __device__ uint32_t words(uint32_t V) { return (V + kPer - 1u) / kPer; }
  static __device__ uint32_t shift(uint32_t v) { return (v % kPer) * B; }
  static __device__ uint32_t get(const uint32_t* a, uint32_t v) { return (a[v / kPer] >> shift(v)) & kMask; }
  // returns v's bits before the OR
  static __device__ uint32_t fetch_or(uint32_t* a, uint32_t v, uint32_t x) {
    const uint32_t sh = shift(v);
    return (atomicOr(&a[v / kPer], x << sh) >> sh) & kMask;
  }
  static __device__ void or_(uint32_t* a, uint32_t v, uint32_t x) { atomicOr(&a[v / kPer], x << shift(v)); }
  static __device__ void clear(uint32_t* a, uint32_t v) { atomicAnd(&a[v / kPer], ~(kMask << shift(v))); }
};

struct MsLayout {
  uint32_t seen, cur, nxt, planes, list0, list1, ovl, src, total;
};

template <typename TB>
__host__ __device__ inline MsLayout ms_layout(uint32_t V, uint32_t D, uint32_t cap) {
  MsLayout l;
  uint32_t off = 32;  // control: [0..2] list counters (triple-buffered), [3] overflow
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  const uint32_t wb = 4u * Lanes<TB>::words(V);
  l.seen = take(wb);
  l.cur = take(wb);
  l.nxt = take(wb);
  l.planes = take(wb * D);
  l.list0 = take(2u * cap);
  l.list1 = take(2u * cap);
  l.ovl = take(4u * ((V + 31u) / 32u));
  l.src = take(4u * Lanes<TB>::B);
  l.total = off;
  return l;
}

template <typename TB, int K, int BLOCK>
__global__ __launch_bounds__(BLOCK) void msbfs_kernel(DevGraph g, SolveArgs a, uint64_t cost, uint32_t D,
                                                      uint32_t glog, uint32_t cap, uint8_t* scratch) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  using LN = Lanes<TB>;
  constexpr uint32_t B = LN::B;
  const uint32_t V = g.V, tid = threadIdx.x;
  const MsLayout lay = ms_layout<TB>(V, D, cap);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  uint32_t* seen = reinterpret_cast<uint32_t*>(base + lay.seen);
  uint32_t* cur = reinterpret_cast<uint32_t*>(base + lay.cur);
  uint32_t* nxt = reinterpret_cast<uint32_t*>(base + lay.nxt);
  uint32_t* planes = reinterpret_cast<uint32_t*>(base + lay.planes);
  uint16_t* lists[2] = {reinterpret_cast<uint16_t*>(base + lay.list0), reinterpret_cast<uint16_t*>(base + lay.list1)};
  uint32_t* ovl = reinterpret_cast<uint32_t*>(base + lay.ovl);
  uint32_t* srcs = reinterpret_cast<uint32_t*>(base + lay.src);
  const uint32_t W = LN::words(V);
  const uint32_t bit_words = (V + 31u) / 32u;
  const uint32_t G = 1u << glog, ngroups = BLOCK >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  uint8_t* scr = scratch + (size_t)blockIdx.x * V * B;  // [V][B] reached level per lane

  for (uint32_t i = tid; i < bit_words; i += BLOCK) ovl[i] = g.ovl_bits[i];

  const uint32_t nbatches = (a.n + B - 1u) / B;
  for (uint32_t bt = blockIdx.x; bt < nbatches; bt += gridDim.x) {
    const uint32_t sid0 = bt * B;
    const uint32_t nl = min(B, a.n - sid0);
    for (uint32_t i = tid; i < W; i += BLOCK) {  // regions are 16-byte padded: clear each
      seen[i] = 0;
      cur[i] = 0;
      nxt[i] = 0;
    }
    for (uint32_t i = tid; i < D * W; i += BLOCK) planes[i] = 0;
    if (tid < 4) ctl[tid] = 0;
    if (tid < B) srcs[tid] = tid < nl ? a.sources[sid0 + tid] : 0xFFFFFFFFu;
    __syncthreads();
    if (tid < nl) {  // level 0: every lane's source, deduplicated into the first list
      const uint32_t u = srcs[tid];
      LN::or_(seen, u, 1u << tid);
      if (LN::fetch_or(cur, u, 1u << tid) == 0) lists[0][atomicAdd(&ctl[0], 1u)] = (uint16_t)u;
      scr[(size_t)u * B + tid] = 0;
    }
    __syncthreads();

    uint32_t cnt = ctl[0], L = 0, which = 0;
    bool overflow = false;
    while (cnt > 0) {
      if (L + 1u >= 255u) {  // level bytes would wrap
        overflow = true;
        break;
      }
      const uint16_t* fl = lists[which];
      uint16_t* nl_list = lists[which ^ 1u];
      uint32_t* ncnt = &ctl[(L + 1u) % 3u];
      if (tid == 0) ctl[(L + 2u) % 3u] = 0;  // counter of level L+2 (last read two barriers ago)
      // Phase A: push the frontier's lane masks over usable edges
      for (uint32_t fb = 0; fb < cnt; fb += ngroups) {
        const uint32_t idx = fb + group;
        uint32_t u = 0, m = 0, beg = 0, end = 0;
        if (idx < cnt) {
          u = fl[idx];
          m = LN::get(cur, u);
          // an overloaded node is a sink except as its lanes' source (level 0 only)
          if (L > 0 && test_bit(ovl, u)) m = 0;
          if (m) {
            const uint2 r = g.row2[u];
            beg = r.x;
            end = r.y;
          }
        }
        uint32_t pu[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pu[j] = (m && L > 0 && (uint32_t)j < D) ? LN::get(planes + j * W, u) : 0u;
        for (uint32_t e0 = beg + lane_g; __any(e0 < end); e0 += G * K) {
          uint32_t av[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t e = e0 + j * G;
            av[j] = e < end ? g.adj[e] : kEdgeDown;
          }
          uint32_t nfresh = 0, fv[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            fv[j] = 0xFFFFFFFFu;
            if (av[j] & kEdgeDown) continue;
            const uint32_t v = av[j];
            const uint32_t nw = m & ~LN::get(seen, v);  // lanes for which u->v is tight
            if (!nw) continue;
            if (LN::fetch_or(nxt, v, nw) == 0) {
              fv[j] = v;
              ++nfresh;
            }
            if (L == 0) {
              LN::or_(planes + (uint32_t)g.nbr[e0 + j * G] * W, v, nw);  // directly connected: {v}
            } else {
#pragma unroll
              for (int jj = 0; jj < 8; ++jj) {
                const uint32_t x = pu[jj] & nw;  // addNextHops(nh(u)) per lane
                if (x) LN::or_(planes + jj * W, v, x);
              }
            }
          }
          uint32_t total;
          uint32_t slot = wave_prefix_small(nfresh, &total);
          uint32_t wbase = 0;
          if (total) {
            const int leader = __ffsll((long long)__ballot(nfresh != 0)) - 1;
            if ((int)__lane_id() == leader) wbase = atomicAdd(ncnt, total);
            wbase = __shfl(wbase, leader);
          }
          slot += wbase;
#pragma unroll
          for (int j = 0; j < K; ++j) {
            if (fv[j] != 0xFFFFFFFFu) {
              if (slot < cap) nl_list[slot] = (uint16_t)fv[j];
              else ctl[3] = 1;
              ++slot;
            }
          }
        }
      }
      __syncthreads();
      const uint32_t ncount = *ncnt;
      if (ctl[3]) {
        overflow = true;
        break;
      }
      // Phase B: fold the new lanes into seen, make them the next frontier, record levels
      for (uint32_t i = tid; i < ncount; i += BLOCK) {
        const uint32_t v = nl_list[i];
        const uint32_t n = LN::get(nxt, v);
        LN::clear(nxt, v);
        LN::or_(seen, v, n);
        LN::clear(cur, v);
        LN::or_(cur, v, n);
        uint8_t* row = scr + (size_t)v * B;
        for (uint32_t bits = n; bits; bits &= bits - 1u) row[__ffs(bits) - 1] = (uint8_t)(L + 1u);
      }
      __syncthreads();
      cnt = ncount;
      which ^= 1u;
      ++L;
    }
    if (overflow) {  // per-source kernels re-run this batch
      if (tid < nl) a.ovf[sid0 + tid] = 1;
      __syncthreads();
      continue;
    }
    // make this workgroup's scratch bytes visible to all its waves: drain the stores,
    // barrier, then drop the CU's L1 copy before reading (agent-scope acquire)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __syncthreads();
    const uint32_t nb = a.nh_bytes;
    for (uint32_t v = tid; v < V; v += BLOCK) {
      const uint32_t sv = LN::get(seen, v);
      uint8_t lv[B];
      if (B == 16) {
        const uint4 q = *reinterpret_cast<const uint4*>(scr + (size_t)v * B);
        const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (uint32_t s = 0; s < B; ++s) lv[s] = (uint8_t)(w4[s >> 2] >> (8u * (s & 3u)));
      } else {
        const uint2 q = *reinterpret_cast<const uint2*>(scr + (size_t)v * B);
        const uint32_t w2[2] = {q.x, q.y};
#pragma unroll
        for (uint32_t s = 0; s < B; ++s) lv[s] = (uint8_t)(w2[(s >> 2) & 1u] >> (8u * (s & 3u)));
      }
      uint32_t pv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[j] = (uint32_t)j < D ? LN::get(planes + j * W, v) : 0u;
#pragma unroll
      for (uint32_t s = 0; s < B; ++s) {
        if (s >= nl) continue;
        const bool reached = (sv >> s) & 1u;
        a.dist[(size_t)(sid0 + s) * V + v] = reached ? (uint64_t)lv[s] * cost : ~0ull;
        if (a.nh) {
          uint32_t byte = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) byte |= ((pv[j] >> s) & 1u) << j;
          uint8_t* o = a.nh + ((size_t)(sid0 + s) * V + v) * nb;
          o[0] = (uint8_t)byte;
          for (uint32_t k = 1; k < nb; ++k) o[k] = 0;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace

uint32_t msbfs_lds_bytes(uint32_t V, uint32_t D, uint32_t lanes, uint32_t cap) {
  if (V > 65535u || D > 8u) return 0;
  const uint32_t t = lanes == 16 ? ms_layout<uint16_t>(V, D, cap).total : ms_layout<uint8_t>(V, D, cap).total;
  return t <= kMaxLds ? t : 0;
}

MsPlan plan_msbfs(const DevGraph& g, uint32_t n, uint32_t nh_bits, bool has_ign, bool tight, int num_cus) {
  MsPlan p;
  if (has_ign || tight || nh_bits > 8u || g.V > 65535u || n < 2) return p;
  // Opt-in (OPENR_SPF_MSBFS=1): on grids the BFS rings of different sources are nearly
  // disjoint, so lane sharing buys nothing and the per-source kernel is faster
  // (measured 2.33 vs 1.61 ms on G100 all-sources, profiles/r01).
  const char* en = std::getenv("OPENR_SPF_MSBFS");
  if (!en || en[0] != '1') return p;
  int lanes = 16;
  if (const char* e = std::getenv("OPENR_SPF_MS_LANES")) lanes = std::atoi(e) == 8 ? 8 : 16;
  const uint32_t wgs_per_cu = lanes == 16 ? 1u : 2u;  // 1024- / 512-thread workgroups
  const uint32_t D = nh_bits ? nh_bits : 1u;
  const uint32_t fixed = lanes == 16 ? ms_layout<uint16_t>(g.V, D, 0).total : ms_layout<uint8_t>(g.V, D, 0).total;
  const uint32_t budget = kMaxLds / wgs_per_cu;
  if (fixed + 64u >= budget) return p;
  uint32_t cap = (budget - fixed) / 4u;  // two u16 lists
  cap &= ~7u;
  if (cap > g.V) cap = (g.V + 7u) & ~7u;
  if (cap < 256u && cap < g.V) return p;
  if (const char* e = std::getenv("OPENR_SPF_MS_CAP")) cap = std::max(8u, (uint32_t)std::atoi(e)) & ~7u;  // tests
  p.use = true;
  p.lanes = lanes;
  p.cap = cap;
  p.lds = lanes == 16 ? ms_layout<uint16_t>(g.V, D, cap).total : ms_layout<uint8_t>(g.V, D, cap).total;
  const uint32_t batches = (n + (uint32_t)lanes - 1u) / (uint32_t)lanes;
  p.grid = std::min<uint32_t>(batches, (uint32_t)num_cus * wgs_per_cu);
  p.scratch = (size_t)p.grid * g.V * (size_t)lanes;
  return p;
}

hipError_t launch_msbfs(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t D, int lanes, int group_lanes,
                        uint32_t cap, uint8_t* scratch, uint32_t grid, hipStream_t s, LaunchInfo* info) {
  uint32_t glog = 0;
  while ((1 << glog) < group_lanes && glog < 6) ++glog;
  constexpr int K = (int)kBfsEdgesPerLane;
  if (lanes == 16) {
    const uint32_t lds = ms_layout<uint16_t>(g.V, D, cap).total;
    auto k = msbfs_kernel<uint16_t, K, 1024>;
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    if (info) {
      info->lds_bytes = lds;
      info->grid = grid;
      info->kernel = "msbfs_kernel<16 lanes>";
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(1024), lds, s, g, a, cost, D, glog, cap, scratch);
  } else {
    const uint32_t lds = ms_layout<uint8_t>(g.V, D, cap).total;
    auto k = msbfs_kernel<uint8_t, K, 512>;
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    if (info) {
      info->lds_bytes = lds;
      info->grid = grid;
      info->kernel = "msbfs_kernel<8 lanes>";
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, s, g, a, cost, D, glog, cap, scratch);
  }
  return hipGetLastError();
}

}  // namespace openr_spf
