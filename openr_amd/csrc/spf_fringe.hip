// spf_fringe.hip — general-metric SPF kernel: one wavefront per solve, settle-safe
// buckets over a fringe list.
//
// Semantics: LinkState::runSpf (/root/reference/openr/decision/LinkState.cpp:808-882)
// in closed form for strictly positive metrics:
//   dist(v) = shortest distance over usable edges, overloaded nodes other than the
//             source are reached but never expanded (:831-838);
//   nh(v)   = OR over tight in-edges u->v of (u == src ? {v} : nh(u))  (:857-873).
//
// Algorithm (Dial / delta-stepping with delta = w_min, the smallest usable metric): the
// fringe F holds every reached, unsettled node once. A step takes m = min dist over F
// and settles the bucket [m, m + w_min): no edge can land inside its own bucket, so
// every member's distance is final. A member pulls its next hops over tight in-edges
// (their tails sit in earlier buckets: final), then pushes its out-edges with LDS
// atomicMin; the push that lowers a node from "unreached" appends it to F. Pushes only
// touch non-members (cand >= m + w_min) and pulls only read settled tails, so members
// of one step need no ordering among themselves.
//
// Shape: a 64-lane wavefront owns a solve (persistent, dynamically scheduled): steps
// are wave-synchronous — no workgroup barrier anywhere — and the per-solve LDS is
// dist (u32, or u64 when V * w_max may overflow) + next-hop sets + two u16 node lists,
// ~10 KB for the 1k-node WAN, so ~15 solves share a CU. The previous 256-thread
// bucket kernel rescanned all V nodes twice per bucket behind four barriers.
// Integer work only; no MFMA (min-plus relaxation is not a matrix contraction).
#include <algorithm>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;
using namespace bfs;

constexpr uint32_t kWave = 64;

struct FringeLayout {
  uint32_t dist, nh, fr, mem, ign, total;
};

__host__ __device__ inline FringeLayout fringe_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t nh_words,
                                                      uint32_t dist_bytes) {
  FringeLayout l;
  uint32_t off = 16;  // control: [0] fringe append counter
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.dist = take(dist_bytes * V);
  l.nh = take(4u * nh_words);
  l.fr = take(2u * V);
  l.mem = take(2u * V);
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.total = off;
  return l;
}

template <typename D>
__device__ __forceinline__ D wave_min(D x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const D y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}

// Wait for this wave's LDS traffic (appends, atomics) before reading it back.
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int MODE, typename D, bool GENERIC>
__global__ __launch_bounds__(kWave) void fringe_kernel(DevGraph g, SolveArgs a, uint32_t delta, uint32_t has_ign_rt,
                                                       uint32_t* ctr) {
  using N = Nh<MODE>;
  constexpr D INF = (D)~(D)0;
  constexpr int K = 4;  // edges of a row loaded ahead together
  const bool has_ign = GENERIC && has_ign_rt != 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V, lane = threadIdx.x;
  const uint32_t nh_words = N::words(V);
  const FringeLayout lay = fringe_layout(V, g.L, has_ign, nh_words, sizeof(D));
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  D* dist = reinterpret_cast<D*>(base + lay.dist);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint16_t* fr = reinterpret_cast<uint16_t*>(base + lay.fr);
  uint16_t* mem = reinterpret_cast<uint16_t*>(base + lay.mem);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  const uint32_t ign_words = (g.L + 31u) / 32u;
  const uint32_t tight_words = (g.E + 63u) / 64u;

  for (uint32_t sid = blockIdx.x; sid < a.n;) {
    const uint32_t src = a.sources[sid];
    if (src < V) {
      for (uint32_t v = lane; v < V; v += kWave) dist[v] = INF;
      for (uint32_t i = lane; i < nh_words; i += kWave) nh[i] = 0;
      if (has_ign) {
        for (uint32_t i = lane; i < ign_words; i += kWave) ign[i] = 0;
        lds_fence();
        load_ignore(ign, ign_words, a, sid, g.L);
      }
      uint64_t* trow = (GENERIC && a.tight) ? a.tight + out_row_of(a, sid) * tight_words : nullptr;
      lds_fence();
      if (lane == 0) {
        dist[src] = 0;
        fr[0] = (uint16_t)src;
      }
      lds_fence();
      uint32_t nf = 1;  // wave-uniform fringe size
      while (nf) {
        // (a) bucket floor m = min tentative distance over the fringe
        D mn = INF;
        for (uint32_t i = lane; i < nf; i += kWave) {
          const D d = dist[fr[i]];
          mn = d < mn ? d : mn;
        }
        mn = wave_min(mn);
        const uint64_t hi = (uint64_t)mn + delta;  // bucket [m, m + w_min)
        // (b) split the fringe: members -> mem[0, nm), the rest compacted to fr[0, nr)
        //     (a chunk is read before any of its slots can be overwritten)
        uint32_t nm = 0, nr = 0;
        for (uint32_t i0 = 0; i0 < nf; i0 += kWave) {
          const uint32_t i = i0 + lane;
          const uint32_t v = i < nf ? fr[i] : 0u;
          const bool live = i < nf;
          const bool in = live && (uint64_t)dist[v] < hi;
          const unsigned long long mi = __ballot(in), mr = __ballot(live && !in);
          const unsigned long long lt = (1ull << lane) - 1ull;
          if (in) mem[nm + (uint32_t)__popcll(mi & lt)] = (uint16_t)v;
          if (live && !in) fr[nr + (uint32_t)__popcll(mr & lt)] = (uint16_t)v;
          nm += (uint32_t)__popcll(mi);
          nr += (uint32_t)__popcll(mr);
        }
        if (lane == 0) ctl[0] = nr;
        lds_fence();
        // (c) members: pull next hops over tight in-edges, push relaxations
        for (uint32_t i = lane; i < nm; i += kWave) {
          const uint32_t v = mem[i];
          const D dv = dist[v];
          const uint2 r = g.row2[v];
          const bool expand = v == src || !g.ovl[v];
          typename N::Val acc{};
          for (uint32_t e0 = r.x; e0 < r.y; e0 += K) {
            uint4 rec[K];  // v->u: {u | down | sink(u), w(u->v), link, rev = u->v}
            uint32_t wo[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j;
              rec[j] = e < r.y ? g.erec[e] : make_uint4(kEdgeDown, 0u, 0u, 0u);
              wo[j] = e < r.y ? g.w[e] : 0u;
            }
            bool ok[K];
            uint32_t uu[K];
            D du[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              uu[j] = rec[j].x & ~(kEdgeDown | kNodeSink);
              ok[j] = !(rec[j].x & kEdgeDown) && !(has_ign && test_bit(ign, rec[j].z));
              du[j] = ok[j] ? dist[uu[j]] : INF;
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
              if (!ok[j]) continue;
              const uint32_t u = uu[j];
              // pull: in-edge u->v (metric win) is tight (LinkState.cpp:857-873)
              if (v != src && du[j] != INF && (uint64_t)du[j] + rec[j].y == (uint64_t)dv &&
                  (u == src || !(rec[j].x & kNodeSink))) {
                const uint32_t re = rec[j].w;
                if (u == src) {
                  const uint32_t b = g.nbr[re];
                  if constexpr (N::kSingle) {
                    acc.x |= 1u << b;
                  } else {
                    acc.x[b >> 5] |= 1u << (b & 31u);
                  }
                } else {
                  const typename N::Val x = N::load(nh, u);
                  if constexpr (N::kSingle) {
                    acc.x |= x.x;
                  } else {
                    for (int k = 0; k < (int)(sizeof(acc.x) / 4); ++k) acc.x[k] |= x.x[k];
                  }
                }
                if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[re >> 6]), 1ull << (re & 63u));
              }
              // push: relax v->u; the arrival that lowers u from "unreached" appends it
              if (expand) {
                const D cand = dv + (D)wo[j];
                if (cand < du[j]) {
                  const D old = atomicMin(&dist[u], cand);
                  if (old == INF) fr[atomicAdd(&ctl[0], 1u)] = (uint16_t)u;
                }
              }
            }
          }
          N::or_val(nh, v, acc);  // v's set is complete: every tight tail was settled earlier
        }
        lds_fence();
        nf = __builtin_amdgcn_readfirstlane(ctl[0]);
      }
      // result rows, coalesced; unreached nodes keep UINT64_MAX
      uint64_t* drow = a.dist + out_row_of(a, sid) * V;
      for (uint32_t v = lane; v < V; v += kWave) {
        const D d = dist[v];
        store_row<uint64_t>(&drow[v], d == INF ? ~0ull : (uint64_t)d, true);
      }
      if (a.nh) {
        const uint32_t nb = a.nh_bytes;
        uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
        const uint32_t total = V * nb;
        for (uint32_t i = lane; i < total; i += kWave) {
          const uint32_t v = i / nb, j = i - v * nb;
          nrow[i] = (uint8_t)N::byte(nh, v, j);
        }
      }
    }
    // next solve: dynamic scheduling (the first gridDim.x solves are static)
    uint32_t nxt = 0;
    if (lane == 0) nxt = gridDim.x + atomicAdd(&ctr[0], 1u);
    sid = __builtin_amdgcn_readfirstlane(__shfl(nxt, 0));
  }
  retire_workgroup(ctr, nullptr);
}

template <int MODE, typename D>
hipError_t launch_fringe_t(const DevGraph& g, const SolveArgs& a, uint32_t delta, uint32_t lds, uint32_t grid,
                           uint32_t* ctr, hipStream_t s) {
  const bool has_ign = a.ign_ptr != nullptr;
  const bool generic = has_ign || a.tight != nullptr;
  auto k = generic ? fringe_kernel<MODE, D, true> : fringe_kernel<MODE, D, false>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  note_launch("fringe_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWave), lds, s, g, a, delta, (uint32_t)has_ign, ctr);
  return hipGetLastError();
}

}  // namespace

uint32_t fringe_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64) {
  if (V > 65535u) return 0;
  const uint32_t t = fringe_layout(V, L, has_ignore, nh_words_for(nh_mode, V), dist64 ? 8u : 4u).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_fringe(const DevGraph& g, const SolveArgs& a, uint32_t delta, bool dist64, int nh_mode,
                         int num_cus, hipStream_t s, LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  const uint32_t lds = fringe_lds_bytes(g.V, g.L, has_ign, nh_mode, dist64);
  if (!lds || delta == 0 || !a.work) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  const uint32_t grid = blocks_for(a.n, lds, num_cus, kWave);
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = dist64 ? "fringe_kernel<u64>" : "fringe_kernel<u32>";
  }
  uint32_t* ctr = a.work + kFringeCtr;
#define OPENR_FRINGE_CASE(M) \
  case M: return dist64 ? launch_fringe_t<M, unsigned long long>(g, a, delta, lds, grid, ctr, s) \
                        : launch_fringe_t<M, uint32_t>(g, a, delta, lds, grid, ctr, s);
  switch (nh_mode) {
    OPENR_FRINGE_CASE(kNhNibble)
    OPENR_FRINGE_CASE(kNhByte)
    OPENR_FRINGE_CASE(kNhHalf)
    OPENR_FRINGE_CASE(kNhW1)
    OPENR_FRINGE_CASE(kNhW2)
    OPENR_FRINGE_CASE(kNhW4)
    OPENR_FRINGE_CASE(kNhW8)
  }
#undef OPENR_FRINGE_CASE
  return hipErrorInvalidValue;
}

}  // namespace openr_spf
