// spf_sweep.hip — device helpers of the per-link-failure what-if sweep
// (openr_spf_whatif, BASELINE config 4).
//
// A what-if unit (i, j) is LinkState::runSpf(sources[j], useLinkMetric, {links[i]})
// (/root/reference/openr/decision/LinkState.cpp:808-882 with linksToIgnore, the same
// call getKthPaths makes at :769-779) compared with the no-failure SPF of sources[j].
// A link that carries no tight edge of the base SPF (neither direction on a shortest
// path) cannot change dist, next hops or pathLinks — nh(v) and dist(v) depend on tight
// edges only — so those units are resolved (0 changes) by the filter without a solve.
// The rest are solved in chunks by the ordinary batched kernels (one (source,
// {link}) ignore set per solve) and reduced against the base rows by rows_compare.
// Integer / byte work only: HBM-bound, coalesced row reads, one workgroup per unit.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "spf_bfs_common.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {

// unit u = i * n_src + j. One thread per unit; affected units are appended with one
// atomic per wave (ballot + prefix), so the work list is dense.
__global__ __launch_bounds__(256) void whatif_filter(const uint2* ledge, uint32_t L, uint32_t tight_words,
                                                     const uint32_t* links, uint32_t n_links,
                                                     const uint32_t* sources, uint32_t n_src,
                                                     const uint64_t* base_tight, uint32_t* changed, uint32_t* wsrc,
                                                     uint32_t* wlink, uint32_t* wunit, uint32_t* wcount) {
  const uint64_t total = (uint64_t)n_links * n_src;
  for (uint64_t u0 = (uint64_t)blockIdx.x * 256u; u0 < total; u0 += (uint64_t)gridDim.x * 256u) {
    const uint64_t u = u0 + threadIdx.x;
    bool hit = false;
    uint32_t l = 0, j = 0;
    if (u < total) {
      const uint32_t i = (uint32_t)(u / n_src);
      j = (uint32_t)(u - (uint64_t)i * n_src);
      l = links[i];
      changed[u] = 0;
      const uint2 ee = l < L ? ledge[l] : make_uint2(UINT32_MAX, UINT32_MAX);
      if (ee.x != UINT32_MAX) {
        if (!base_tight) {
          hit = true;  // exact-order plans: every unit is solved
        } else {
          const uint64_t* trow = base_tight + (size_t)j * tight_words;
          hit = ((trow[ee.x >> 6] >> (ee.x & 63u)) & 1ull) || ((trow[ee.y >> 6] >> (ee.y & 63u)) & 1ull);
        }
      }
    }
    const unsigned long long m = __ballot(hit);
    if (!m) continue;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(wcount, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    if (hit) {
      const uint32_t k = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      wsrc[k] = sources[j];
      wlink[k] = l;
      wunit[k] = (uint32_t)u;
    }
  }
}

// changed[wunit[k]] = number of nodes whose distance or next-hop bytes differ from the
// base row of source j = wunit[k] % n_src. One workgroup per solved unit.
__global__ __launch_bounds__(256) void rows_compare(uint32_t n, uint32_t V, uint32_t nb, const uint64_t* dist,
                                                    const uint8_t* nh, const uint64_t* base_dist,
                                                    const uint8_t* base_nh, const uint32_t* wunit, uint32_t n_src,
                                                    uint32_t* changed, WhatifDelta dl) {
  __shared__ uint32_t part[4];
  __shared__ unsigned long long s_base;
  const uint32_t lane = __lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t unit = wunit[k], j = unit % n_src;
    const uint64_t* d = dist + (size_t)k * V;
    const uint64_t* bd = base_dist + (size_t)j * V;
    const uint8_t* h = nh ? nh + (size_t)k * V * nb : nullptr;
    const uint8_t* bh = nh ? base_nh + (size_t)j * V * nb : nullptr;
    auto differs = [&](uint32_t v) {
      bool diff = d[v] != bd[v];
      if (h)
        for (uint32_t b = 0; b < nb && !diff; ++b) diff = h[(size_t)v * nb + b] != bh[(size_t)v * nb + b];
      return diff;
    };
    uint32_t c = 0;
    for (uint32_t v = threadIdx.x; v < V; v += 256u) c += differs(v) ? 1u : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) part[wave] = c;
    __syncthreads();
    const uint32_t total = part[0] + part[1] + part[2] + part[3];
    if (threadIdx.x == 0) changed[unit] = total;
    if (dl.node) {  // the unit's delta: one pool reservation, then each wave's diffs in order
      if (threadIdx.x == 0) {
        const unsigned long long b = total ? atomicAdd(dl.used, (unsigned long long)total) : 0ull;
        s_base = b;
        if (total) dl.off[unit] = dl.base_of(b);
      }
      __syncthreads();
      unsigned long long cur = s_base;
      for (uint32_t w = 0; w < wave; ++w) cur += part[w];
      for (uint32_t v0 = wave * 64u; v0 < V; v0 += 256u) {
        const uint32_t v = v0 + lane;
        const bool diff = v < V && differs(v);
        const unsigned long long m = __ballot(diff);
        const unsigned long long pos =
            cur + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (diff && pos < dl.cap) {
          dl.node[pos] = v;
          dl.dist[pos] = d[v];
          uint8_t* o = dl.nh + (size_t)pos * dl.nhb;
          for (uint32_t b = 0; b < dl.nhb; ++b) o[b] = (h && b < nb) ? h[(size_t)v * nb + b] : 0u;
        }
        cur += (uint32_t)__popcll(m);
      }
    }
    __syncthreads();
  }
}

// --- incremental what-if (one wavefront per affected unit) ---------------------------
//
// Removing link l from the SPF of s changes only part of the result. With (a->b) the
// tight direction of l in the base SPF (dist D, next hops H):
//   A = nodes whose distance grows: b if it has no other live tight in-edge, then every
//       tight successor of an A node whose tight in-edges all come from A (decremental
//       propagation over the base tight DAG). Every A node's distance strictly grows, and
//       no A node can become a tight predecessor of a node outside A.
//   D'  = D outside A; inside A: the best entry from outside A, then relaxation within A.
//   nh' = recomputed in increasing D' for the dirty nodes: A, b, the non-A tight
//         successors of A nodes, and the tight successors of every non-A node whose set
//         changed (pulled over the new tight in-edges; clean nodes keep H).
// changed = |A| + non-A nodes whose set changed — the same count rows_compare gets from a
// full re-solve (the parity tests check both against oracle re-solves).
struct IncrLayout {
  uint32_t dist, nh, ina, dq, alist, dlist, total;
};

__host__ __device__ inline IncrLayout incr_layout(uint32_t V, uint32_t nb, uint32_t dist_bytes) {
  IncrLayout l;
  uint32_t off = 16;  // control: [0] A count, [1] dirty count, [2] flag
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.dist = take(dist_bytes * V);
  l.nh = take(nb * V);
  l.ina = take(4u * ((V + 31u) / 32u));
  l.dq = take(4u * ((V + 31u) / 32u));
  l.alist = take(2u * V);  // A list; in (3) split scratch: members from the front, rest from the back
  l.dlist = take(2u * V);
  l.total = off;
  return l;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ bool bit_of(const uint32_t* b, uint32_t i) { return (b[i >> 5] >> (i & 31u)) & 1u; }

// DPP lane moves (VALU, no LDS round trip; ds_bpermute shuffles cost one each). An
// invalid source lane (disabled by EXEC) yields x itself, neutral for min / or.
template <int C, typename T>
__device__ __forceinline__ T dppmv(T x) {
  static_assert(sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8, "16-, 32- or 64-bit lanes");
  if constexpr (sizeof(T) <= 4) {
    return (T)__builtin_amdgcn_update_dpp((int)(uint32_t)x, (int)(uint32_t)x, C, 0xF, 0xF, false);
  } else {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)x, (int)(uint32_t)x, C, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(x >> 32), (int)(uint32_t)(x >> 32), C,
                                                              0xF, 0xF, false);
    return (T)((uint64_t)lo | ((uint64_t)hi << 32));
  }
}
// LDS atomic min for the repair's distance types (16-bit: a CAS loop on the word)
__device__ __forceinline__ void lds_atomic_min(uint16_t* p, uint16_t v) {
  uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
  const uint32_t sh = (reinterpret_cast<uintptr_t>(p) & 2u) * 8u;
  uint32_t old = *w;
  while (((old >> sh) & 0xFFFFu) > v) {
    const uint32_t seen = atomicCAS(w, old, (old & ~(0xFFFFu << sh)) | ((uint32_t)v << sh));
    if (seen == old) break;
    old = seen;
  }
}
__device__ __forceinline__ void lds_atomic_min(uint32_t* p, uint32_t v) { atomicMin(p, v); }
__device__ __forceinline__ void lds_atomic_min(unsigned long long* p, unsigned long long v) { atomicMin(p, v); }

constexpr int kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppRowMirror = 0x140, kDppHalfMirror = 0x141;

template <typename T>
__device__ __forceinline__ T readlane_t(T x, int l) {
  if constexpr (sizeof(T) <= 4) {
    return (T)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  } else {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return (T)((uint64_t)lo | ((uint64_t)hi << 32));
  }
}

// min over the 8-lane group of the calling lane (every lane of the group gets it)
template <typename D>
__device__ __forceinline__ D grp8_min(D x) {
  D y = dppmv<kDppQuadXor1>(x);
  x = y < x ? y : x;
  y = dppmv<kDppQuadXor2>(x);
  x = y < x ? y : x;
  y = dppmv<kDppHalfMirror>(x);
  return y < x ? y : x;
}

// wave-wide minimum, uniform result: rows of 16 by DPP, then four lane reads
template <typename D>
__device__ __forceinline__ D wave_min_t(D x) {
  x = grp8_min(x);
  const D y = dppmv<kDppRowMirror>(x);
  x = y < x ? y : x;
  const D a = readlane_t(x, 0), b = readlane_t(x, 16), c = readlane_t(x, 32), d = readlane_t(x, 48);
  const D ab = a < b ? a : b, cd = c < d ? c : d;
  return ab < cd ? ab : cd;
}

// OR over the lanes [0, n) of the wave (other lanes hold 0), uniform result
__device__ __forceinline__ uint32_t wave_or_prefix(uint32_t x, uint32_t n) {
  x |= dppmv<kDppQuadXor1>(x);
  x |= dppmv<kDppQuadXor2>(x);
  x |= dppmv<kDppHalfMirror>(x);
  if (n <= 8u) return readlane_t(x, 0);
  x |= dppmv<kDppRowMirror>(x);
  if (n <= 16u) return readlane_t(x, 0);
  return readlane_t(x, 0) | readlane_t(x, 16) | readlane_t(x, 32) | readlane_t(x, 48);
}

template <typename D>
struct IncrCtx {
  const DevGraph* g;
  uint32_t src, link, nb;
  bool unit;
  D* dist;
  uint8_t* nh;
  uint32_t *ina, *dq, *ctl;
  uint16_t *alist, *dlist;
  __device__ uint32_t wout(uint32_t e) const { return unit ? 1u : g->w[e]; }
  __device__ bool expands(uint32_t x) const { return x == src || !g->ovl[x]; }
};

// Does v keep a tight in-edge from a node outside A (other than link l)? Lanes over v's
// in-edges; wave-uniform.
template <typename D>
__device__ bool live_pred(const IncrCtx<D>& c, uint32_t v) {
  const DevGraph& g = *c.g;
  constexpr D INF = (D)~(D)0;
  const D dv = c.dist[v];
  const uint2 r = g.row2[v];
  for (uint32_t e = r.x + threadIdx.x; __any(e < r.y); e += 64u) {
    bool ok = false;
    if (e < r.y) {
      const uint4 rec = g.erec[e];  // v->u: {u | down | sink(u), w(u->v), link, rev}
      const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
      if (!(rec.x & kEdgeDown) && rec.z != c.link && (u == c.src || !(rec.x & kNodeSink)) && !bit_of(c.ina, u)) {
        const D du = c.dist[u];
        ok = du != INF && (uint64_t)du + (c.unit ? 1u : rec.y) == (uint64_t)dv;
      }
    }
    if (__any(ok)) return true;
  }
  return false;
}

// Same test by a single lane (sequential in-edge loop, 4 records in flight).
template <typename D>
__device__ bool live_pred_lane(const IncrCtx<D>& c, uint32_t v, D INF) {
  const DevGraph& g = *c.g;
  const D dv = c.dist[v];
  const uint2 r = g.row2[v];
  for (uint32_t e0 = r.x; e0 < r.y; e0 += 4u) {
    uint4 rec[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) rec[q] = e0 + q < r.y ? g.erec[e0 + q] : make_uint4(kEdgeDown, 0u, 0u, 0u);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t u = rec[q].x & ~(kEdgeDown | kNodeSink);
      if ((rec[q].x & kEdgeDown) || rec[q].z == c.link || bit_of(c.ina, u)) continue;
      if (u != c.src && (rec[q].x & kNodeSink)) continue;
      const D du = c.dist[u];
      if (du != INF && (uint64_t)du + (c.unit ? 1u : rec[q].y) == (uint64_t)dv) return true;
    }
  }
  return false;
}

template <typename D>
__device__ void push_dirty(const IncrCtx<D>& c, uint32_t y) {  // lane 0 only
  if (!bit_of(c.dq, y)) {
    c.dq[y >> 5] |= 1u << (y & 31u);
    c.dlist[c.ctl[1]++] = (uint16_t)y;
  }
}

template <typename D>
__global__ __launch_bounds__(64) void whatif_incr_kernel(DevGraph g, const uint32_t* wsrc, const uint32_t* wlink,
                                                         const uint32_t* wunit, uint32_t count, uint32_t n_src,
                                                         const uint64_t* base_dist, const uint8_t* base_nh,
                                                         uint32_t nb, uint32_t unit, uint32_t* changed,
                                                         uint32_t* ctr) {
  constexpr D INF = (D)~(D)0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V, lane = threadIdx.x, vw = (V + 31u) / 32u;
  const IncrLayout lay = incr_layout(V, nb, sizeof(D));
  char* base = reinterpret_cast<char*>(smem);
  IncrCtx<D> c;
  c.g = &g;
  c.nb = nb;
  c.unit = unit != 0;
  c.ctl = smem;
  c.dist = reinterpret_cast<D*>(base + lay.dist);
  c.nh = reinterpret_cast<uint8_t*>(base + lay.nh);
  c.ina = reinterpret_cast<uint32_t*>(base + lay.ina);
  c.dq = reinterpret_cast<uint32_t*>(base + lay.dq);
  c.alist = reinterpret_cast<uint16_t*>(base + lay.alist);
  c.dlist = reinterpret_cast<uint16_t*>(base + lay.dlist);
  for (uint32_t k = blockIdx.x; k < count;) {
    const uint32_t unit_id = wunit[k], j = unit_id % n_src;
    c.src = wsrc[k];
    c.link = wlink[k];
    const uint64_t* drow = base_dist + (size_t)j * V;
    const uint8_t* hrow = base_nh + (size_t)j * V * nb;
    for (uint32_t v = lane; v < V; v += 64u) {
      const uint64_t d = drow[v];
      c.dist[v] = d == ~0ull ? INF : (D)d;
    }
    for (uint32_t i = lane; i < V * nb; i += 64u) c.nh[i] = hrow[i];
    for (uint32_t i = lane; i < vw; i += 64u) {
      c.ina[i] = 0;
      c.dq[i] = 0;
    }
    if (lane == 0) c.ctl[0] = c.ctl[1] = 0;
    lds_fence();
    // the tight direction a->b of link l (the filter guarantees one)
    const uint2 ee = g.ledge[c.link];
    uint32_t bnode = UINT32_MAX;
    for (int t = 0; t < 2; ++t) {
      const uint32_t e = t ? ee.y : ee.x;
      const uint32_t av = g.adj[e];
      const uint32_t head = av & ~kEdgeDown, tail = g.adj[g.rev[e]] & ~kEdgeDown;
      if ((av & kEdgeDown) || !c.expands(tail)) continue;
      const D dt = c.dist[tail], dh = c.dist[head];
      if (dt != INF && dh != INF && (uint64_t)dt + c.wout(e) == (uint64_t)dh) bnode = head;
    }
    uint32_t nchanged = 0;
    if (bnode != UINT32_MAX) {
      // (1) A by decremental propagation over the base tight DAG
      if (lane == 0) push_dirty(c, bnode);
      if (!live_pred(c, bnode) && lane == 0) {
        c.ina[bnode >> 5] |= 1u << (bnode & 31u);
        c.alist[c.ctl[0]++] = (uint16_t)bnode;
      }
      lds_fence();
      for (uint32_t idx = 0; idx < __builtin_amdgcn_readfirstlane(c.ctl[0]); ++idx) {
        const uint32_t x = c.alist[idx];
        if (!c.expands(x)) continue;
        const D dx = c.dist[x];
        const uint2 r = g.row2[x];
        for (uint32_t e0 = r.x; e0 < r.y; e0 += 64u) {
          // lane per out-edge: a base-tight successor y outside A either keeps a live
          // pred or joins A (checked in parallel; a pred that joins A later re-checks y)
          const uint32_t e = e0 + lane;
          if (e < r.y) {
            const uint32_t av = g.adj[e];
            const uint32_t y = av & ~kEdgeDown;
            if (!(av & kEdgeDown) && g.lid[e] != c.link && !bit_of(c.ina, y) && c.dist[y] != INF &&
                (uint64_t)dx + c.wout(e) == (uint64_t)c.dist[y]) {
              const uint32_t bit = 1u << (y & 31u);
              if (!(atomicOr(&c.dq[y >> 5], bit) & bit)) c.dlist[atomicAdd(&c.ctl[1], 1u)] = (uint16_t)y;
              if (!live_pred_lane(c, y, INF)) {
                if (!(atomicOr(&c.ina[y >> 5], bit) & bit)) c.alist[atomicAdd(&c.ctl[0], 1u)] = (uint16_t)y;
              }
            }
          }
          lds_fence();
        }
      }
      const uint32_t na = __builtin_amdgcn_readfirstlane(c.ctl[0]);
      // (2) new distances inside A: best entry from outside A, then relaxation within A
      for (uint32_t i = lane; i < na; i += 64u) {
        const uint32_t x = c.alist[i];
        const uint2 r = g.row2[x];
        D best = INF;
        for (uint32_t e0 = r.x; e0 < r.y; e0 += 4u) {
          uint4 rec[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) rec[q] = e0 + q < r.y ? g.erec[e0 + q] : make_uint4(kEdgeDown, 0u, 0u, 0u);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t u = rec[q].x & ~(kEdgeDown | kNodeSink);
            if ((rec[q].x & kEdgeDown) || rec[q].z == c.link || bit_of(c.ina, u)) continue;
            if (u != c.src && (rec[q].x & kNodeSink)) continue;
            const D du = c.dist[u];
            if (du == INF) continue;
            const D cand = du + (D)(c.unit ? 1u : rec[q].y);
            best = cand < best ? cand : best;
          }
        }
        c.dist[x] = best;  // only non-A distances are read above
      }
      lds_fence();
      for (;;) {
        if (lane == 0) c.ctl[2] = 0;
        lds_fence();
        for (uint32_t i = lane; i < na; i += 64u) {
          const uint32_t x = c.alist[i];
          const D dx = c.dist[x];
          if (dx == INF || !c.expands(x)) continue;
          const uint2 r = g.row2[x];
          for (uint32_t e = r.x; e < r.y; ++e) {
            const uint32_t av = g.adj[e];
            const uint32_t y = av & ~kEdgeDown;
            if ((av & kEdgeDown) || g.lid[e] == c.link || !bit_of(c.ina, y)) continue;
            const D cand = dx + (D)c.wout(e);
            if (cand < c.dist[y]) {
              atomicMin(&c.dist[y], cand);
              c.ctl[2] = 1;
            }
          }
        }
        lds_fence();
        if (!__builtin_amdgcn_readfirstlane(c.ctl[2])) break;
      }
      // (3) next hops in increasing new distance over the dirty set; bucket members are
      //     independent (positive metrics), one lane per member
      uint32_t nd = __builtin_amdgcn_readfirstlane(c.ctl[1]), done = 0;
      while (done < nd) {
        D mn = INF;
        for (uint32_t i = done + lane; i < nd; i += 64u) {
          const D d = c.dist[c.dlist[i]];
          mn = d < mn ? d : mn;
        }
        mn = wave_min_t(mn);
        // split [done, nd): members first (alist is free after (2): scratch)
        uint32_t nm = 0, nr = 0;
        for (uint32_t i0 = done; i0 < nd; i0 += 64u) {
          const uint32_t i = i0 + lane;
          const bool live = i < nd;
          const uint32_t v = live ? c.dlist[i] : 0u;
          const bool in = live && c.dist[v] == mn;
          const unsigned long long mi = __ballot(in), mr = __ballot(live && !in);
          const unsigned long long lt = (1ull << lane) - 1ull;
          if (in) c.alist[nm + (uint32_t)__popcll(mi & lt)] = (uint16_t)v;
          if (live && !in) c.alist[V - 1u - (nr + (uint32_t)__popcll(mr & lt))] = (uint16_t)v;
          nm += (uint32_t)__popcll(mi);
          nr += (uint32_t)__popcll(mr);
        }
        lds_fence();
        for (uint32_t i = lane; i < nm + nr; i += 64u)
          c.dlist[done + i] = i < nm ? c.alist[i] : c.alist[V - 1u - (i - nm)];
        if (lane == 0) c.ctl[1] = nd;  // appends of this bucket go after the list
        lds_fence();
        uint32_t cnt_changed = 0;
        for (uint32_t i0 = 0; i0 < nm; i0 += 64u) {
          const uint32_t i = i0 + lane;
          bool counted = false;
          if (i < nm) {
            const uint32_t v = c.dlist[done + i];
            uint8_t acc[32];
            uint32_t acc1 = 0;  // nb == 1 (<= 8 next hops): register accumulator
            if (nb > 1)
              for (uint32_t b = 0; b < nb; ++b) acc[b] = 0;
            const D dv = c.dist[v];
            const uint2 r = g.row2[v];
            if (dv != INF)
              for (uint32_t e0 = r.x; e0 < r.y; e0 += 4u) {
                uint4 rec[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  rec[q] = e0 + q < r.y ? g.erec[e0 + q] : make_uint4(kEdgeDown, 0u, 0u, 0u);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const uint32_t u = rec[q].x & ~(kEdgeDown | kNodeSink);
                  if ((rec[q].x & kEdgeDown) || rec[q].z == c.link) continue;
                  if (u != c.src && (rec[q].x & kNodeSink)) continue;
                  const D du = c.dist[u];
                  if (du == INF || (uint64_t)du + (c.unit ? 1u : rec[q].y) != (uint64_t)dv) continue;
                  if (u == c.src) {
                    const uint32_t bit = g.nbr[rec[q].w];
                    if (nb == 1) acc1 |= 1u << bit;
                    else acc[bit >> 3] |= (uint8_t)(1u << (bit & 7u));
                  } else if (nb == 1) {
                    acc1 |= c.nh[u];
                  } else {
                    for (uint32_t b = 0; b < nb; ++b) acc[b] |= c.nh[(size_t)u * nb + b];
                  }
                }
              }
            bool diff = false;
            if (nb == 1) {
              diff = (uint8_t)acc1 != c.nh[v];
              if (diff) c.nh[v] = (uint8_t)acc1;
            } else {
              for (uint32_t b = 0; b < nb; ++b) diff |= acc[b] != c.nh[(size_t)v * nb + b];
              if (diff)
                for (uint32_t b = 0; b < nb; ++b) c.nh[(size_t)v * nb + b] = acc[b];
            }
            const bool in_a = bit_of(c.ina, v);
            counted = in_a || diff;
            // a non-A node whose set changed dirties its tight successors (an A node's new
            // tight successors are A nodes, already dirty)
            if (diff && !in_a && c.expands(v)) {
              const uint2 ro = g.row2[v];
              for (uint32_t e = ro.x; e < ro.y; ++e) {
                const uint32_t av = g.adj[e];
                const uint32_t y = av & ~kEdgeDown;
                if ((av & kEdgeDown) || g.lid[e] == c.link || y == c.src || c.dist[y] == INF) continue;
                if ((uint64_t)dv + c.wout(e) != (uint64_t)c.dist[y]) continue;
                const uint32_t bit = 1u << (y & 31u);
                if (!(atomicOr(&c.dq[y >> 5], bit) & bit)) c.dlist[atomicAdd(&c.ctl[1], 1u)] = (uint16_t)y;
              }
            }
          }
          cnt_changed += (uint32_t)__popcll(__ballot(counted));
        }
        nchanged += cnt_changed;
        lds_fence();
        done += nm;
        nd = __builtin_amdgcn_readfirstlane(c.ctl[1]);
      }
    }
    if (lane == 0) changed[unit_id] = nchanged;
    uint32_t nxt = 0;
    if (lane == 0) nxt = gridDim.x + atomicAdd(&ctr[0], 1u);
    k = __builtin_amdgcn_readfirstlane(__shfl(nxt, 0));
    lds_fence();
  }
  bfs::retire_workgroup(ctr, nullptr);
}

// --- grouped what-if: one workgroup per (source, chunk of links) -----------------------
//
// The same repair as whatif_incr_kernel (A set by decremental propagation, distances
// inside A, next hops over the dirty set in increasing new distance), restructured for
// the hardware:
//  * a source's base rows are read ONCE per work item instead of once per unit: the
//    workgroup stages dist / next hops / tight mask of source j in LDS (read-only, shared
//    by its wavefronts) and every wavefront repairs affected links of the item one after
//    another on a private OVERLAY: new distances of A nodes (valid where the wave's A bit
//    is set) and rewritten next-hop sets (valid where its nh bit is set); everything else
//    reads the shared base. Per unit only three V-bit masks are cleared;
//  * the repair is a chain of small dependent graph reads (rows, edge records) — L2
//    latency dominated it. When the graph fits (V, L <= 32767, usable metrics <= 65535),
//    each workgroup stages a compact copy of the graph in LDS once per launch
//    (GraphView<true>: row pointers, 8-byte edge records, next-hop bit of in-edges from
//    the source, overload bits), so every read of the repair is an LDS read;
//  * the link filter is fused (a link with no tight edge of the base SPF of j leaves the
//    unit unchanged: 0), so there is no global work list and no host round trip.
// Unit (i, j) writes changed[i * n_src + j].
struct EdgeRec {
  uint32_t col, lid, wout, win;  // e = x -> col: its link, metric x->col and col->x
  bool down, sink;               // !Link::isUp(), col overloaded
};

template <bool LG>
struct GraphView;
template <>
struct GraphView<false> {  // the device mirror in global memory
  const DevGraph* g;
  __device__ uint2 row(uint32_t x) const { return g->row2[x]; }
  __device__ EdgeRec rec(uint32_t e) const {
    const uint4 r = g->erec[e];
    EdgeRec o;
    o.col = r.x & ~(kEdgeDown | kNodeSink);
    o.down = (r.x & kEdgeDown) != 0;
    o.sink = (r.x & kNodeSink) != 0;
    o.win = r.y;
    o.lid = r.z;
    o.wout = g->w[e];
    return o;
  }
  __device__ uint32_t nbr_in(uint32_t e) const { return g->nbr[g->erec[e].w]; }
  __device__ bool ovl(uint32_t x) const { return g->ovl[x] != 0; }
};
template <>
struct GraphView<true> {  // compact LDS copy
  const uint32_t* rowp;   // [V+1]
  const uint2* crec;      // [E] {col | down << 15 | lid << 16 | sink << 31, wout | win << 16}
  const uint8_t* nbrin;   // [E] next-hop bit of the in-edge col -> x when col is the source
  const uint32_t* ovlb;   // [ceil(V/32)]
  __device__ uint2 row(uint32_t x) const { return make_uint2(rowp[x], rowp[x + 1]); }
  __device__ EdgeRec rec(uint32_t e) const {
    const uint2 r = crec[e];
    EdgeRec o;
    o.col = r.x & 0x7FFFu;
    o.down = (r.x >> 15) & 1u;
    o.lid = (r.x >> 16) & 0x7FFFu;
    o.sink = (r.x >> 31) != 0;
    o.wout = r.y & 0xFFFFu;
    o.win = r.y >> 16;
    return o;
  }
  __device__ uint32_t nbr_in(uint32_t e) const { return nbrin[e]; }
  __device__ bool ovl(uint32_t x) const { return (ovlb[x >> 5] >> (x & 31u)) & 1u; }
};

constexpr uint32_t kGrpMaxChunk = 2048;  // links per work item
constexpr uint32_t kGrpMaxCap = 255;     // dirty slots per wave (u8 slot index)
constexpr uint32_t kGrpCap1 = 128;       // dirty slots per wave of the first pass
constexpr uint32_t kGrpWaves = 4;        // waves per workgroup of the first pass

struct GrpLayout {
  uint32_t grow, grec, gnbr, govl;                                  // LDS graph (LG only)
  uint32_t bdist, bnh, btight, btin, ulist, wave0, wstride;         // wave w at wave0 + w * wstride
  uint32_t w_ina, w_dq, w_nhm, w_dec, w_didx, w_adist, w_anh, w_alist, w_dlist;  // offsets inside a wave block
  uint32_t total;
};

// Per-wave state is dense only where it is a bitmap or a byte per node; the overlays a
// repair writes (new distances, next hops, the A and dirty lists) hold at most `cap`
// dirty nodes (<= 255, indexed by didx[v] - 1); a unit with more is re-solved after
// the launch (full SPF with the link ignored + row compare, spf_capi.hip).
__host__ __device__ inline GrpLayout grp_layout(uint32_t V, uint32_t E, uint32_t nb, uint32_t dist_bytes, bool lg,
                                                uint32_t waves, uint32_t chunk, uint32_t cap) {
  GrpLayout l;
  uint32_t off = 16;  // workgroup control: [0] next link group of the item
  auto take = [](uint32_t& o, uint32_t bytes) {
    const uint32_t r = o;
    o += (bytes + 15u) & ~15u;
    return r;
  };
  const uint32_t vw = (V + 31u) / 32u;
  l.grow = lg ? take(off, 4u * (V + 1u)) : 0u;
  l.grec = lg ? take(off, 8u * E) : 0u;
  l.gnbr = lg ? take(off, E) : 0u;
  l.govl = lg ? take(off, 4u * vw) : 0u;
  l.bdist = take(off, dist_bytes * V);
  l.bnh = take(off, nb * V);
  l.btight = take(off, 8u * ((E + 63u) / 64u));
  l.btin = take(off, V + 4u);  // u8 base-tight in-degree per node (rows <= 255 edges)
  l.ulist = take(off, 4u * chunk);  // the item's affected links: offset in the chunk << 16 | b
  uint32_t w = 16;  // wave control: [0] A count, [1] dirty count, [2] flag
  l.w_ina = take(w, 4u * vw);
  l.w_dq = take(w, 4u * vw);
  l.w_nhm = take(w, 4u * vw);
  l.w_dec = take(w, V + 4u);   // u8 per node: tight in-edges whose tail joined A
  l.w_didx = take(w, V + 4u);  // u8 per node: 1 + its slot in the dirty list, 0 = clean
  l.w_adist = take(w, dist_bytes * cap);
  l.w_anh = take(w, nb * cap);
  l.w_alist = take(w, 2u * cap);
  l.w_dlist = take(w, 2u * cap);
  l.wave0 = off;
  l.wstride = w;
  l.total = off + waves * w;
  return l;
}

// next-hop sets of the grouped repair as u32 words in registers (<= 256 bits)
constexpr uint32_t kGrpNhWords = 8;  // W = 1 (sets <= 32 bits) or 8 (<= 256 bits): kernel variants

// acc |= (sel ? a : b), nb-byte sets: both rows are loaded before the select, so an
// overlay lookup costs one LDS round trip, not a bitmap read and then a row read
template <uint32_t W>
__device__ __forceinline__ void nh_or_sel(uint32_t (&acc)[W], const uint8_t* a, const uint8_t* b, bool sel,
                                          uint32_t nb) {
#pragma unroll
  for (uint32_t k = 0; k < W; ++k) {
    if (4u * k >= nb) break;
    uint32_t wa = 0, wb = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j)
      if (4u * k + j < nb) {
        wa |= (uint32_t)a[4u * k + j] << (8u * j);
        wb |= (uint32_t)b[4u * k + j] << (8u * j);
      }
    acc[k] |= sel ? wa : wb;
  }
}


template <typename D, bool LG, uint32_t W>
struct GrpWave {
  const DevGraph* g;  // ledge / rev / adj of the unit's link (read once per unit)
  GraphView<LG> gv;
  uint32_t src, link, nb;
  bool unit;
  const D* bdist;
  const uint8_t* bnh;
  D* adist;
  uint8_t* anh;
  uint32_t *ina, *dq, *nhm, *ctl;
  const uint64_t* btight;  // base-tight mask of the source (workgroup rows)
  const uint8_t* tin;      // base-tight in-degree (workgroup rows)
  uint8_t* dec;            // per unit: tight in-edges of v lost (tail in A, or the failed edge)
  uint8_t* didx;           // per unit: 1 + v's dirty slot (adist / anh index), 0 = clean
  uint32_t cap;            // dirty slots
  uint16_t *alist, *dlist;
  unsigned long long* prof;  // tuning (OPENR_SPF_PROF): per-phase cycles and sizes, or null
  WhatifDelta dl;            // delta output (the DL kernel variant)
  unsigned long long pcur, pend;  // DL: this wave's current block of pool slots [pcur, pend)
  uint32_t uidx;             // the unit's index in the API rows (link index * n_src + source index)
  __device__ uint32_t w(const EdgeRec& r) const { return unit ? 1u : r.wout; }
  __device__ uint32_t wi(const EdgeRec& r) const { return unit ? 1u : r.win; }
  __device__ bool expands(uint32_t x) const { return x == src || !gv.ovl(x); }
  // distance after step (2): A nodes from the overlay slot, the rest from the base (the
  // bitmap, slot index and base value load together; only A nodes read the slot)
  __device__ D dist(uint32_t u) const {
    bool in;
    return dist_a(u, in);
  }
  __device__ D dist_a(uint32_t u, bool& in) const {
    const uint32_t k = didx[u];
    const D b = bdist[u];
    in = bit_of(ina, u);
    return in ? adist[k - 1u] : b;
  }
  __device__ void nh_or(uint32_t (&acc)[W], uint32_t u) const {
    const uint32_t k = didx[u];
    const bool o = bit_of(nhm, u);
    nh_or_sel(acc, anh + (size_t)(o ? k - 1u : 0u) * nb, bnh + (size_t)u * nb, o, nb);
  }
  // append v to the dirty list at slot pos (false: the unit outgrows the slots)
  __device__ bool put_dirty(uint32_t v, uint32_t pos) const {
    if (pos >= cap) return false;
    dlist[pos] = (uint16_t)v;
    didx[v] = (uint8_t)(pos + 1u);
    return true;
  }
  // in-edge u -> v (the record of v -> u) usable, not the failed link, u may expand
  __device__ bool in_usable(const EdgeRec& r) const { return !r.down && r.lid != link && (r.col == src || !r.sink); }
};

constexpr uint32_t kGrpOverflow = UINT32_MAX;  // grp_repair: the unit outgrew the dirty slots

// One affected unit: returns the changed-node count (uniform across the wave), or
// kGrpOverflow.
// Delta output (DL): a wave takes pool slots in blocks of kDeltaBlock from the pool
// cursor and hands them to its units in order, so the cursor sees one atomic per block
// instead of one per unit (a million units on one address serialised: 12 ms against the
// 2.5 ms repair). A unit that does not fit the rest of the block starts a new block (the
// rest is a gap); a unit larger than half a block reserves its own slots. The pool is
// library scratch: openr_spf_whatif_delta compacts it into the caller's CSR.
constexpr uint32_t kDeltaBlock = 256;

template <typename D, bool LG, uint32_t W, bool DL>
__device__ uint32_t grp_repair(GrpWave<D, LG, W>& c, uint32_t lane, uint32_t V, uint32_t bnode) {
  constexpr D INF = (D)~(D)0;
  const uint32_t vw = (V + 31u) / 32u, nb = c.nb;
  for (uint32_t i = lane; i < vw; i += 64u) {
    c.ina[i] = 0;
    c.dq[i] = 0;
    c.nhm[i] = 0;
  }
  for (uint32_t i = lane; i < (V + 4u) / 4u; i += 64u) {
    reinterpret_cast<uint32_t*>(c.dec)[i] = 0;
    reinterpret_cast<uint32_t*>(c.didx)[i] = 0;
  }
  if (lane == 0) c.ctl[0] = c.ctl[1] = c.ctl[2] = 0;  // [2]: the unit outgrew the dirty slots
  lds_fence();
  long long pt0 = c.prof ? (long long)__builtin_amdgcn_s_memtime() : 0, pt1 = 0, pt2 = 0, pt3 = 0;
  // (1) A by decremental propagation over the base tight DAG: v joins A when every one of
  // its tight in-edges is lost (the failed edge a->b, or a tail already in A). dec[v]
  // counts the lost ones; the lane whose increment reaches tin[v] appends v.
  if (lane == 0) {
    c.dq[bnode >> 5] |= 1u << (bnode & 31u);
    c.put_dirty(bnode, c.ctl[1]++);
    if (c.tin[bnode] == 1u) {
      c.ina[bnode >> 5] |= 1u << (bnode & 31u);
      c.alist[c.ctl[0]++] = (uint16_t)bnode;
    }
  }
  lds_fence();
  // 8-lane groups: eight A members per wave pass, a lane per out-edge (members appended
  // during a pass are taken by the next)
  for (uint32_t idx0 = 0, na0; idx0 < (na0 = __builtin_amdgcn_readfirstlane(c.ctl[0])) &&
                               !__builtin_amdgcn_readfirstlane(c.ctl[2]);
       idx0 += min(8u, na0 - idx0)) {
    const uint32_t idx = idx0 + (lane >> 3), sub = lane & 7u;
    if (idx < na0) {
      const uint32_t x = c.alist[idx];
      const uint2 r = c.gv.row(x);
      for (uint32_t e = r.x + sub; e < r.y; e += 8u) {
        if (!((c.btight[e >> 6] >> (e & 63u)) & 1ull)) continue;  // base-tight x -> y (x expands)
        const uint32_t y = c.gv.rec(e).col;
        const uint32_t bit = 1u << (y & 31u);
        if (!(atomicOr(&c.dq[y >> 5], bit) & bit) && !c.put_dirty(y, atomicAdd(&c.ctl[1], 1u))) c.ctl[2] = 1;
        const uint32_t sh = 8u * (y & 3u);
        const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(c.dec) + (y >> 2), 1u << sh);
        if (((old >> sh) & 0xFFu) + 1u == c.tin[y]) {
          atomicOr(&c.ina[y >> 5], bit);
          const uint32_t pa = atomicAdd(&c.ctl[0], 1u);  // A is part of the dirty set: pa < cap
          if (pa < c.cap) c.alist[pa] = (uint16_t)y;
        }
      }
    }
    lds_fence();
  }
  if (__builtin_amdgcn_readfirstlane(c.ctl[2])) return kGrpOverflow;
  const uint32_t na = __builtin_amdgcn_readfirstlane(c.ctl[0]);
  if (c.prof) pt1 = (long long)__builtin_amdgcn_s_memtime();
  // (2) tentative distances inside A: the best entry from outside A (an 8-lane group per
  // A node, a lane per in-edge, then a min). Relaxation within A happens in step (3),
  // which settles A members in increasing distance together with the other dirty nodes.
  const uint32_t sub = lane & 7u;
  for (uint32_t i0 = 0; i0 < na; i0 += 8u) {
    const uint32_t i = i0 + (lane >> 3);
    D best = INF;
    uint32_t x = 0;
    if (i < na) {
      x = c.alist[i];
      const uint2 r = c.gv.row(x);
      for (uint32_t e = r.x + sub; e < r.y; e += 8u) {
        const EdgeRec q = c.gv.rec(e);
        if (!c.in_usable(q) || bit_of(c.ina, q.col)) continue;
        const D du = c.bdist[q.col];
        if (du == INF) continue;
        const D cand = du + (D)c.wi(q);
        best = cand < best ? cand : best;
      }
    }
    best = grp8_min(best);
    if (i < na && sub == 0) c.adist[c.didx[x] - 1u] = best;
  }
  lds_fence();
  // (3) Dijkstra over the dirty set: buckets of equal (new) distance in increasing order. A
  // bucket's A members are final (every node nearer was settled and relaxed its edges into
  // A); settling a node pulls its next hops over tight in-edges, an A member relaxes its
  // edges into A, and a non-A node whose set changed makes its tight successors dirty
  // (both land strictly beyond the bucket). One node at a time across the wave, a lane
  // per edge of its row. The dirty list's first 64 entries live in lanes (entry i in
  // lane i), later ones are re-read from LDS.
  if (c.prof) pt2 = (long long)__builtin_amdgcn_s_memtime();
  const uint32_t nbw = (nb + 3u) / 4u;
  uint32_t nchanged = 0, buckets = 0;
  uint32_t nd = __builtin_amdgcn_readfirstlane(c.ctl[1]), loaded = 0;
  uint32_t ev = 0;
  uint2 er = make_uint2(0u, 0u);  // the lane's entry's row, loaded with the entry
  D ed = INF;
  bool pend = false, ea = false;  // ea: the lane's entry is in A (its distance may still drop)
  // one dirty node v (wave-uniform, row r) at new distance dv: pull its set over tight
  // in-edges; if it changed and v keeps its base distance, its tight successors become dirty
  auto process = [&](uint32_t v, D dv, uint2 r) {
    const uint32_t deg = r.y - r.x;
    uint32_t cur[W], acc[W];
#pragma unroll
    for (uint32_t k = 0; k < W; ++k) cur[k] = acc[k] = 0;
    c.nh_or(cur, v);
    const bool in_a = bit_of(c.ina, v);
    EdgeRec q{};
    D du = INF;
    bool ua = false;
    const bool relax = in_a && dv != INF && c.expands(v);
    for (uint32_t e0 = r.x; e0 < r.y; e0 += 64u) {
      const uint32_t e = e0 + lane;
      du = INF;
      if (e < r.y) {
        q = c.gv.rec(e);
        du = c.dist_a(q.col, ua);
        if (relax && ua && !q.down && q.lid != c.link) {  // v settled: relax v -> u inside A
          const D cand = dv + (D)c.w(q);
          if (cand < du) lds_atomic_min(&c.adist[c.didx[q.col] - 1u], cand);
        }
        if (dv != INF && c.in_usable(q) && du != INF && (uint64_t)du + c.wi(q) == (uint64_t)dv) {
          if (q.col == c.src) {
            const uint32_t bit = c.gv.nbr_in(e);
#pragma unroll
            for (uint32_t k = 0; k < W; ++k)
              if (bit >> 5 == k) acc[k] |= 1u << (bit & 31u);
          } else {
            c.nh_or(acc, q.col);
          }
        }
      }
    }
    bool diff = false;
#pragma unroll
    for (uint32_t k = 0; k < W; ++k) {
      if (W > 1 && k >= nbw) break;
      acc[k] = wave_or_prefix(acc[k], min(deg, 64u));
      diff |= acc[k] != __builtin_amdgcn_readfirstlane(cur[k]);
    }
    if (diff) {
      if (lane == 0) {
        uint8_t* o = c.anh + (size_t)(c.didx[v] - 1u) * nb;
        for (uint32_t b = 0; b < nb; ++b) o[b] = (uint8_t)(acc[b >> 2] >> (8u * (b & 3u)));
        c.nhm[v >> 5] |= 1u << (v & 31u);
      }
    }
    if (in_a || diff) ++nchanged;
    if (!diff || in_a || dv == INF || !c.expands(v)) return;
    for (uint32_t e0 = r.x; e0 < r.y; e0 += 64u) {
      const uint32_t e = e0 + lane;
      if (deg > 64u) {  // rows longer than a wave: the first pass kept only its last chunk
        du = INF;
        if (e < r.y) {
          q = c.gv.rec(e);
          du = c.dist(q.col);
        }
      }
      const uint32_t y = q.col;
      bool fresh = false;
      if (e < r.y && !q.down && q.lid != c.link && y != c.src && du != INF && (uint64_t)dv + c.w(q) == (uint64_t)du) {
        const uint32_t bit = 1u << (y & 31u);
        fresh = !(atomicOr(&c.dq[y >> 5], bit) & bit);
      }
      const unsigned long long m = __ballot(fresh);
      if (fresh)  // past the slots: nd > cap aborts the unit after this node
        c.put_dirty(y, nd + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)));
      nd += (uint32_t)__popcll(m);
    }
  };
  // Every exit of the bucket loop is wave-uniform and seen as such by the compiler: nd,
  // loaded and the exit flags are scalars (ballots, readfirstlane), and the lanes' entry
  // loads (the only divergent branch of the loop body outside process()) join at the top
  // of the body, not at the latch ("the hang").
  bool first = true, ovf = false;
  D last = 0;
  for (;;) {
    // the lanes' entries: A members re-read their (relaxed) distance, new entries load
    if (pend && ea) ed = c.adist[lane];  // entry i sits in lane i and in slot i
    const uint32_t hi = min(nd, 64u);
    if (lane >= loaded && lane < hi) {
      ev = c.dlist[lane];
      er = c.gv.row(ev);  // in flight with the distance read: process() starts at the records
      ed = c.dist_a(ev, ea);
      pend = true;
    }
    loaded = hi;
    // bucket minimum over pending entries (lanes, then the LDS overflow beyond 64)
    D mn = pend ? ed : INF;
    unsigned long long anyb = __ballot(pend);
    for (uint32_t i0 = 64; i0 < nd; i0 += 64u) {
      const uint32_t i = i0 + lane;
      bool p = false;
      if (i < nd) {
        const D d = c.dist(c.dlist[i]);
        p = first || d > last;
        mn = (p && d < mn) ? d : mn;
      }
      anyb |= __ballot(p);
    }
    if (!anyb) break;
    mn = wave_min_t(mn);
    ++buckets;
    unsigned long long m = __ballot(pend && ed == mn);
    const uint32_t nd0 = nd;
    while (m) {
      const int k = __builtin_ctzll(m);
      m &= m - 1ull;
      process((uint32_t)__builtin_amdgcn_readlane((int)ev, k), mn,
              make_uint2((uint32_t)__builtin_amdgcn_readlane((int)er.x, k),
                         (uint32_t)__builtin_amdgcn_readlane((int)er.y, k)));
      nd = __builtin_amdgcn_readfirstlane(nd);
      if (nd > c.cap) {
        ovf = true;
        break;
      }
    }
    for (uint32_t i0 = 64; !ovf && i0 < nd0; i0 += 64u) {
      const uint32_t i = i0 + lane;
      uint32_t v = 0;
      bool hit = false;
      if (i < nd0) {
        v = c.dlist[i];
        const D d = c.dist(v);
        hit = (first || d > last) && d == mn;
      }
      unsigned long long mo = __ballot(hit);
      while (mo) {
        const int k = __builtin_ctzll(mo);
        mo &= mo - 1ull;
        const uint32_t vk = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
        process(vk, mn, c.gv.row(vk));
        nd = __builtin_amdgcn_readfirstlane(nd);
        if (nd > c.cap) {
          ovf = true;
          break;
        }
      }
    }
    if (ovf) break;
    if (pend && ed == mn) pend = false;
    first = false;
    last = mn;
    if (mn == INF) break;  // unreachable nodes expand nothing: this was the last bucket
    lds_fence();
  }
  if (ovf) return kGrpOverflow;
  if (DL && nchanged) {
    // delta output: the changed dirty nodes (A members, and nodes whose set changed) with
    // their new distance and next hops, from the overlays (slot k holds dlist[k])
    unsigned long long b = 0;
    if (nchanged > kDeltaBlock / 2u) {
      if (lane == 0) b = atomicAdd(c.dl.used, (unsigned long long)nchanged);
      b = readlane_t(b, 0);
    } else {
      if (c.pcur + nchanged > c.pend) {
        unsigned long long nbk = 0;
        if (lane == 0) nbk = atomicAdd(c.dl.used, (unsigned long long)kDeltaBlock);
        nbk = readlane_t(nbk, 0);
        c.pcur = nbk;
        c.pend = nbk + kDeltaBlock;
      }
      b = c.pcur;
      c.pcur += nchanged;
    }
    if (lane == 0) c.dl.off[c.uidx] = c.dl.base_of(b);
    for (uint32_t k0 = 0; k0 < nd; k0 += 64u) {
      const uint32_t k = k0 + lane;
      uint32_t v = 0;
      bool in_a = false, own = false;
      if (k < nd) {
        v = c.dlist[k];
        in_a = bit_of(c.ina, v);
        own = bit_of(c.nhm, v);
      }
      const bool ch = in_a || own;
      const unsigned long long m = __ballot(ch);
      const unsigned long long pos =
          b + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (ch && pos < c.dl.cap) {
        c.dl.node[pos] = v;
        const D dv = in_a ? c.adist[k] : c.bdist[v];
        c.dl.dist[pos] = dv == INF ? ~0ull : (unsigned long long)dv;
        const uint8_t* h = own ? c.anh + (size_t)k * nb : c.bnh + (size_t)v * nb;
        uint8_t* o = c.dl.nh + (size_t)pos * c.dl.nhb;
        for (uint32_t q = 0; q < c.dl.nhb; ++q) o[q] = q < nb ? h[q] : 0u;
      }
      b += (uint32_t)__popcll(m);
    }
  }
  if (c.prof && lane == 0) {
    pt3 = (long long)__builtin_amdgcn_s_memtime();
    atomicAdd(&c.prof[0], (unsigned long long)(pt1 - pt0));
    atomicAdd(&c.prof[1], (unsigned long long)(pt2 - pt1));
    atomicAdd(&c.prof[2], (unsigned long long)(pt3 - pt2));
    atomicAdd(&c.prof[3], 1ull);
    atomicAdd(&c.prof[4], (unsigned long long)na);
    atomicAdd(&c.prof[5], (unsigned long long)nd);
    atomicAdd(&c.prof[6], (unsigned long long)buckets);
    atomicAdd(&c.prof[7], (unsigned long long)nchanged);
  }
  __builtin_amdgcn_wave_barrier();  // the lane-0 branch joins here, not at the caller's latch
  return nchanged;
}

constexpr uint32_t kGrpMaxBlock = 512;
constexpr uint32_t kGrpProfWg = 4096;  // workgroups whose start / end times the profile keeps

// WPE: waves per SIMD the compiler must fit registers for (1: no constraint). Unconstrained
// the <= 32-bit-set variant takes 119 VGPRs, i.e. 4 waves per SIMD (16 per CU) whatever
// LDS allows; 7 (its default since round 4) forces 72 VGPRs at the price of 140 B of
// scratch spills per lane, and the 28 waves per CU the LDS layout allows win (kernel
// 3.66 -> 2.81 ms on the WAN).
template <typename D, bool LG, uint32_t W, int WPE, bool DL>
__global__ __launch_bounds__(kGrpMaxBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void whatif_group_kernel(
    DevGraph g, const uint32_t* links, uint32_t n_links, const uint32_t* sources, uint32_t n_src, uint32_t chunk,
    uint32_t lbig, uint32_t schunk,
    const uint64_t* base_dist, const uint8_t* base_nh, const uint64_t* base_tight, const uint16_t* base_tin,
    uint32_t nb, uint32_t unit, uint32_t cap, uint32_t heavy_first, uint32_t* changed_t, uint32_t* affected, uint32_t* ovf_src, uint32_t* ovf_link, uint32_t* ovf_unit,
    uint32_t* ctr, unsigned long long* prof, WhatifDelta dl) {
  constexpr D INF = (D)~(D)0;
  const long long kt0 = prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
  const unsigned long long wt0 = prof ? wall_clock64() : 0ull;  // workgroup span (100 MHz), tail analysis
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t s_item;
  const uint32_t V = g.V, E = g.E, tid = threadIdx.x, lane = __lane_id(), wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform to the compiler: per-wave LDS pointers stay scalar
  const uint32_t block = blockDim.x, waves = block >> 6;
  const uint32_t tw = (E + 63u) / 64u, vw = (V + 31u) / 32u;
  const GrpLayout lay = grp_layout(V, E, nb, sizeof(D), LG, waves, chunk, cap);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* wctl = smem;
  D* bdist = reinterpret_cast<D*>(base + lay.bdist);
  uint8_t* bnh = reinterpret_cast<uint8_t*>(base + lay.bnh);
  uint64_t* btight = reinterpret_cast<uint64_t*>(base + lay.btight);
  uint32_t* ulist = reinterpret_cast<uint32_t*>(base + lay.ulist);
  uint8_t* btin = reinterpret_cast<uint8_t*>(base + lay.btin);
  char* wb = base + lay.wave0 + wave * lay.wstride;
  GrpWave<D, LG, W> c;
  c.g = &g;
  if constexpr (LG) {
    // stage the compact graph once per workgroup (a launch serves many items)
    uint32_t* rowp = reinterpret_cast<uint32_t*>(base + lay.grow);
    uint2* crec = reinterpret_cast<uint2*>(base + lay.grec);
    uint8_t* nbrin = reinterpret_cast<uint8_t*>(base + lay.gnbr);
    uint32_t* ovlb = reinterpret_cast<uint32_t*>(base + lay.govl);
    for (uint32_t v = tid; v <= V; v += block) rowp[v] = g.row[v];
    for (uint32_t e = tid; e < E; e += block) {
      const uint4 r = g.erec[e];  // e = x -> col: {col | down | sink(col), w(col -> x), link, rev}
      const uint32_t col = r.x & ~(kEdgeDown | kNodeSink);
      crec[e] = make_uint2(col | ((r.x & kEdgeDown) ? 0x8000u : 0u) | (r.z << 16) | ((r.x & kNodeSink) ? 0x80000000u : 0u),
                           (g.w[e] & 0xFFFFu) | (r.y << 16));
      nbrin[e] = (uint8_t)g.nbr[r.w];
    }
    for (uint32_t i = tid; i < vw; i += block) ovlb[i] = g.ovl_bits[i];
    c.gv.rowp = rowp;
    c.gv.crec = crec;
    c.gv.nbrin = nbrin;
    c.gv.ovlb = ovlb;
  } else {
    c.gv.g = &g;
  }
  c.nb = nb;
  c.unit = unit != 0;
  // prof[15] != 0: workgroup start / end times only (no per-unit counters and their atomics)
  const bool tail_only = prof && prof[15] != 0ull;
  c.prof = tail_only ? nullptr : prof;
  c.dl = dl;
  c.pcur = c.pend = 0;
  c.bdist = bdist;
  c.bnh = bnh;
  c.btight = btight;
  c.tin = btin;
  c.ctl = reinterpret_cast<uint32_t*>(wb);
  c.ina = reinterpret_cast<uint32_t*>(wb + lay.w_ina);
  c.dq = reinterpret_cast<uint32_t*>(wb + lay.w_dq);
  c.nhm = reinterpret_cast<uint32_t*>(wb + lay.w_nhm);
  c.dec = reinterpret_cast<uint8_t*>(wb + lay.w_dec);
  c.didx = reinterpret_cast<uint8_t*>(wb + lay.w_didx);
  c.cap = cap;
  c.adist = reinterpret_cast<D*>(wb + lay.w_adist);
  c.anh = reinterpret_cast<uint8_t*>(wb + lay.w_anh);
  c.alist = reinterpret_cast<uint16_t*>(wb + lay.w_alist);
  c.dlist = reinterpret_cast<uint16_t*>(wb + lay.w_dlist);
  // items: every source's links [0, lbig) in chunks of `chunk`, then (the queue's tail, so
  // that the last workgroups finish together) its links [lbig, n_links) in chunks of `schunk`
  const uint32_t bchunks = (lbig + chunk - 1u) / chunk;
  const uint32_t schunks = lbig < n_links ? (n_links - lbig + schunk - 1u) / schunk : 0u;
  const uint32_t nbig = n_src * bchunks, items = nbig + n_src * schunks;
  unsigned long long* ist = tail_only ? prof + 16 + 2 * kGrpProfWg : nullptr;  // per-item stamps (tuning)
  for (uint32_t item = blockIdx.x; item < items;) {
    uint32_t j, l0, l1;
    if (item < nbig) {
      j = item / bchunks;
      l0 = (item - j * bchunks) * chunk;
      l1 = min(lbig, l0 + chunk);
    } else {
      const uint32_t k = item - nbig;
      j = k / schunks;
      l0 = lbig + (k - j * schunks) * schunk;
      l1 = min(n_links, l0 + schunk);
    }
    if (ist && lane == 0) ist[(size_t)(item * waves + wave) * 4u + 0u] = __builtin_amdgcn_s_memtime();
    c.src = sources[j];
    // stage source j's base rows (read once per item)
    const uint64_t* drow = base_dist + (size_t)j * V;
    for (uint32_t v = tid; v < V; v += block) {
      const uint64_t d = drow[v];
      bdist[v] = d == ~0ull ? INF : (D)d;
    }
    const uint8_t* hrow = base_nh + (size_t)j * V * nb;
    const uint32_t nbytes = V * nb;
    if (((reinterpret_cast<uintptr_t>(hrow) | nbytes) & 3u) == 0) {
      for (uint32_t i = tid; i < nbytes / 4u; i += block)
        reinterpret_cast<uint32_t*>(bnh)[i] = reinterpret_cast<const uint32_t*>(hrow)[i];
    } else {
      for (uint32_t i = tid; i < nbytes; i += block) bnh[i] = hrow[i];
    }
    const uint64_t* trow = base_tight + (size_t)j * tw;
    for (uint32_t i = tid; i < tw; i += block) btight[i] = trow[i];
    if (base_tin) {
      // the base SPF's tight in-degree row (rounds plan), four nodes per word
      const uint16_t* tr = base_tin + (size_t)j * V;
      for (uint32_t i = tid; i < (V + 4u) / 4u; i += block) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          const uint32_t v = 4u * i + q;
          w |= (v < V ? (uint32_t)tr[v] : 0u) << (8u * q);  // max_deg <= 255
        }
        reinterpret_cast<uint32_t*>(btin)[i] = w;
      }
    } else {
      for (uint32_t i = tid; i < (V + 4u) / 4u; i += block) reinterpret_cast<uint32_t*>(btin)[i] = 0;
    }
    if (tid == 0) wctl[0] = wctl[1] = wctl[2] = 0;  // [0] / [2] affected links listed, [1] next one to repair
    __syncthreads();
    if (!base_tin)
      for (uint32_t e = tid; e < E; e += block)  // base-tight in-degrees from the tight mask
        if ((btight[e >> 6] >> (e & 63u)) & 1ull) {
          const uint32_t v = c.gv.rec(e).col;
          atomicAdd(reinterpret_cast<uint32_t*>(btin) + (v >> 2), 1u << (8u * (v & 3u)));
        }
    // fused filter, a thread per link: a link with no base-tight edge changes nothing;
    // the others are listed with b, the head of their tight edge a->b (at most one
    // direction of a link is tight), so a repair starts without dependent loads. With
    // heavy_first, a unit whose b has no other base-tight in-edge (b's distance grows: A is
    // not empty, the long repairs) is listed from the front (wctl[0]), the others from the
    // back (wctl[2]): the item's last repairs are short ones, so its waves reach the item's
    // barrier closer together
    for (uint32_t i0 = l0; i0 < l1; i0 += block) {
      const uint32_t i = i0 + tid;
      bool hit = false;
      uint32_t bnode = 0;
      if (i < l1) {
        const uint32_t l = links[i];
        const uint2 ee = l < g.L ? g.ledge[l] : make_uint2(UINT32_MAX, UINT32_MAX);
        if (ee.x != UINT32_MAX) {
          const bool tx = (btight[ee.x >> 6] >> (ee.x & 63u)) & 1ull;
          hit = tx || ((btight[ee.y >> 6] >> (ee.y & 63u)) & 1ull);
          if (hit) bnode = g.adj[tx ? ee.x : ee.y] & ~kEdgeDown;
        }
        if (!hit) changed_t[(size_t)j * n_links + i] = 0;
      }
      const bool heavy = hit && (!heavy_first || btin[bnode] == 1u);
      const unsigned long long m = __ballot(heavy), ml = __ballot(hit && !heavy);
      uint32_t basei = 0, basel = 0;
      if (lane == 0 && m) basei = atomicAdd(&wctl[0], (uint32_t)__popcll(m));
      if (lane == 0 && ml) basel = atomicAdd(&wctl[2], (uint32_t)__popcll(ml));
      basei = __builtin_amdgcn_readfirstlane(__shfl(basei, 0));
      basel = __builtin_amdgcn_readfirstlane(__shfl(basel, 0));
      if (heavy)
        ulist[basei + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
            ((i - l0) << 16) | bnode;
      else if (hit)
        ulist[chunk - 1u - (basel + __builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)ml, 0u)))] =
            ((i - l0) << 16) | bnode;
    }
    __syncthreads();
    const uint32_t n_front = wctl[0], n_hit = n_front + wctl[2];
    if (ist && lane == 0) ist[(size_t)(item * waves + wave) * 4u + 1u] = __builtin_amdgcn_s_memtime();
    if (tid == 0 && n_hit) atomicAdd(affected, n_hit);  // per item: no counter live across the repairs
    // waves take the listed units one at a time: the item ends within one repair of balance
    for (;;) {
      uint32_t idx = 0;
      if (lane == 0) idx = atomicAdd(&wctl[1], 1u);
      idx = __builtin_amdgcn_readfirstlane(__shfl(idx, 0));
      if (idx >= n_hit) break;
      const uint32_t ent = __builtin_amdgcn_readfirstlane(ulist[idx < n_front ? idx : chunk - 1u - (idx - n_front)]);
      const uint32_t i = l0 + (ent >> 16);
      c.link = links[i];  // first needed in step (2): the load overlaps step (1)
      c.uidx = i * n_src + j;
      const uint32_t cnt = grp_repair<D, LG, W, DL>(c, lane, V, ent & 0xFFFFu);
      if (lane == 0) {
        // results source-major (changed_t[j][i]): an item's units share cache lines, where the
        // link-major API rows put every unit of an item on a line of its own (whatif_transpose)
        changed_t[(size_t)j * n_links + i] = cnt != kGrpOverflow ? cnt : 0u;
        if (cnt == kGrpOverflow) {  // more dirty nodes than slots: re-solved after the launch (openr_spf_whatif)
          const uint32_t k = atomicAdd(&affected[1], 1u);
          ovf_src[k] = c.src;
          ovf_link[k] = c.link;
          ovf_unit[k] = i * n_src + j;
        }
      }
      __builtin_amdgcn_wave_barrier();  // the lane-0 branch joins here: the latch is taken by the whole wave
    }
    if (ist && lane == 0) ist[(size_t)(item * waves + wave) * 4u + 2u] = __builtin_amdgcn_s_memtime();
    __syncthreads();  // every wave is done with this item's shared rows and s_item
    if (ist && lane == 0) ist[(size_t)(item * waves + wave) * 4u + 3u] = __builtin_amdgcn_s_memtime();
    if (tid == 0) s_item = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    item = s_item;
  }
  if (prof && !tail_only && lane == 0) {
    atomicAdd(&prof[8], (unsigned long long)((long long)__builtin_amdgcn_s_memtime() - kt0));  // wave lifetime
    atomicAdd(&prof[9], 1ull);
  }
  if (prof && tid == 0 && blockIdx.x < kGrpProfWg) {
    prof[16 + blockIdx.x] = wt0;
    prof[16 + kGrpProfWg + blockIdx.x] = wall_clock64();
  }
  bfs::retire_workgroup(ctr, nullptr);
}

// changed[i * n_src + j] = changed_t[j * n_links + i] through 64 x 64 LDS tiles (both sides
// coalesced)
__global__ __launch_bounds__(256) void whatif_transpose(const uint32_t* changed_t, uint32_t* changed, uint32_t n_links,
                                                        uint32_t n_src) {
  __shared__ uint32_t tile[64][65];
  const uint32_t tl = (n_links + 63u) / 64u, ts = (n_src + 63u) / 64u;
  for (uint32_t t = blockIdx.x; t < tl * ts; t += gridDim.x) {
    const uint32_t i0 = (t % tl) * 64u, j0 = (t / tl) * 64u;
    const uint32_t c = threadIdx.x & 63u, r0 = threadIdx.x >> 6;
    for (uint32_t r = r0; r < 64u; r += 4u) {  // rows of changed_t: sources j0 + r, links i0 + c
      const uint32_t j = j0 + r, i = i0 + c;
      if (j < n_src && i < n_links) tile[r][c] = changed_t[(size_t)j * n_links + i];
    }
    __syncthreads();
    for (uint32_t r = r0; r < 64u; r += 4u) {  // rows of changed: links i0 + r, sources j0 + c
      const uint32_t i = i0 + r, j = j0 + c;
      if (i < n_links && j < n_src) changed[(size_t)i * n_src + j] = tile[c][r];
    }
    __syncthreads();
  }
}

// --- what-if delta compaction (openr_spf_whatif_delta) --------------------------------
// ptr[0, n] = exclusive scan of changed[0, n) (u64), in three passes over tiles of
// kScanTile units: tile sums, a scan of the sums in one workgroup, tile-local scans.
constexpr uint32_t kScanTile = 4096;  // 256 threads x 16 units

__device__ __forceinline__ unsigned long long block_excl_scan256(unsigned long long x, unsigned long long* tmp,
                                                                 unsigned long long& total) {
  const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
  unsigned long long inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) tmp[wave] = inc;
  __syncthreads();
  unsigned long long before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += tmp[w];
  total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return before + inc - x;
}

__global__ __launch_bounds__(256) void delta_tile_sums(const uint32_t* c, size_t n, unsigned long long* tsum) {
  __shared__ unsigned long long tmp[4];
  const size_t t0 = (size_t)blockIdx.x * kScanTile;
  unsigned long long x = 0;
  for (uint32_t k = 0; k < kScanTile / 256u; ++k) {
    const size_t u = t0 + (size_t)k * 256u + threadIdx.x;
    if (u < n) x += c[u];
  }
  unsigned long long total;
  (void)block_excl_scan256(x, tmp, total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void delta_scan_sums(unsigned long long* tsum, uint32_t nt) {
  __shared__ unsigned long long tmp[4];
  unsigned long long carry = 0;
  for (uint32_t i0 = 0; i0 < nt; i0 += 256u) {
    const uint32_t i = i0 + threadIdx.x;
    const unsigned long long x = i < nt ? tsum[i] : 0ull;
    unsigned long long total;
    const unsigned long long ex = block_excl_scan256(x, tmp, total);
    if (i < nt) tsum[i] = carry + ex;
    carry += total;
  }
}

__global__ __launch_bounds__(256) void delta_tile_scan(const uint32_t* c, size_t n, const unsigned long long* tsum,
                                                       unsigned long long* ptr) {
  __shared__ unsigned long long tmp[4];
  const size_t t0 = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * (kScanTile / 256u);
  uint32_t v[kScanTile / 256u];
  unsigned long long x = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanTile / 256u; ++k) {
    v[k] = t0 + k < n ? c[t0 + k] : 0u;
    x += v[k];
  }
  unsigned long long total;
  unsigned long long at = tsum[blockIdx.x] + block_excl_scan256(x, tmp, total);
#pragma unroll
  for (uint32_t k = 0; k < kScanTile / 256u; ++k) {
    if (t0 + k < n) ptr[t0 + k] = at;
    at += v[k];
  }
  if (t0 < n && t0 + kScanTile / 256u >= n) ptr[n] = at;  // the thread holding unit n - 1: the total
}

// unit u's entries from its pool slots [off[u], off[u] + changed[u]) to the CSR slots
// [ptr[u], ptr[u + 1]) (the order inside a unit is kept). A wave takes 64 consecutive
// units, whose CSR slots are one contiguous range, and gives each lane one slot of it at a
// time: the lane finds its unit by a binary search over the 64 offsets in LDS. Writes are
// coalesced and every lane has work whatever the units' sizes (a thread per unit left
// most lanes idle on a WAN unit's ~6 entries: 0.76 ms per step, r06).
__global__ __launch_bounds__(256) void delta_gather(size_t n, const uint32_t* off, const unsigned long long* ptr,
                                                    WhatifDelta pool, uint32_t* node, unsigned long long* dist,
                                                    uint8_t* nh) {
  __shared__ unsigned long long sp[4][65];
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned long long* p = sp[wave];
  const size_t groups = (n + 63u) / 64u;
  for (size_t gi = (size_t)blockIdx.x * 4u + wave; gi < groups; gi += (size_t)gridDim.x * 4u) {
    const size_t u0 = gi * 64u;
    p[lane] = ptr[min(u0 + lane, n)];
    if (lane == 0) p[64] = ptr[min(u0 + 64u, n)];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const unsigned long long b0 = p[0], b1 = p[64];
    for (unsigned long long t = b0 + lane; t < b1; t += 64u) {
      uint32_t lo = 0, hi = 63;  // the last unit whose first slot is <= t (empty units share it)
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (p[mid] <= t) lo = mid;
        else hi = mid - 1u;
      }
      const size_t src = off[u0 + lo] + (size_t)(t - p[lo]);
      node[t] = pool.node[src];
      dist[t] = pool.dist[src];
      const uint8_t* hs = pool.nh + src * pool.nhb;
      uint8_t* hd = nh + (size_t)t * pool.nhb;
      for (uint32_t q = 0; q < pool.nhb; ++q) hd[q] = hs[q];
    }
    __builtin_amdgcn_wave_barrier();  // every lane's reads of p precede the next group's writes
  }
}

__global__ __launch_bounds__(256) void iota_u32(uint32_t* p, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) p[i] = i;
}

uint32_t grid_for(uint64_t items, uint32_t per_block, int num_cus) {
  const uint64_t want = (items + per_block - 1) / per_block;
  const uint64_t cap = (uint64_t)num_cus * 8u;
  return (uint32_t)std::max<uint64_t>(1, std::min(want, cap));
}

}  // namespace

hipError_t launch_whatif_filter(const DevGraph& g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                                uint32_t n_src, const uint64_t* base_tight, uint32_t* changed, uint32_t* wsrc,
                                uint32_t* wlink, uint32_t* wunit, uint32_t* wcount, int num_cus, hipStream_t s) {
  hipError_t err = hipMemsetAsync(wcount, 0, sizeof(uint32_t), s);
  if (err != hipSuccess) return err;
  const uint64_t total = (uint64_t)n_links * n_src;
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(whatif_filter, dim3(grid_for(total, 256u, num_cus)), dim3(256), 0, s, g.ledge, g.L,
                     (g.E + 63u) / 64u, links, n_links, sources, n_src, base_tight, changed, wsrc, wlink, wunit,
                     wcount);
  return hipGetLastError();
}

hipError_t launch_rows_compare(uint32_t n, uint32_t V, uint32_t nb, const uint64_t* dist, const uint8_t* nh,
                               const uint64_t* base_dist, const uint8_t* base_nh, const uint32_t* wunit,
                               uint32_t n_src, uint32_t* changed, const WhatifDelta& dl, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(rows_compare, dim3(grid_for(n, 1u, num_cus)), dim3(256), 0, s, n, V, nb, dist, nh, base_dist,
                     base_nh, wunit, n_src, changed, dl);
  return hipGetLastError();
}

uint32_t whatif_incr_lds_bytes(uint32_t V, uint32_t nb, bool dist64) {
  if (V > 65535u || nb > 32u) return 0;
  const uint32_t t = incr_layout(V, nb, dist64 ? 8u : 4u).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_whatif_incr(const DevGraph& g, const uint32_t* wsrc, const uint32_t* wlink, const uint32_t* wunit,
                              uint32_t count, uint32_t n_src, const uint64_t* base_dist, const uint8_t* base_nh,
                              uint32_t nb, bool unit_cost, bool dist64, uint32_t* changed, uint32_t* ctr,
                              int num_cus, hipStream_t s) {
  if (!count) return hipSuccess;
  const uint32_t lds = whatif_incr_lds_bytes(g.V, nb, dist64);
  if (!lds) return hipErrorInvalidValue;
  const uint32_t grid = blocks_for(count, lds, num_cus, 64u);
  auto k = dist64 ? whatif_incr_kernel<unsigned long long> : whatif_incr_kernel<uint32_t>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, s, g, wsrc, wlink, wunit, count, n_src, base_dist, base_nh, nb,
                     (uint32_t)unit_cost, changed, ctr);
  return hipGetLastError();
}

namespace {
// LDS graph eligibility: ids / link ids / metrics fit the compact record, next-hop bits a byte
bool grp_lds_graph_ok(const DevGraph& g, uint32_t w_max, uint32_t nh_bits) {
  return g.V <= 32767u && g.L <= 32767u && w_max <= 65535u && nh_bits <= 256u &&
         bfs::env_u32("OPENR_SPF_WHATIF_LDSG", 0u, 0u, 1u);  // measured slower (fewer waves): opt-in
}
}  // namespace

uint32_t whatif_group_lds_bytes(uint32_t V, uint32_t E, uint32_t nb, bool dist64, uint32_t max_deg) {
  if (V > 65535u || nb > 32u || max_deg > 255u) return 0;  // u16 ids, u8 in-degree counters
  const uint32_t t = grp_layout(V, E, nb, dist64 ? 8u : 4u, false, 4, kGrpMaxChunk, kGrpMaxCap).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_whatif_group(const DevGraph& g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                               uint32_t n_src, const uint64_t* base_dist, const uint8_t* base_nh,
                               const uint64_t* base_tight, const uint16_t* base_tin, uint32_t nb, bool unit_cost,
                               bool dist64, uint32_t w_max,
                               uint32_t nh_bits, uint32_t* changed, uint32_t* changed_t, uint32_t* affected,
                               uint32_t* ovf_src, uint32_t* ovf_link, uint32_t* ovf_unit, uint32_t* ctr,
                               const WhatifDelta& dl, int num_cus, hipStream_t s) {
  // [0] affected units, [1] units listed for a re-solve
  hipError_t err = hipMemsetAsync(affected, 0, 2u * sizeof(uint32_t), s);
  if (err != hipSuccess || !n_links || !n_src) return err;
  // distances as u16 when every finite one fits (V * w_max < 0xFFFF): half the LDS rows,
  // more workgroups per CU
  const bool d16 = (uint64_t)g.V * (unit_cost ? 1u : w_max) < 0xFFFFull && !bfs::env_u32("OPENR_SPF_WHATIF_D32", 0u, 0u, 1u);
  const uint32_t db = d16 ? 2u : dist64 ? 8u : 4u;
  // the LDS-graph variant (opt-in) with as many waves per workgroup (one workgroup per
  // CU) as fit, else the global-graph variant at kGrpWaves per workgroup
  bool lg = false;
  // Few dirty slots per wave (LDS per wave ~3.5 KB on the WAN: 7 workgroups of 4 waves per
  // CU); the units that outgrow them are listed for a re-solve. WAN kernel time (cap /
  // waves, round 3): 255 / 3 4.57 ms, 160 / 3 4.07, 128 / 4 3.66, 96 / 4 3.46, 64 / 4 3.09,
  // 48 / 4 2.90 (fewer slots: more re-solves; the step is shortest at 128 / 4: 5.02 ms,
  // against 5.11 at 112, 5.19 at 96, 5.09 at 160; at 7 waves per SIMD, round 4: 96 4.36,
  // 112 4.25, 128 4.16, 144 4.17, 160 4.15, 192 4.21 ms). A second pass repairing the
  // overflowed units with every slot on one wavefront each was slower than the re-solves
  // (5.34 vs 5.18 ms, round 3; 4.68 vs 4.16 ms, round 4) and was removed.
  uint32_t waves = bfs::env_u32("OPENR_SPF_WHATIF_WAVES", kGrpWaves, 1u, 8u);  // tuning / tests
  const uint32_t cap = bfs::env_u32("OPENR_SPF_WHATIF_CAP", kGrpCap1, 1u, kGrpMaxCap);  // tests force small caps
  auto layout_bytes = [&](bool l, uint32_t w, uint32_t ch) { return grp_layout(g.V, g.E, nb, db, l, w, ch, cap).total; };
  if (grp_lds_graph_ok(g, w_max, nh_bits)) {
    for (uint32_t w = kGrpMaxBlock / 64u; w >= 2u; --w) {
      if (layout_bytes(true, w, kGrpMaxChunk) <= kMaxLds) {
        lg = true;
        waves = w;
        break;
      }
    }
  }
  if (!lg && layout_bytes(false, waves, kGrpMaxChunk) > kMaxLds) waves = 4;
  if (!lg && layout_bytes(false, waves, kGrpMaxChunk) > kMaxLds) return hipErrorInvalidValue;
  const uint32_t block = 64u * waves;
  auto slots_for = [&](uint32_t bytes) {
    return (uint64_t)num_cus * std::max<uint32_t>(1u, std::min<uint32_t>(kMaxLds / bytes, 2048u / block));
  };
  // work items of (source, chunk of links): ~8 per resident workgroup, so the tail is short
  const uint64_t slots0 = slots_for(layout_bytes(lg, waves, kGrpMaxChunk));
  // ~3 full-size items per resident workgroup, then (below) the last fifth of every
  // source's links in quarter-size chunks: an item ends at a workgroup barrier where the
  // waves that are done wait for the last repair (~10 % of the wave time at 8 items per
  // workgroup, OPENR_SPF_WHATIF_TAIL), so items are large while the queue is long and small
  // at its end, where the workgroups must finish together. WAN step 3.486 -> 3.375 ms
  // (IPW 8 / no tail split -> 3 / 20 % / 4, interleaved; r06)
  const uint32_t ipw = bfs::env_u32("OPENR_SPF_WHATIF_IPW", 3u, 1u, 64u);
  uint64_t cps = (ipw * slots0 + n_src - 1u) / n_src;
  cps = std::max<uint64_t>(1u, std::min<uint64_t>(cps, n_links));
  uint32_t chunk = (uint32_t)((n_links + cps - 1u) / cps);
  chunk = std::min(chunk, kGrpMaxChunk);
  const uint32_t lds = layout_bytes(lg, waves, chunk);  // the list sized to the chunk
  const uint64_t slots = slots_for(lds);
  // the last part of every source's links in smaller chunks at the queue's end
  // (OPENR_SPF_WHATIF_TAILFRAC percent, 0: one chunk size; OPENR_SPF_WHATIF_TAILDIV: the split)
  const uint32_t tail_pct = bfs::env_u32("OPENR_SPF_WHATIF_TAILFRAC", 20u, 0u, 100u);
  const uint32_t tail_div = bfs::env_u32("OPENR_SPF_WHATIF_TAILDIV", 4u, 1u, 64u);
  uint32_t lbig = n_links, schunk = chunk;
  if (tail_pct && tail_div > 1u && chunk >= tail_div) {
    const uint64_t keep = (uint64_t)n_links * (100u - tail_pct) / 100u;
    lbig = (uint32_t)(keep / chunk * chunk);
    schunk = (chunk + tail_div - 1u) / tail_div;
  }
  const uint64_t items = (uint64_t)n_src * ((lbig + chunk - 1u) / chunk) +
                         (lbig < n_links ? (uint64_t)n_src * ((n_links - lbig + schunk - 1u) / schunk) : 0u);
  if (items >= (1ull << 32)) return hipErrorInvalidValue;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(slots, items);
  // tuning aid: per-phase cycle sums and set sizes, printed after the launch
  static unsigned long long* prof_buf = nullptr;
  unsigned long long* prof = nullptr;
  if (prof_enabled()) {
    const size_t words = 16u + 2u * kGrpProfWg + 4u * 8u * 65536u;  // + per-item stamps (<= 64 K items x 8 waves)
    if (!prof_buf && hipMalloc(&prof_buf, words * sizeof(unsigned long long)) != hipSuccess) prof_buf = nullptr;
    prof = prof_buf;
    if (prof) {
      (void)hipMemsetAsync(prof, 0, words * sizeof(unsigned long long), s);
      // OPENR_SPF_WHATIF_TAIL=1: only the workgroup times (the per-unit counters' atomics
      // slow the kernel ~40x and distort its tail)
      static const unsigned long long one = 1ull;
      if (bfs::env_u32("OPENR_SPF_WHATIF_TAIL", 0u, 0u, 1u))
        (void)hipMemcpyAsync(prof + 15, &one, sizeof(one), hipMemcpyHostToDevice, s);
    }
  }
  // base-tight in-degrees from the base SPF's rows when it left them (OPENR_SPF_WHATIF_TIN=0:
  // recounted from the tight mask per item, A/B)
  const uint16_t* tin = bfs::env_u32("OPENR_SPF_WHATIF_TIN", 1u, 0u, 1u) ? base_tin : nullptr;
  // long repairs first within an item (needs the staged in-degrees; OPENR_SPF_WHATIF_ORDER=0: link order)
  const uint32_t heavy_first = tin && bfs::env_u32("OPENR_SPF_WHATIF_ORDER", 1u, 0u, 1u) ? 1u : 0u;
  // the <= 32-bit-set variant is compiled for 7 waves per SIMD, the occupancy its LDS
  // layout allows (28 waves per CU): WAN step 5.03 -> 4.17 ms (unconstrained: 119 VGPRs,
  // 4 waves per SIMD; 5 waves: 4.56 ms), round 4
#define OPENR_GRP_LAUNCH(DT, LGV)                                                                              \
  do {                                                                                                         \
    auto k = dl.node ? (nb <= 4u ? whatif_group_kernel<DT, LGV, 1, 7, true>                                  \
                                 : whatif_group_kernel<DT, LGV, kGrpNhWords, 1, true>)                         \
                     : (nb <= 4u ? whatif_group_kernel<DT, LGV, 1, 7, false>                                 \
                                 : whatif_group_kernel<DT, LGV, kGrpNhWords, 1, false>);                       \
    err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,    \
                              (int)lds);                                                                       \
    if (err != hipSuccess) return err;                                                                         \
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, s, g, links, n_links, sources, n_src, chunk, lbig, schunk, \
                       base_dist, \
                       base_nh, base_tight, tin, nb, (uint32_t)unit_cost, cap, heavy_first, changed_t, affected,     \
                       ovf_src, ovf_link,                                                                      \
                       ovf_unit, ctr, prof, dl);                                                               \
  } while (0)
  if (d16) {
    if (lg) OPENR_GRP_LAUNCH(uint16_t, true);
    else OPENR_GRP_LAUNCH(uint16_t, false);
  } else if (dist64) {
    if (lg) OPENR_GRP_LAUNCH(unsigned long long, true);
    else OPENR_GRP_LAUNCH(unsigned long long, false);
  } else {
    if (lg) OPENR_GRP_LAUNCH(uint32_t, true);
    else OPENR_GRP_LAUNCH(uint32_t, false);
  }
#undef OPENR_GRP_LAUNCH
  err = hipGetLastError();
  if (err == hipSuccess) {
    const uint32_t tiles = ((n_links + 63u) / 64u) * ((n_src + 63u) / 64u);
    hipLaunchKernelGGL(whatif_transpose, dim3(std::min<uint32_t>(tiles, (uint32_t)num_cus * 8u)), dim3(256), 0, s,
                       changed_t, changed, n_links, n_src);
    err = hipGetLastError();
  }
  if (err == hipSuccess && prof) {
    unsigned long long h[16];
    if (hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess) {
      const double u = h[3] ? (double)h[3] : 1.0;
      std::fprintf(stderr,
                   "whatif_group: lds_graph=%d waves=%u grid=%u chunk=%u units=%llu | cycles/unit: A %.0f dist %.0f "
                   "nh %.0f | |A| %.2f dirty %.2f buckets %.2f changed %.2f | wave lifetime %.0f x %llu, repair "
                   "share %.2f\n",
                   (int)lg, waves, grid, chunk, h[3], h[0] / u, h[1] / u, h[2] / u, h[4] / u, h[5] / u, h[6] / u,
                   h[7] / u, h[9] ? (double)h[8] / h[9] : 0.0, h[9],
                   h[8] ? (double)(h[0] + h[1] + h[2]) / (double)h[8] : 0.0);
      // the launch's tail: workgroup end times against the last one (100 MHz clock)
      const uint32_t nw = std::min<uint32_t>(grid, kGrpProfWg);
      std::vector<unsigned long long> t((size_t)2 * nw);
      if (hipMemcpy(t.data(), prof + 16, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess &&
          hipMemcpy(t.data() + nw, prof + 16 + kGrpProfWg, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost) ==
              hipSuccess && nw) {
        unsigned long long t0 = ~0ull, t1 = 0;
        for (uint32_t b = 0; b < nw; ++b) {
          t0 = std::min(t0, t[b]);
          t1 = std::max(t1, t[nw + b]);
        }
        std::vector<double> ends(nw), starts(nw);
        double busy = 0.0;
        for (uint32_t b = 0; b < nw; ++b) {
          starts[b] = (double)(t[b] - t0) / 100.0;
          ends[b] = (double)(t[nw + b] - t0) / 100.0;
          busy += ends[b] - starts[b];
        }
        std::sort(ends.begin(), ends.end());
        std::sort(starts.begin(), starts.end());
        const double span = (double)(t1 - t0) / 100.0;
        if (items <= 65536u) {
          const size_t ns = (size_t)items * waves * 4u;
          std::vector<unsigned long long> it(ns);
          if (hipMemcpy(it.data(), prof + 16 + 2 * kGrpProfWg, ns * sizeof(unsigned long long), hipMemcpyDeviceToHost) ==
              hipSuccess) {
            double st = 0, un = 0, wt = 0, n = 0;
            for (size_t q = 0; q + 3 < ns; q += 4) {
              if (!it[q] || !it[q + 3]) continue;
              st += (double)(it[q + 1] - it[q]);
              un += (double)(it[q + 2] - it[q + 1]);
              wt += (double)(it[q + 3] - it[q + 2]);
              n += 1;
            }
            if (n) std::fprintf(stderr, "whatif_group items: %llu items, per wave-item cycles: stage+filter %.0f, units %.0f, barrier wait %.0f\n",
                                (unsigned long long)items, st / n, un / n, wt / n);
          }
        }
        std::fprintf(stderr,
                     "whatif_group tail: span %.1f us, workgroups %u; starts p50 %.1f p90 %.1f max %.1f; ends p10 %.1f "
                     "p50 %.1f p90 %.1f p99 %.1f max %.1f us; workgroup-time / (span x resident %u) %.3f\n",
                     span, nw, starts[nw / 2], starts[nw * 9 / 10], starts.back(), ends[nw / 10], ends[nw / 2],
                     ends[nw * 9 / 10], ends[nw * 99 / 100], ends.back(), (uint32_t)std::min<uint64_t>(nw, slots),
                     busy / (span * (double)std::min<uint64_t>(nw, slots)));
      }
    }
  }
  return err;
}

hipError_t launch_delta_scan(const uint32_t* changed, size_t n, unsigned long long* tsum, unsigned long long* ptr,
                             hipStream_t s) {
  const size_t nt = (n + kScanTile - 1) / kScanTile;
  if (nt > 0xFFFFFFFFull) return hipErrorInvalidValue;
  if (!n) return hipMemsetAsync(ptr, 0, sizeof(unsigned long long), s);
  hipLaunchKernelGGL(delta_tile_sums, dim3((uint32_t)nt), dim3(256), 0, s, changed, n, tsum);
  hipLaunchKernelGGL(delta_scan_sums, dim3(1), dim3(256), 0, s, tsum, (uint32_t)nt);
  hipLaunchKernelGGL(delta_tile_scan, dim3((uint32_t)nt), dim3(256), 0, s, changed, n, tsum, ptr);
  return hipGetLastError();
}

hipError_t launch_delta_gather(const uint32_t* changed, size_t n, const uint32_t* off, const unsigned long long* ptr,
                               const WhatifDelta& pool, uint32_t* node, unsigned long long* dist, uint8_t* nh,
                               int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  (void)changed;  // the unit sizes are ptr's differences
  const uint32_t grid = (uint32_t)std::min<size_t>((n + 255u) / 256u, (size_t)num_cus * 16u);
  hipLaunchKernelGGL(delta_gather, dim3(grid), dim3(256), 0, s, n, off, ptr, pool, node, dist, nh);
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* p, uint32_t n, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(iota_u32, dim3(grid_for(n, 256u, num_cus)), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

}  // namespace openr_spf
