// spf_rounds.hip — general-metric SPF kernel for shallow graphs: distance rounds, then
// next hops in topological order of the shortest-path DAG. One wavefront per solve.
//
// Semantics: LinkState::runSpf (/root/reference/openr/decision/LinkState.cpp:808-882)
// in closed form for strictly positive metrics:
//   dist(v) = shortest distance over usable edges; overloaded nodes other than the
//             source are reached but never expanded (:831-838);
//   nh(v)   = OR over tight in-edges u->v of (u == src ? {v} : nh(u))  (:857-873),
//   u->v tight iff usable, u may expand and dist[u] + w(u->v) == dist[v].
//
// The fringe kernel (spf_fringe.hip) settles one bucket of width w_min per step, so a
// solve costs one dependent chain of L2 loads per DISTINCT distance (~150-200 on the
// 1k-node WAN with metrics U[1,64]). Here the sequential steps scale with the HOP depth
// instead (~10 on the WAN):
//   1. distance rounds (Bellman-Ford over a frontier): every node whose distance dropped
//      in the last round relaxes its out-edges with LDS atomicMin; a node re-enters the
//      next frontier at most once per round (an LDS bitmap dedups);
//   2. tight in-degree of every reached node (lane per node over its in-edges);
//   3. Kahn rounds over the tight DAG: a node whose tight in-degree reached 0 has its
//      final next-hop set; it ORs it into its tight successors and decrements them.
// Chosen per graph when the sampled hop depth is small (spf_capi.hip); the fringe kernel
// keeps deep or chain-like graphs. Integer work only, no MFMA.
#include <algorithm>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;
using namespace bfs;

constexpr uint32_t kWave = 64;

struct RoundsLayout {
  uint32_t dist, nh, cnt, fa, fb, inq, ign, alist, total;
};

__host__ __device__ inline RoundsLayout rounds_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t nh_words,
                                                      uint32_t dist_bytes) {
  RoundsLayout l;
  uint32_t off = 16;  // control: [0] next-frontier append counter
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.dist = take(dist_bytes * V);
  l.nh = take(4u * nh_words);
  l.cnt = take(2u * V);
  l.fa = take(2u * V);
  l.fb = take(2u * V);
  l.inq = take(4u * ((V + 31u) / 32u));
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.alist = has_ign ? take(2u * V) : 0u;  // seeded re-solves: the nodes whose distance grows
  l.total = off;
  return l;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Seeded start of a re-solve with an ignore set (what-if units too large for the repair
// kernel's slots, round 4): the base SPF's distances, except the set A of nodes whose
// every base-tight in-edge is lost — over an ignored link, or out of a member of A —
// which restart at their best entry from outside A. Nodes outside A keep their base
// distance (a base shortest path avoids the ignored links), so the distance rounds then
// run over A alone instead of the whole graph. Tight edges come from the base tight mask
// (seed_tight). Leaves the first frontier (A's members with a finite entry, inq bits set)
// in cur and returns its size.
template <typename D, uint32_t BLOCK>
__device__ uint32_t seed_from_base(const DevGraph& g, const SolveArgs& a, uint32_t sid, uint32_t src, D* dist,
                                   uint16_t* cnt, uint16_t*& cur, uint16_t*& nxt, uint32_t* inq, const uint32_t* ign,
                                   uint16_t* alist, uint32_t* ctl, uint32_t& r, uint32_t tid, uint32_t tight_words,
                                   uint32_t& na_out) {
  constexpr D INF = (D)~(D)0;
  auto sync = [&]() {
    if constexpr (BLOCK == kWave) lds_fence();
    else __syncthreads();
  };
  const uint32_t V = g.V;
  const uint32_t j = a.seed_unit[sid] % a.seed_nsrc;
  if (a.seed_changed && tid == 0) a.seed_changed[a.seed_unit[sid]] = 0;  // counted at the end
  const uint64_t* bd = a.seed_dist + (size_t)j * V;
  const uint64_t* bt = a.seed_tight + (size_t)j * tight_words;
  auto tight = [&](uint32_t e) { return ((bt[e >> 6] >> (e & 63u)) & 1ull) != 0; };
  // (a) base distances; live base-tight in-degree of every node (in-edges over an ignored
  //     link are lost); A's seeds: nodes that had tight in-edges and lost them all
  if (a.seed_tin) {
    // the base SPF's tight in-degree row, less the tight edges of the ignored links (one
    // lane per listed link; a link listed twice counts once)
    uint32_t* const ac = &ctl[r % 3u];
    if (tid == 0) ctl[(r + 1u) % 3u] = 0;
    const uint16_t* bc = a.seed_tin + (size_t)j * V;
    for (uint32_t v = tid; v < V; v += BLOCK) {
      const uint64_t b = bd[v];
      dist[v] = b == UINT64_MAX ? INF : (D)b;
      cnt[v] = bc[v];
    }
    sync();
    const uint32_t i0 = a.ign_ptr[sid], i1 = a.ign_end ? a.ign_end[sid] : a.ign_ptr[sid + 1];
    for (uint32_t i = i0 + tid; i < i1; i += BLOCK) {
      const uint32_t l = a.ign_links[i];
      bool dup = l >= g.L;
      for (uint32_t k = i0; k < i && !dup; ++k) dup = a.ign_links[k] == l;
      if (dup) continue;
      const uint2 le = g.ledge[l];
      for (int h = 0; h < 2; ++h) {
        const uint32_t e = h ? le.y : le.x;
        if (e == UINT32_MAX || !tight(e)) continue;
        const uint32_t v = g.adj[e] & ~kEdgeDown;
        const uint32_t sh = 16u * (v & 1u);
        const uint32_t old = atomicSub(reinterpret_cast<uint32_t*>(cnt) + (v >> 1), 1u << sh);
        if (((old >> sh) & 0xFFFFu) == 1u) cur[atomicAdd(ac, 1u)] = (uint16_t)v;
      }
    }
    sync();
  } else {
    uint32_t* const ac = &ctl[r % 3u];
    if (tid == 0) ctl[(r + 1u) % 3u] = 0;
    for (uint32_t v = tid; v < V; v += BLOCK) {
      const uint64_t b = bd[v];
      dist[v] = b == UINT64_MAX ? INF : (D)b;
      uint32_t live = 0, all = 0;
      if (b != UINT64_MAX && v != src) {
        const uint2 rr = g.row2[v];
        for (uint32_t e = rr.x; e < rr.y; ++e) {
          const uint4 rec = g.erec[e];  // v->u: {u | down | sink(u), w(u->v), link, rev}
          if (!tight(rec.w)) continue;
          ++all;
          live += test_bit(ign, rec.z) ? 0u : 1u;
        }
      }
      cnt[v] = (uint16_t)live;
      if (all && !live) cur[atomicAdd(ac, 1u)] = (uint16_t)v;
    }
    sync();
  }
  if (a.prof_solve && tid == 0) a.prof_solve[10 * (size_t)sid + 1] = wall_clock64();
  uint32_t n = __builtin_amdgcn_readfirstlane(ctl[r % 3u]);
  ++r;
  // (b) A: rounds down the live base-tight out-edges of A's members (listed in alist)
  uint32_t na = 0;
  while (n) {
    uint32_t* const ac = &ctl[r % 3u];
    if (tid == 0) ctl[(r + 1u) % 3u] = 0;
    for (uint32_t i = tid; i < n; i += BLOCK) {
      const uint32_t u = cur[i];
      alist[na + i] = (uint16_t)u;
      dist[u] = INF;  // re-solved below
      const uint2 rr = g.row2[u];
      for (uint32_t e = rr.x; e < rr.y; ++e) {
        if (!tight(e) || test_bit(ign, g.lid[e])) continue;  // an ignored link's loss counted in (a)
        const uint32_t v = g.adj[e] & ~kEdgeDown;
        const uint32_t sh = 16u * (v & 1u);
        const uint32_t old = atomicSub(reinterpret_cast<uint32_t*>(cnt) + (v >> 1), 1u << sh);
        if (((old >> sh) & 0xFFFFu) == 1u) nxt[atomicAdd(ac, 1u)] = (uint16_t)v;
      }
    }
    na += n;
    sync();
    n = __builtin_amdgcn_readfirstlane(*ac);
    ++r;
    uint16_t* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (a.prof_solve && tid == 0) {
    a.prof_solve[10 * (size_t)sid + 2] = wall_clock64();
    a.prof_solve[10 * (size_t)sid + 8] = na;
  }
  // (c) each member of A enters at its best in-edge from a node outside A (or from a
  //     member already entered: any finite value is a path length, the rounds improve it)
  uint32_t* const ac = &ctl[r % 3u];
  if (tid == 0) ctl[(r + 1u) % 3u] = 0;
  for (uint32_t i = tid; i < na; i += BLOCK) {
    const uint32_t v = alist[i];
    D best = INF;
    const uint2 rr = g.row2[v];
    for (uint32_t e = rr.x; e < rr.y; ++e) {
      const uint4 rec = g.erec[e];
      if ((rec.x & kEdgeDown) || test_bit(ign, rec.z)) continue;
      const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
      if (u != src && (rec.x & kNodeSink)) continue;  // an overloaded tail does not expand
      const D du = dist[u];
      if (du == INF) continue;
      const D c = du + (D)rec.y;
      best = c < best ? c : best;
    }
    if (best != INF) {
      atomicMin(&dist[v], best);
      atomicOr(&inq[v >> 5], 1u << (v & 31u));
      cur[atomicAdd(ac, 1u)] = (uint16_t)v;
    }
  }
  sync();
  n = __builtin_amdgcn_readfirstlane(*ac);
  ++r;
  if (a.prof_solve && tid == 0) a.prof_solve[10 * (size_t)sid + 3] = wall_clock64();
  na_out = na;
  return n;
}

// BLOCK threads per solve: 64 (one wavefront, LDS ordering alone between rounds) or a
// multi-wave workgroup for batches that fill under a quarter of the CUs' wave slots (the
// 1 000-source WAN base SPF of the what-if sweep: ~4 solves per CU). Every round loop
// strides the frontier / the node range by BLOCK and ends at a workgroup barrier. The
// append counter of round r is ctl[r % 3]; round r zeroes ctl[(r + 1) % 3], whose last
// reads (round r - 2's count) all precede round r - 1's barrier.
template <int MODE, typename D, bool GENERIC, uint32_t BLOCK>
__global__ __launch_bounds__(BLOCK) void rounds_kernel(DevGraph g, SolveArgs a, uint32_t has_ign_rt, uint32_t* ctr) {
  using N = Nh<MODE>;
  constexpr D INF = (D)~(D)0;
  constexpr int K = 4;
  const bool has_ign = GENERIC && has_ign_rt != 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V, tid = threadIdx.x;
  const uint32_t nh_words = N::words(V);
  const RoundsLayout lay = rounds_layout(V, g.L, has_ign, nh_words, sizeof(D));
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;  // [0..2] rotating append counters, [3] next solve
  D* dist = reinterpret_cast<D*>(base + lay.dist);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint16_t* cnt = reinterpret_cast<uint16_t*>(base + lay.cnt);
  uint16_t* fa = reinterpret_cast<uint16_t*>(base + lay.fa);
  uint16_t* fb = reinterpret_cast<uint16_t*>(base + lay.fb);
  uint32_t* inq = reinterpret_cast<uint32_t*>(base + lay.inq);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  const uint32_t vw = (V + 31u) / 32u, ign_words = (g.L + 31u) / 32u;
  const uint32_t tight_words = (g.E + 63u) / 64u;
  auto sync = [&]() {
    if constexpr (BLOCK == kWave) lds_fence();
    else __syncthreads();
  };
  uint32_t r = 0;  // round number (append counter rotation)
  uint32_t n_sol = a.n;
  if (GENERIC && a.n_dev) n_sol = min(n_sol, __builtin_amdgcn_readfirstlane(*a.n_dev));

  for (uint32_t sid = blockIdx.x; sid < n_sol;) {
    const uint32_t src = a.sources[sid];
    const unsigned long long t_start = (GENERIC && a.prof_solve) ? wall_clock64() : 0ull;
    const uint32_t r_start = r;
    uint32_t r_dist = 0, r_kahn = 0;
    if (src < V) {
      for (uint32_t v = tid; v < V; v += BLOCK) dist[v] = INF;
      for (uint32_t i = tid; i < nh_words; i += BLOCK) nh[i] = 0;
      for (uint32_t i = tid; i < vw; i += BLOCK) inq[i] = 0;
      if (tid < 3) ctl[tid] = 0;
      if (has_ign) {
        for (uint32_t i = tid; i < ign_words; i += BLOCK) ign[i] = 0;
        sync();
        load_ignore(ign, ign_words, a, sid, g.L);
      }
      uint64_t* trow = (GENERIC && a.tight) ? a.tight + out_row_of(a, sid) * tight_words : nullptr;
      sync();
      uint16_t *cur = fa, *nxt = fb;
      uint32_t n = 1, na = 0;
      if (GENERIC && a.seed_dist) {
        n = seed_from_base<D, BLOCK>(g, a, sid, src, dist, cnt, cur, nxt, inq, ign,
                                     reinterpret_cast<uint16_t*>(base + lay.alist), ctl, r, tid, tight_words, na);
      } else {
        if (tid == 0) {
          dist[src] = 0;
          fa[0] = (uint16_t)src;
        }
        sync();
      }

      // (1) distance rounds over the frontier of nodes whose distance dropped
      while (n) {
        uint32_t* const ac = &ctl[r % 3u];
        if (tid == 0) ctl[(r + 1u) % 3u] = 0;
        for (uint32_t i = tid; i < n; i += BLOCK) {
          const uint32_t u = cur[i];
          atomicAnd(&inq[u >> 5], ~(1u << (u & 31u)));  // may re-enter the next frontier
          // the clear is issued before dist[u] is read (LDS operations of a wave complete in
          // order): an improvement another wave makes after the read finds the bit clear and
          // re-lists u
          asm volatile("" ::: "memory");
          if (u != src && g.ovl[u]) continue;  // reached, never expanded
          const D du = dist[u];
          const uint2 rr = g.row2[u];
          for (uint32_t e0 = rr.x; e0 < rr.y; e0 += K) {
            uint32_t av[K], wo[K], lv[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j;
              av[j] = e < rr.y ? g.adj[e] : kEdgeDown;
              wo[j] = e < rr.y ? g.w[e] : 0u;
              lv[j] = (has_ign && e < rr.y) ? g.lid[e] : 0u;
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
              if ((av[j] & kEdgeDown) || (has_ign && test_bit(ign, lv[j]))) continue;
              const uint32_t v = av[j];
              const D cand = du + (D)wo[j];
              if (cand < dist[v]) {
                const D old = atomicMin(&dist[v], cand);
                if (cand < old) {
                  const uint32_t bit = 1u << (v & 31u);
                  if (!(atomicOr(&inq[v >> 5], bit) & bit)) nxt[atomicAdd(ac, 1u)] = (uint16_t)v;
                }
              }
            }
          }
        }
        sync();
        n = __builtin_amdgcn_readfirstlane(*ac);
        ++r;
        uint16_t* t = cur;
        cur = nxt;
        nxt = t;
      }

      r_dist = r;
      if (GENERIC && a.prof_solve && tid == 0) a.prof_solve[10 * (size_t)sid + 4] = wall_clock64();
      // (2) tight in-degree of every reached node; the source (and nodes with no tight
      //     in-edge) start the topological rounds. After a seeded start only A's members
      //     are counted: a node outside A keeps its distance and gains no tight in-edge
      //     (every A member's distance grew), so its count is the base count less the
      //     in-edges the seed took away (the ignored links', A members')
      auto tight_in = [&](uint32_t v) -> uint32_t {
        const D dv = dist[v];
        uint32_t c = 0;
        if (dv != INF && v != src) {
          const uint2 rr = g.row2[v];
          for (uint32_t e0 = rr.x; e0 < rr.y; e0 += K) {
            uint4 rec[K];  // v->u: {u | down | sink(u), w(u->v), link, rev}
#pragma unroll
            for (int j = 0; j < K; ++j) rec[j] = e0 + j < rr.y ? g.erec[e0 + j] : make_uint4(kEdgeDown, 0u, 0u, 0u);
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t u = rec[j].x & ~(kEdgeDown | kNodeSink);
              if ((rec[j].x & kEdgeDown) || (has_ign && test_bit(ign, rec[j].z))) continue;
              if (u != src && (rec[j].x & kNodeSink)) continue;
              const D du = dist[u];
              c += (du != INF && (uint64_t)du + rec[j].y == (uint64_t)dv) ? 1u : 0u;
            }
          }
        }
        return c;
      };
      uint32_t* const ac2 = &ctl[r % 3u];
      if (tid == 0) ctl[(r + 1u) % 3u] = 0;
      if (GENERIC && a.seed_dist) {
        const uint16_t* al = reinterpret_cast<const uint16_t*>(base + lay.alist);
        for (uint32_t i = tid; i < na; i += BLOCK) {
          const uint32_t v = al[i];
          cnt[v] = (uint16_t)tight_in(v);
        }
        if (tid == 0) cur[atomicAdd(ac2, 1u)] = (uint16_t)src;
        sync();
      } else {
        for (uint32_t v = tid; v < V; v += BLOCK) {
          cnt[v] = (uint16_t)tight_in(v);
          if (v == src) cur[atomicAdd(ac2, 1u)] = (uint16_t)v;
        }
        sync();
        if (GENERIC && a.tin_out) {  // the base SPF of a what-if sweep: counts for seeded starts
          uint16_t* trow_in = a.tin_out + out_row_of(a, sid) * V;
          for (uint32_t v = tid; v < V; v += BLOCK) trow_in[v] = cnt[v];
        }
      }
      n = __builtin_amdgcn_readfirstlane(*ac2);
      ++r;
      if (GENERIC && a.prof_solve && tid == 0) a.prof_solve[10 * (size_t)sid + 5] = wall_clock64();

      // (3) Kahn rounds: a finished node pushes its set down its tight out-edges; the
      //     decrement that empties a successor's count makes it finished next round
      while (n) {
        uint32_t* const ac = &ctl[r % 3u];
        if (tid == 0) ctl[(r + 1u) % 3u] = 0;
        for (uint32_t i = tid; i < n; i += BLOCK) {
          const uint32_t u = cur[i];
          if (u != src && g.ovl[u]) continue;  // a sink has no tight out-edges
          const D du = dist[u];
          const typename N::Val xu = N::load(nh, u);
          const uint2 rr = g.row2[u];
          for (uint32_t e0 = rr.x; e0 < rr.y; e0 += K) {
            uint32_t av[K], wo[K], lv[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j;
              av[j] = e < rr.y ? g.adj[e] : kEdgeDown;
              wo[j] = e < rr.y ? g.w[e] : 0u;
              lv[j] = (has_ign && e < rr.y) ? g.lid[e] : 0u;
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
              if ((av[j] & kEdgeDown) || (has_ign && test_bit(ign, lv[j]))) continue;
              const uint32_t v = av[j], e = e0 + j;
              const D dv = dist[v];
              if (dv == INF || (uint64_t)du + wo[j] != (uint64_t)dv) continue;  // not tight
              if (u == src) N::or_bit(nh, v, g.nbr[e]);
              else N::or_val(nh, v, xu);
              if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[e >> 6]), 1ull << (e & 63u));
              const uint32_t sh = 16u * (v & 1u);
              const uint32_t old = atomicSub(reinterpret_cast<uint32_t*>(cnt) + (v >> 1), 1u << sh);
              if (((old >> sh) & 0xFFFFu) == 1u) nxt[atomicAdd(ac, 1u)] = (uint16_t)v;
            }
          }
        }
        sync();
        n = __builtin_amdgcn_readfirstlane(*ac);
        ++r;
        uint16_t* t = cur;
        cur = nxt;
        nxt = t;
      }
      r_kahn = r;
      if (GENERIC && a.prof_solve && tid == 0) a.prof_solve[10 * (size_t)sid + 6] = wall_clock64();
      if (GENERIC && a.seed_changed) {
        // what-if unit: the count of nodes whose distance or next-hop bytes differ from the
        // base rows, instead of the rows (no row round trip through HBM)
        const uint32_t unit = a.seed_unit[sid], j = unit % a.seed_nsrc, nb = a.nh_bytes;
        const uint64_t* bd = a.seed_dist + (size_t)j * V;
        const uint8_t* bh = a.seed_nh + (size_t)j * V * nb;
        auto differs = [&](uint32_t v) {
          const D dv = dist[v];
          bool diff = (dv == INF ? ~0ull : (uint64_t)dv) != bd[v];
          for (uint32_t b = 0; b < nb && !diff; ++b) diff = (uint8_t)N::byte(nh, v, b) != bh[(size_t)v * nb + b];
          return diff;
        };
        uint32_t c = 0;
        for (uint32_t v = tid; v < V; v += BLOCK) c += differs(v) ? 1u : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if ((tid & 63u) == 0 && c) atomicAdd(&a.seed_changed[unit], c);  // zeroed by the seeded start
        if (a.delta.node) {
          // the unit's delta (WhatifDelta): one pool reservation for the workgroup, then each
          // wave writes its differing nodes in order. The frontier queues are free now.
          constexpr uint32_t W = BLOCK / 64u;
          const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
          uint32_t* sc = reinterpret_cast<uint32_t*>(base + lay.fa);  // >= 8 words (fa, fb)
          if (lane == 0) sc[wave] = c;
          sync();
          if (tid == 0) {
            uint32_t total = 0;
            for (uint32_t w = 0; w < W; ++w) total += sc[w];
            const unsigned long long b = total ? atomicAdd(a.delta.used, (unsigned long long)total) : 0ull;
            sc[4] = (uint32_t)b;
            sc[5] = (uint32_t)(b >> 32);
            if (total) a.delta.off[unit] = a.delta.base_of(b);
          }
          sync();
          unsigned long long cur = (unsigned long long)sc[4] | ((unsigned long long)sc[5] << 32);
          for (uint32_t w = 0; w < wave; ++w) cur += sc[w];
          for (uint32_t v0 = wave * 64u; v0 < V; v0 += BLOCK) {
            const uint32_t v = v0 + lane;
            const bool diff = v < V && differs(v);
            const unsigned long long m = __ballot(diff);
            const unsigned long long pos =
                cur + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (diff && pos < a.delta.cap) {
              a.delta.node[pos] = v;
              const D dv = dist[v];
              a.delta.dist[pos] = dv == INF ? ~0ull : (unsigned long long)dv;
              uint8_t* o = a.delta.nh + (size_t)pos * a.delta.nhb;
              for (uint32_t b = 0; b < a.delta.nhb; ++b) o[b] = b < nb ? (uint8_t)N::byte(nh, v, b) : 0u;
            }
            cur += (uint32_t)__popcll(m);
          }
        }
        goto next_solve;
      }
      {
      // (result rows, coalesced; unreached nodes keep UINT64_MAX)
      uint64_t* drow = a.dist + out_row_of(a, sid) * V;
      for (uint32_t v = tid; v < V; v += BLOCK) {
        const D d = dist[v];
        store_row<uint64_t>(&drow[v], d == INF ? ~0ull : (uint64_t)d, true);
      }
      if (a.nh) {
        const uint32_t nb = a.nh_bytes;
        uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
        for (uint32_t i = tid; i < V * nb; i += BLOCK) {
          const uint32_t v = i / nb, j = i - v * nb;
          nrow[i] = (uint8_t)N::byte(nh, v, j);
        }
      }
      }
    }
  next_solve:
    if (GENERIC && a.prof_solve && tid == 0) {
      a.prof_solve[10 * (size_t)sid] = t_start;
      a.prof_solve[10 * (size_t)sid + 7] = wall_clock64();
      a.prof_solve[10 * (size_t)sid + 9] = (unsigned long long)(r_dist - r_start) | ((unsigned long long)(r_kahn - r_dist) << 32);
    }
    if constexpr (BLOCK == kWave) {
      uint32_t nxt_sid = 0;
      if (tid == 0) nxt_sid = gridDim.x + atomicAdd(&ctr[0], 1u);
      sid = __builtin_amdgcn_readfirstlane(__shfl(nxt_sid, 0));
    } else {
      // every thread is past this solve's write-out before the next one's init
      if (tid == 0) ctl[3] = gridDim.x + atomicAdd(&ctr[0], 1u);
      __syncthreads();
      sid = __builtin_amdgcn_readfirstlane(ctl[3]);
      __syncthreads();  // ctl[3] read by every wave before a later solve rewrites it
    }
  }
  retire_workgroup(ctr, nullptr);
}

template <int MODE, typename D, uint32_t BLOCK>
hipError_t launch_rounds_b(const DevGraph& g, const SolveArgs& a, uint32_t lds, uint32_t grid, uint32_t* ctr,
                           hipStream_t s) {
  const bool has_ign = a.ign_ptr != nullptr;
  const bool generic = has_ign || a.tight != nullptr;
  auto k = generic ? rounds_kernel<MODE, D, true, BLOCK> : rounds_kernel<MODE, D, false, BLOCK>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  note_launch("rounds_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), lds, s, g, a, (uint32_t)has_ign, ctr);
  return hipGetLastError();
}

template <int MODE, typename D>
hipError_t launch_rounds_t(const DevGraph& g, const SolveArgs& a, uint32_t lds, uint32_t block, int num_cus,
                           uint32_t* ctr, hipStream_t s) {
  const uint32_t grid = blocks_for(a.n, lds, num_cus, block);
  switch (block) {
    case 256u: return launch_rounds_b<MODE, D, 256u>(g, a, lds, grid, ctr, s);
    case 128u: return launch_rounds_b<MODE, D, 128u>(g, a, lds, grid, ctr, s);
    default: return launch_rounds_b<MODE, D, kWave>(g, a, lds, grid, ctr, s);
  }
}

}  // namespace

uint32_t rounds_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64) {
  if (V > 65535u) return 0;
  const uint32_t t = rounds_layout(V, L, has_ignore, nh_words_for(nh_mode, V), dist64 ? 8u : 4u).total;
  return t <= kMaxLds ? t : 0;
}

// Threads per solve: 256 for batches of up to four rounds of 256-thread workgroups per CU,
// one wavefront per solve (no barriers) beyond. Measured on the WAN what-if: the base SPF
// (1 000 sources) 0.41 -> 0.21 ms, the 6 533 re-solved large units 64 / 128 / 256 threads:
// step 5.33 / 5.25 / 5.18 ms (a solve's rounds are latency chains: four waves cut each
// round's serial passes even when the CUs are full). OPENR_SPF_ROUNDS_BLOCK=64|128|256
// forces one (tests, A/B).
uint32_t rounds_block(uint32_t n, uint32_t lds, int num_cus) {
  const uint32_t knob = env_u32("OPENR_SPF_ROUNDS_BLOCK", 0u, 64u, 256u);
  if (knob == 64u || knob == 128u || knob == 256u) return knob;
  const uint64_t per_cu = ((uint64_t)n + (uint64_t)std::max(num_cus, 1) - 1u) / (uint64_t)std::max(num_cus, 1);
  const uint64_t by_lds = lds ? kMaxLds / lds : 32u;
  return per_cu <= 4u * std::min<uint64_t>(by_lds, 2048u / 256u) ? 256u : kWave;
}

hipError_t launch_rounds(const DevGraph& g, const SolveArgs& a, bool dist64, int nh_mode, int num_cus, hipStream_t s,
                         LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  const uint32_t lds = rounds_lds_bytes(g.V, g.L, has_ign, nh_mode, dist64);
  if (!lds || !a.work) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  uint32_t block = rounds_block(a.n, lds, num_cus);
  if (a.n_dev && !std::getenv("OPENR_SPF_ROUNDS_BLOCK") && (a.n_block == 64u || a.n_block == 128u || a.n_block == 256u))
    block = a.n_block;
  if (info) {
    info->lds_bytes = lds;
    info->grid = blocks_for(a.n, lds, num_cus, block);
    info->kernel = dist64 ? "rounds_kernel<u64>" : "rounds_kernel<u32>";
  }
  uint32_t* ctr = a.work + kFringeCtr;
#define OPENR_ROUNDS_CASE(M) \
  case M: return dist64 ? launch_rounds_t<M, unsigned long long>(g, a, lds, block, num_cus, ctr, s) \
                        : launch_rounds_t<M, uint32_t>(g, a, lds, block, num_cus, ctr, s);
  switch (nh_mode) {
    OPENR_ROUNDS_CASE(kNhNibble)
    OPENR_ROUNDS_CASE(kNhByte)
    OPENR_ROUNDS_CASE(kNhHalf)
    OPENR_ROUNDS_CASE(kNhW1)
    OPENR_ROUNDS_CASE(kNhW2)
    OPENR_ROUNDS_CASE(kNhW4)
    OPENR_ROUNDS_CASE(kNhW8)
  }
#undef OPENR_ROUNDS_CASE
  return hipErrorInvalidValue;
}

}  // namespace openr_spf
