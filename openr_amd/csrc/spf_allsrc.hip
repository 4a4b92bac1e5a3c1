// spf_allsrc.hip — all-sources batches on uniform-cost graphs: levels first, next hops
// from the level rows of the sources' neighbours (round 3; BASELINE configs 2 and 3).
//
// Two level passes feed the same next-hop pass:
//  * msbfs_kernel (default when a batch holds >= V sources and V <= 10 240): bit-parallel
//    multi-source BFS. A 512-thread workgroup solves 32 sources at once: every node holds a
//    32-bit word (bit j = source j) of the current frontier in LDS, each thread owns 20 nodes
//    and keeps their visited word and their levels (as 8 bit-planes) in registers, and a
//    level is one dense pull over every node: new = (OR of the neighbours' frontier words)
//    & ~visited. No queue, no atomics, no per-source LDS state: the cost of a level is
//    V node reads shared by 32 sources instead of a dependent chain per source.
//  * bfs_reach_kernel: per-source BFS with u8 levels and a visited bitmap (no next-hop
//    state), for batches that still hold every neighbour but do not fit msbfs.
// Both write u8 level rows; nh_from_levels_kernel then derives every next-hop set from
// them (derivation below) and, optionally, the u64 distance rows.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;
using namespace bfs;

// ---------------------------------------------------------------------------
// Reach pass + next hops from neighbour level rows (round 3: all-sources batches on
// ELL-only graphs, the G100 path).
//
// For uniform cost the closed form of LinkState::runSpf (LinkState.cpp:808-882) has a
// second reading. Let n_i be the i-th distinct neighbour of s (next-hop bit i). For a node
// v at level l = lvl_s(v) >= 1:
//     bit i of nh_s(v)  <=>  some usable edge s-n_i exists and
//                            (v == n_i and l == 1)  or  (n_i not overloaded and lvl_{n_i}(v) + 1 == l)
// Proof sketch: nh_s(v) is the set of second nodes of shortest s-v paths whose inner nodes
// all expand (LinkState.cpp:831-838, 867-872). Usable edges are symmetric (Link::isUp is
// per link) and cost the same, so for a non-overloaded n_i every n_i-v path extends to an
// s-v path one hop longer whose inner nodes expand in s's solve exactly when they expand in
// n_i's (both treat every overloaded node but their own source as a sink): lvl_s(v) <=
// lvl_{n_i}(v) + 1, with equality iff a shortest s-v path runs through n_i. Such a path
// never returns to s, so s being a sink in n_i's solve changes nothing. An overloaded
// n_i is a sink in s's solve: it is the next hop of itself only.
//
// So when a batch holds every source's usable, non-overloaded neighbours (an all-sources
// batch does), the BFS itself needs no next-hop state, and each solve drops to a u8 level
// per node plus a visited bitmap (12.6 vs 16.3 KB of LDS on G100: 12 instead of 10 solves
// per CU). Per edge slot: one ds_or_rtn on the visited bitmap elects the first arrival (no
// level read before it, no next-hop read / merge). Phase 2 (nh_from_levels_kernel) is a
// streaming pass: per source, its level row against its neighbours' rows, four nodes per
// dword with SWAR byte compares. A solve deeper than 253 levels or wider than a queue half,
// and a source whose neighbour row is missing or invalid, is listed for the u16
// full-order re-run of bfs_lvl_kernel, which computes dist and next hops itself.
// ---------------------------------------------------------------------------
struct ReachLayout {
  uint32_t vis, ring, total;
};
// [0, 32) control, [32, 32 + V + 4) u8 levels, visited bits (ids >= V pre-set: padding V and
// the sentinels V + 32k), two queue halves
__host__ __device__ inline uint32_t reach_vis_words(uint32_t V) {
  return (V + kReachSentinelStride * (kReachSentinels - 1u) + 1u + 31u) / 32u;
}
__host__ __device__ inline ReachLayout reach_layout(uint32_t V, uint32_t ring_cap) {
  ReachLayout l;
  uint32_t off = 32u + ((V + 4u + 15u) & ~15u);
  l.vis = off;
  off += (4u * reach_vis_words(V) + 15u) & ~15u;
  l.ring = off;
  off += (2u * ring_cap + 15u) & ~15u;
  l.total = off;
  return l;
}

// flags: bit 0 non-temporal stores, bit 1 leave the distance row to phase 2
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void bfs_reach_kernel(
    DevGraph g, SolveArgs a, uint64_t cost, uint32_t half, uint32_t ring_alloc, uint32_t* ctr, uint32_t* ovf_count,
    uint32_t flags) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const ReachLayout lay = reach_layout(V, ring_alloc);  // >= half + BLOCK entries
  lds_u32* const ctl = (lds_u32*)(size_t)0u;  // [0..3] append counters, [7] next unit
  lds_u8* const lvl = (lds_u8*)(size_t)32u;
  lds_u32* const lvl_w = (lds_u32*)(size_t)32u;
  lds_u32* const vis = (lds_u32*)(size_t)lay.vis;
  lds_u16* const ring = (lds_u16*)(size_t)lay.ring;
  const uint8_t* lvl_g = reinterpret_cast<const uint8_t*>(reinterpret_cast<char*>(smem) + 32);
  const uint32_t lvl_words = (V + 3u) / 4u, vis_words = reach_vis_words(V), vfull = V / 32u;
  const uint32_t rb = reach_row_bytes(V);
  const bool nt = (flags & 1u) != 0, dist_here = (flags & 2u) == 0;
  const uint32_t sent = V + kReachSentinelStride * lane;  // this lane's sentinel row / visited bit
  for (uint32_t unit = blockIdx.x; unit < a.n;) {
    const uint32_t src = a.sources[unit];
    bool ok = false;
    if (src < V) {  // block-uniform
      for (uint32_t i = tid; i < lvl_words; i += BLOCK) lvl_w[i] = 0xFFFFFFFFu;
      for (uint32_t i = tid; i < vis_words; i += BLOCK)
        vis[i] = i < vfull ? 0u : i > vfull ? 0xFFFFFFFFu : ~((1u << (V & 31u)) - 1u);  // every id >= V visited
      if (tid < 5) ctl[tid] = 0;
      __syncthreads();
      if (tid == 0) {
        lvl[src] = 0;
        vis[src >> 5] |= 1u << (src & 31u);
      }
      __syncthreads();
      // level 0: the source expands its full CSR row even when overloaded (LinkState.cpp:831-838)
      {
        const uint2 rs = g.row2[src];
        for (uint32_t e0 = rs.x; e0 < rs.y; e0 += BLOCK) {
          const uint32_t e = e0 + tid;
          bool fresh = false;
          uint32_t v = 0;
          if (e < rs.y) {
            const uint32_t av = g.adj[e];
            v = av & ~kEdgeDown;
            if (!(av & kEdgeDown) && v != src) {
              const uint32_t bit = 1u << (v & 31u);
              fresh = (lds_or(&vis[v >> 5], bit) & bit) == 0u;
              if (fresh) lvl[v] = 1;
            }
          }
          const uint32_t slot = wave_append(fresh, reinterpret_cast<uint32_t*>(smem) + 1);
          if (fresh) ring[half + slot] = (uint16_t)v;  // slot < deg(src) <= half (host-checked)
        }
      }
      __syncthreads();

      uint32_t cur = __builtin_amdgcn_readfirstlane(ctl[1]), L = 1, reached = 1u + cur;
      bool overflow = false;  // block-uniform
      constexpr uint32_t K = 4u, NPP = 64u, NPB = (uint32_t)BLOCK;
      uint32_t q = ring[half + wave * NPP + lane];  // first pass's queue entry of level 1
      while (cur) {
        if (L + 1u >= 0xFFu) {  // next level not representable in u8
          overflow = true;
          break;
        }
        lds_u32* const cnt = &ctl[(L + 1u) & 3u];
        if (tid == 0) ctl[(L + 2u) & 3u] = 0;  // last read three barriers ago
        const uint32_t rd = (L & 1u) * half, wr = half - rd;
        const uint8_t lnext = (uint8_t)(L + 1u);
        for (uint32_t fb = wave * NPP; fb < cur; fb += NPB) {
          const uint32_t idx = fb + lane;
          if (fb != wave * NPP) q = ring[rd + idx];
          const uint32_t u = idx < cur ? q : sent;  // past the level: this lane's sentinel row
          const uint4 ell = g.ellv[u];              // down / padding / sink-row slots hold V
          const uint32_t vv[K] = {ell.x, ell.y, ell.z, ell.w};
          uint32_t old[K];
#pragma unroll
          for (uint32_t j = 0; j < K; ++j) old[j] = lds_or(&vis[vv[j] >> 5], 1u << (vv[j] & 31u));
          __builtin_amdgcn_sched_barrier(0);  // all atomics in flight before their results are used
          unsigned long long bj[K];
          bool fresh[K];
          uint32_t off[K + 1];
          off[0] = 0;
#pragma unroll
          for (uint32_t j = 0; j < K; ++j) {
            fresh[j] = __builtin_amdgcn_ubfe(old[j], vv[j] & 31u, 1u) == 0u;  // first arrival
            bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
            off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
          }
          const uint32_t total = off[K];
          if (total) {  // wave-uniform
            const uint32_t leader = (uint32_t)__builtin_amdgcn_readfirstlane(lane);
            uint32_t wbase = 0;
            if (lane == leader) wbase = lds_add(cnt, total);
            const uint32_t bse = __builtin_amdgcn_readfirstlane(wbase);
            if (bse + total <= half) {  // wave-uniform: the level fits its half so far
#pragma unroll
              for (uint32_t j = 0; j < K; ++j) {
                if (fresh[j]) {
                  const uint32_t slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                  ring[wr + bse + off[j] + slot] = (uint16_t)vv[j];
                  lvl[vv[j]] = lnext;
                }
              }
            } else if (lane == leader) {
              lds_or(cnt, 0x80000000u);  // the level outgrows its half
            }
          }
        }
        lds_barrier();
        const uint32_t c = __builtin_amdgcn_readfirstlane(*cnt);
        q = ring[wr + wave * NPP + lane];
        ++L;
        if (c >> 31) {  // uniform after the barrier
          overflow = true;
          break;
        }
        cur = c;
        reached += cur;
        if (reached == V) break;  // every node reached: the newest level reaches nothing new
      }
      if (overflow) {
        if (tid == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = unit;
      } else {
        ok = true;
        // the u8 level row (phase 2 input), dword stores
        uint32_t* lrow = reinterpret_cast<uint32_t*>(a.lvl8 + (size_t)unit * rb);
        for (uint32_t i = tid; i < rb / 4u; i += BLOCK) lrow[i] = lvl_w[i];
        if (dist_here) {
          uint64_t* drow = a.dist + (size_t)unit * V;
          if (((reinterpret_cast<uintptr_t>(drow) & 15u) | (V & 1u)) == 0) {
            ulonglong2* d2 = reinterpret_cast<ulonglong2*>(drow);
            for (uint32_t i = tid; i < V / 2u; i += BLOCK) {
              const uint32_t l0 = lvl_g[2u * i], l1 = lvl_g[2u * i + 1u];
              const uint64_t x0 = l0 != 0xFFu ? (uint64_t)l0 * cost : ~0ull;
              const uint64_t x1 = l1 != 0xFFu ? (uint64_t)l1 * cost : ~0ull;
              if (nt) {
                __builtin_nontemporal_store(x0, &d2[i].x);
                __builtin_nontemporal_store(x1, &d2[i].y);
              } else {
                d2[i] = make_ulonglong2(x0, x1);
              }
            }
          } else {
            for (uint32_t v = tid; v < V; v += BLOCK) {
              const uint32_t l = lvl_g[v];
              store_row<uint64_t>(&drow[v], l != 0xFFu ? (uint64_t)l * cost : ~0ull, nt);
            }
          }
        }
      }
    }
    if (tid == 0) a.rowok[unit] = ok ? 1u : 0u;
    __syncthreads();  // every lane is done with this unit's LDS and ctl[7]
    if (tid == 0) ctl[7] = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = ctl[7];
  }
  retire_workgroup(ctr, nullptr);
}

// rowmap[v] = UINT32_MAX for every node, then rowmap[sources[k]] = k (a later duplicate wins:
// its row holds the same results)
__global__ void reach_map_clear_kernel(uint32_t* rowmap, uint32_t V) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) rowmap[i] = ~0u;
}
__global__ void reach_map_fill_kernel(uint32_t* rowmap, const uint32_t* sources, uint32_t n, uint32_t V) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
    if (sources[k] < V) rowmap[sources[k]] = k;
}

// Batch order of the multi-source BFS: when the call's sources are every node exactly once
// (rowmap[sources[k]] == k for all k and n == V), position i takes the row of the i-th node
// of the cluster order (DevGraph::corder), else row i.
__global__ void ms_perm_count_kernel(const uint32_t* sources, uint32_t n, const uint32_t* rowmap, uint32_t V,
                                     uint32_t* cnt) {
  uint32_t c = 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
    c += (sources[k] < V && rowmap[sources[k]] == k) ? 1u : 0u;
  c = __reduce_add_sync(~0ull, c);
  if (__lane_id() == 0 && c) atomicAdd(cnt, c);
}
__global__ void ms_perm_fill_kernel(const uint32_t* corder, const uint32_t* rowmap, uint32_t n, uint32_t V,
                                    const uint32_t* cnt, uint32_t* perm) {
  const bool perm_all = corder && n == V && *cnt == n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    perm[i] = perm_all ? rowmap[corder[i]] : i;
}

// ---------------------------------------------------------------------------
// Extended batch of a partial all-sources call (tile-active multi-source pass, round 3:
// strong-scaling shards, LFA prefetches). The next-hop derivation needs the level rows of
// every usable, non-overloaded neighbour of a source; a batch that lacks some gets them as
// halo rows (levels only), appended after the call's rows: xsrc = [sources | halo]. The
// batch sequence follows the cluster order restricted to the extended batch (xslot[crank of
// a source] = its row; duplicates and invalid sources go last), so 32-source batches stay
// compact. Results do not depend on the order.
// ---------------------------------------------------------------------------
constexpr uint32_t kExtPending = 0xFFFFFFFEu;
__global__ void ms_ext_clear_kernel(uint32_t* rowmap, uint32_t* slot, uint32_t V, uint32_t* xcount) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < V; i += gridDim.x * blockDim.x) {
    rowmap[i] = ~0u;
    slot[i] = ~0u;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) xcount[threadIdx.x] = 0;  // [0] halo rows, [1] tail rows
}
__global__ void ms_ext_fill_kernel(const uint32_t* sources, uint32_t n, uint32_t V, const uint32_t* crank,
                                   uint32_t* rowmap, uint32_t* slot, uint32_t* xsrc, uint32_t* xdup, uint32_t* xcount) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t s = sources[k];
    xsrc[k] = s;
    if (s < V) rowmap[s] = k;  // a duplicate's row holds the same results: any one serves
    if (s >= V || atomicCAS(&slot[crank[s]], ~0u, k) != ~0u) xdup[atomicAdd(&xcount[1], 1u)] = k;
  }
}
__global__ void ms_ext_halo_kernel(DevGraph g, const uint32_t* sources, uint32_t n, uint32_t* rowmap,
                                   uint32_t* slot, uint32_t* xsrc, uint32_t* xcount) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t s = sources[k];
    if (s >= g.V) continue;
    const uint2 r = g.row2[s];
    for (uint32_t e = r.x; e < r.y; ++e) {
      const uint32_t av = g.adj[e];
      if (av & kEdgeDown) continue;
      const uint32_t x = av;
      if (x == s || g.ovl[x]) continue;  // an overloaded neighbour is a next hop by id, no row
      if (atomicCAS(&rowmap[x], ~0u, kExtPending) != ~0u) continue;  // has a row, or another thread adds it
      const uint32_t row = n + atomicAdd(&xcount[0], 1u);
      xsrc[row] = x;
      rowmap[x] = row;
      slot[g.crank[x]] = row;  // x is no call source: its slot is free
    }
  }
}
// one workgroup: msperm = the occupied slots in cluster order, then the tail rows
__global__ __launch_bounds__(1024) void ms_ext_order_kernel(const uint32_t* slot, uint32_t V, const uint32_t* xdup,
                                                            const uint32_t* xcount, uint32_t* perm) {
  __shared__ uint32_t cnt[1024];
  const uint32_t tid = threadIdx.x, per = (V + 1023u) / 1024u;
  const uint32_t lo = min(V, tid * per), hi = min(V, lo + per);
  uint32_t c = 0;
  for (uint32_t i = lo; i < hi; ++i) c += slot[i] != ~0u ? 1u : 0u;
  cnt[tid] = c;
  __syncthreads();
  for (uint32_t d = 1; d < 1024u; d <<= 1) {  // inclusive scan
    const uint32_t x = tid >= d ? cnt[tid - d] : 0u;
    __syncthreads();
    cnt[tid] += x;
    __syncthreads();
  }
  uint32_t o = cnt[tid] - c;
  for (uint32_t i = lo; i < hi; ++i)
    if (slot[i] != ~0u) perm[o++] = slot[i];
  const uint32_t placed = cnt[1023], tail = xcount[1];
  for (uint32_t j = tid; j < tail; j += 1024u) perm[placed + j] = xdup[j];
}

// Four u8 levels per dword: bytes b of `ln` with ln_b + 1 == ls_b (mod 256) -> bit 7 of byte b
__device__ __forceinline__ uint32_t swar_succ_eq(uint32_t ln, uint32_t ls) {
  const uint32_t inc = ((ln & 0x7F7F7F7Fu) + 0x01010101u) ^ (ln & 0x80808080u);  // per-byte +1, no carries
  const uint32_t x = inc ^ ls;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // bit 7 of each zero byte
}
__device__ __forceinline__ uint32_t swar_zero_hi(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}


// ---------------------------------------------------------------------------
// Next hops from level rows. One wavefront per batch row; each lane takes 16 nodes (one
// 16-byte load of levels per row) per step. Rows are dealt to XCDs in contiguous ranges
// (workgroup i runs on XCD i % 8), so the rows of a source's neighbours, which are mostly
// near it in batch order, are read from the same XCD's L2. flags: bit 0 non-temporal
// stores, bit 1 also write the distance row. Next-hop sets of <= 8 bits (one byte per
// node; bytes past the first of a wider caller stride are zero); a source with a missing
// or invalid neighbour row, a wider set or a row of more than 64 edges is listed for the
// u16 full-order re-run.
// ---------------------------------------------------------------------------
constexpr uint32_t kNhlWaves = 4;  // rows in flight per workgroup
__global__ __launch_bounds__(64 * kNhlWaves) void nh_from_levels_kernel(DevGraph g, SolveArgs a, uint64_t cost,
                                                                         uint32_t* ovf_count, uint32_t flags) {
  const uint32_t V = g.V, lane = __lane_id(), rb = reach_row_bytes(V), nb = a.nh_bytes;
  const bool nt = (flags & 1u) != 0, want_dist = (flags & 2u) != 0;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // this wave's share: XCD x (= blockIdx.x % 8) owns rows [x * n / 8, (x + 1) * n / 8)
  const uint32_t xcd = blockIdx.x % 8u, wgs_x = (gridDim.x + 7u - xcd) / 8u, wg_x = blockIdx.x / 8u;
  const uint32_t r0 = (uint32_t)((uint64_t)a.n * xcd / 8u), r1 = (uint32_t)((uint64_t)a.n * (xcd + 1u) / 8u);
  const uint32_t steps = rb / 16u;
  for (uint32_t k = r0 + wg_x * kNhlWaves + wave; k < r1; k += wgs_x * kNhlWaves) {
    const uint32_t src = a.sources[k];
    if (src >= V || !a.rowok[k]) continue;  // wave-uniform; a flagged row is re-run whole
    // the source's usable neighbours, one per lane: non-overloaded ones by level row,
    // overloaded ones (sinks: next hop of themselves only) by id
    const uint2 rs = g.row2[src];
    const uint32_t deg = rs.y - rs.x;
    bool use = false, sink = false, bad = deg > 64u;
    uint32_t nrow = 0, nbit = 0, nid = 0;
    if (lane < deg && !bad) {
      const uint32_t e = rs.x + lane;
      const uint32_t av = g.adj[e];
      nid = av & ~kEdgeDown;
      if (!(av & kEdgeDown) && nid != src) {
        nbit = g.nbr[e];
        if (g.ovl[nid]) {
          sink = true;
        } else {
          use = true;
          nrow = a.rowmap[nid];
          bad = nrow == ~0u || nbit >= 8u || !a.rowok[nrow];
        }
      }
    }
    if (__builtin_amdgcn_ballot_w64(bad || (sink && nbit >= 8u)) != 0ull) {
      if (lane == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = k;
      continue;
    }
    const unsigned long long um = __builtin_amdgcn_ballot_w64(use), sm = __builtin_amdgcn_ballot_w64(sink);
    const uint4* lrow = reinterpret_cast<const uint4*>(a.lvl8 + (size_t)k * rb);
    uint8_t* orow = a.nh ? a.nh + (size_t)k * V * nb : nullptr;
    uint64_t* drow = a.dist + (size_t)k * V;
    const bool fast_nh = orow && nb == 1u && (reinterpret_cast<uintptr_t>(orow) & 15u) == 0u;
    for (uint32_t w = lane; w < steps; w += 64u) {
      const uint4 ls = lrow[w];
      uint4 acc = make_uint4(0, 0, 0, 0);
      for (unsigned long long m = um; m; m &= m - 1ull) {
        const int j = __builtin_ctzll(m);
        const uint32_t r = __builtin_amdgcn_readlane(nrow, j), b = __builtin_amdgcn_readlane(nbit, j);
        const uint4 ln = reinterpret_cast<const uint4*>(a.lvl8 + (size_t)r * rb)[w];
        acc.x |= (swar_succ_eq(ln.x, ls.x) >> 7) << b;
        acc.y |= (swar_succ_eq(ln.y, ls.y) >> 7) << b;
        acc.z |= (swar_succ_eq(ln.z, ls.z) >> 7) << b;
        acc.w |= (swar_succ_eq(ln.w, ls.w) >> 7) << b;
      }
      // no next hops at the source (level 0) or an unreached node (0xFF)
      acc.x &= ((~(swar_zero_hi(ls.x) | swar_zero_hi(~ls.x)) & 0x80808080u) >> 7) * 0xFFu;
      acc.y &= ((~(swar_zero_hi(ls.y) | swar_zero_hi(~ls.y)) & 0x80808080u) >> 7) * 0xFFu;
      acc.z &= ((~(swar_zero_hi(ls.z) | swar_zero_hi(~ls.z)) & 0x80808080u) >> 7) * 0xFFu;
      acc.w &= ((~(swar_zero_hi(ls.w) | swar_zero_hi(~ls.w)) & 0x80808080u) >> 7) * 0xFFu;
      const uint32_t v0 = 16u * w;
      for (unsigned long long m = sm; m; m &= m - 1ull) {  // overloaded direct neighbours
        const int j = __builtin_ctzll(m);
        const uint32_t id = __builtin_amdgcn_readlane(nid, j), b = __builtin_amdgcn_readlane(nbit, j);
        if (id - v0 < 16u) {
          const uint32_t sh = 8u * (id & 3u), bitv = (1u << b) << sh;
          switch ((id - v0) >> 2) {
            case 0: acc.x |= bitv; break;
            case 1: acc.y |= bitv; break;
            case 2: acc.z |= bitv; break;
            default: acc.w |= bitv; break;
          }
        }
      }
      if (orow) {
        if (fast_nh && v0 + 16u <= V) {
          if (nt) {
            uint32_t* o = reinterpret_cast<uint32_t*>(orow + v0);
            __builtin_nontemporal_store(acc.x, o);
            __builtin_nontemporal_store(acc.y, o + 1);
            __builtin_nontemporal_store(acc.z, o + 2);
            __builtin_nontemporal_store(acc.w, o + 3);
          } else {
            *reinterpret_cast<uint4*>(orow + v0) = acc;
          }
        } else {
          const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
          for (uint32_t j = 0; j < 16u && v0 + j < V; ++j) {
            uint8_t* o = orow + (size_t)(v0 + j) * nb;
            o[0] = (uint8_t)(wv[j >> 2] >> (8u * (j & 3u)));
            for (uint32_t c = 1; c < nb; ++c) o[c] = 0;
          }
        }
      }
    }
    if (want_dist) {
      // distance row from the level row (just read: L2), four nodes per lane and step so a
      // wavefront's stores cover whole lines
      const uint32_t* lw = reinterpret_cast<const uint32_t*>(a.lvl8 + (size_t)k * rb);
      if (((reinterpret_cast<uintptr_t>(drow) & 15u) | (V & 3u)) == 0) {
        ulonglong2* d2 = reinterpret_cast<ulonglong2*>(drow);
        for (uint32_t i = lane; i < V / 4u; i += 64u) {
          const uint32_t w = lw[i];
          uint64_t xd[4];
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) {
            const uint32_t l = (w >> (8u * j)) & 0xFFu;
            xd[j] = l != 0xFFu ? (uint64_t)l * cost : ~0ull;
          }
          if (nt) {
            __builtin_nontemporal_store(xd[0], &d2[2u * i].x);
            __builtin_nontemporal_store(xd[1], &d2[2u * i].y);
            __builtin_nontemporal_store(xd[2], &d2[2u * i + 1u].x);
            __builtin_nontemporal_store(xd[3], &d2[2u * i + 1u].y);
          } else {
            d2[2u * i] = make_ulonglong2(xd[0], xd[1]);
            d2[2u * i + 1u] = make_ulonglong2(xd[2], xd[3]);
          }
        }
      } else {
        const uint8_t* lb = a.lvl8 + (size_t)k * rb;
        for (uint32_t v = lane; v < V; v += 64u) {
          const uint32_t l = lb[v];
          store_row<uint64_t>(&drow[v], l != 0xFFu ? (uint64_t)l * cost : ~0ull, nt);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Bit-parallel multi-source BFS (msbfs_kernel). Batch b = 32 consecutive positions of the
// batch order (bit j <-> row msperm[32 b + j]: for an all-sources call the compact
// clusters of DevGraph::corder, deepest first; else the call's own order). Closed form of LinkState::runSpf for uniform
// cost (LinkState.cpp:808-882), levels only: v is on level L+1 for source j iff bit j is
// in no visited word of v so far and in the frontier word of some usable neighbour u on
// level L that expands for j (u not overloaded, or u == the source itself: an overloaded
// source expands, LinkState.cpp:831-838). Usable edges are symmetric (Link::isUp is per
// link), so v pulls over its own row of up edges.
//
// LDS: F[2][kMaxV + 4] u32 frontier words (double-buffered by level parity, both at
// compile-time offsets so the buffer is an immediate of the ds instruction; slot kMaxV is
// a zero word that padding slots read, the next three hold control words), then the pull
// rows, four u16 byte offsets into F per node (8 B: one ds_read_b64). Thread t owns nodes t + 512 i (consecutive lanes,
// consecutive nodes: conflict-free banks) and keeps per node in registers its levels as 8
// bit-planes (plane b holds bit j iff bit b of the level of (source j, node) is set); a
// source's own bit is set in every plane (level 0xFF marks level 0: levels stop at 254, so
// 0xFF is free), and a visited word per node. Planes 0-1 take a step's new bits where the level's low bits are set (the
// level loop is unrolled by 4, so that is compile-time), planes 2-7 under uniform masks.
// A level ends with a barrier whose flag tells whether any node gained a bit; a batch
// deeper than 254 levels is abandoned and its rows listed for the u16 full-order re-run.
// At the end each node's planes are transposed (8 x 8 bit blocks) into 32 level bytes,
// written as u64 distance rows (level x cost, UINT64_MAX if unreached) and as u8 level
// rows for the next-hop pass.
// ---------------------------------------------------------------------------
constexpr uint32_t kMsThreads = 512, kMsBatch = 32;
template <uint32_t NPT>
struct MsLayout {
  static constexpr uint32_t kMaxV = kMsThreads * NPT;                // nodes a workgroup owns
  static constexpr uint32_t kF1 = (4u * (kMaxV + 4u) + 15u) & ~15u;  // byte offset of F[1]
  // control words in the padding after F[0]'s zero slot: [0..2] level flags, then F[1]'s
  // padding: the next batch
  static constexpr uint32_t kFlags = 4u * (kMaxV + 1u), kNext = kF1 + 4u * (kMaxV + 1u);
  static constexpr uint32_t kEll = 2u * kF1;  // pull rows (8 B per node)
  // Pull rows are stored for nodes < V. Every node slot but a thread's last is read each
  // step (nodes >= V read garbage rows and never gain a bit: their planes are all ones), so
  // the layout covers the rows of slots 0 .. NPT-2 of every thread; a thread's last slot
  // reads through a base clamped to row 0 when its node is >= V.
  __host__ __device__ static constexpr uint32_t bytes(uint32_t V) {
    const uint32_t a = kEll + 8u * V, b = kEll + 8u * (kMaxV - kMsThreads);
    return ((a > b ? a : b) + 15u) & ~15u;
  }
};

__device__ __forceinline__ uint32_t ms_rd(uint32_t boff) { return *(lds_u32*)(size_t)boff; }
__device__ __forceinline__ void ms_wr(uint32_t boff, uint32_t x) { *(lds_u32*)(size_t)boff = x; }
// Frontier store of a level step, opaque to the compiler's alias analysis: it goes to the
// other buffer than the step reads, so the next nodes' reads may issue before it (a plain
// store would serialise every node behind the previous one's store). The barrier that ends
// the level (s_waitcnt lgkmcnt(0); s_barrier, a memory clobber) orders it for the reads of
// the next level; in-order LDS completion keeps the compiler's counted waits conservative.
template <uint32_t OFF>
__device__ __forceinline__ void ms_wr_async(uint32_t base, uint32_t x) {
  asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(base), "v"(x), "i"(OFF));
}

// One level step: reads frontier buffer CUR (byte offset), writes NXT; M = L % 4; hm[b]
// = all ones iff bit b (2..7) of the new level L+1 is set.
// Address bases (opaque to the compiler, so it keeps two VGPRs and folds the rest into
// the ds instructions' 16-bit immediate offsets instead of holding one address per node):
// eb[h] = this thread's pull row of node i = 8h + (0..7), wb[x] = its frontier word of
// node i in buffer x (x = 0: F[0], 1: F[1])
struct MsBases {
  uint32_t eb[3], elast, wb[2];
};
// compile-time loop: f(std::integral_constant<uint32_t, I>) for I in [I0, N)
template <uint32_t I, uint32_t N>
struct MsUnroll {
  template <typename F>
  __device__ __forceinline__ static void run(F&& f) {
    if constexpr (I < N) {
      f(std::integral_constant<uint32_t, I>{});
      MsUnroll<I + 1u, N>::run(f);
    }
  }
};

// One level step over the thread's nodes in chunks of kMsChunk, software-pipelined in
// program order (LDS stores are never reordered with later loads, so the order written
// here is the issue order): the frontier reads of chunk c, then the pull-row reads of
// chunk c + 1, then chunk c's arithmetic and frontier stores.
constexpr uint32_t kMsChunk = 4;
template <uint32_t NPT, uint32_t CUR, uint32_t NXT>
__device__ __forceinline__ uint32_t ms_step(const MsBases& ab, uint32_t sink, uint32_t (&vis)[NPT],
                                            uint32_t (&p)[8][NPT], const uint32_t (&hm)[8]) {
  typedef __attribute__((address_space(3))) uint64_t lds_u64;
  static_assert(NPT % kMsChunk == 0, "whole chunks");
  constexpr uint32_t NC = NPT / kMsChunk;
  auto ell_of = [&](uint32_t i) {
    const uint32_t addr = i + 1u == NPT ? ab.elast : ab.eb[i / 8u] + 8u * kMsThreads * (i % 8u);
    const uint64_t x = *(const lds_u64*)(size_t)addr;
    return make_uint2((uint32_t)x, (uint32_t)(x >> 32));
  };
  uint2 er[kMsChunk];
#pragma unroll
  for (uint32_t r = 0; r < kMsChunk; ++r) er[r] = ell_of(r);
  uint32_t any = 0;
  MsUnroll<0, NC>::run([&](auto ic) {
    constexpr uint32_t c = decltype(ic)::value;
    uint32_t acc[kMsChunk];
#pragma unroll
    for (uint32_t r = 0; r < kMsChunk; ++r)
      acc[r] = ms_rd(CUR + (er[r].x & 0xFFFFu)) | ms_rd(CUR + (er[r].x >> 16)) | ms_rd(CUR + (er[r].y & 0xFFFFu)) |
               ms_rd(CUR + (er[r].y >> 16));
    if constexpr (c + 1u < NC) {
#pragma unroll
      for (uint32_t r = 0; r < kMsChunk; ++r) er[r] = ell_of(kMsChunk * (c + 1u) + r);
    }
#pragma unroll
    for (uint32_t r = 0; r < kMsChunk; ++r) {
      constexpr uint32_t i0 = kMsChunk * c;
      const uint32_t i = i0 + r;
      const uint32_t nw = acc[r] & ~vis[i];
      vis[i] |= nw;
      ms_wr(ab.wb[NXT != 0u] + 4u * kMsThreads * i, ((sink >> i) & 1u) ? 0u : nw);
#pragma unroll
      for (uint32_t b = 0; b < 8u; ++b) {
        p[b][i] |= nw & hm[b];  // the bits of level L+1
        asm volatile("" : "+v"(p[b][i]));  // updated here: not sunk past the barrier with nw live
      }
      any |= nw;
    }
  });
  return any;
}

template <uint32_t NPT>
__global__ __launch_bounds__(kMsThreads, 1) void msbfs_kernel(DevGraph g, SolveArgs a, uint64_t cost, uint32_t* ctr,
                                                              uint32_t* ovf_count, uint32_t flags) {
  using Lay = MsLayout<NPT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id();
  lds_u32* const ctl = (lds_u32*)(size_t)Lay::kFlags;  // [0..2] level flags
  lds_u32* const next_unit = (lds_u32*)(size_t)Lay::kNext;
  const bool nt = (flags & 1u) != 0, dist_here = (flags & 2u) == 0;
  const uint32_t rb = reach_row_bytes(V);
  const uint32_t ebase = Lay::kEll + 8u * tid;  // this thread's first pull row
  // zero both frontier buffers (slots of nodes >= V and the zero slot stay zero), then the
  // pull rows: rows hold <= 4 edges; a down edge or a missing slot reads the zero slot
  for (uint32_t w = tid; w < Lay::kEll / 4u; w += kMsThreads) smem[w] = 0u;  // F[0], F[1], control
  uint32_t sink = 0;
#pragma unroll
  for (uint32_t i = 0; i < NPT; ++i) {
    const uint32_t v = tid + kMsThreads * i;
    if (v < V) {
      uint32_t o[4] = {4u * Lay::kMaxV, 4u * Lay::kMaxV, 4u * Lay::kMaxV, 4u * Lay::kMaxV};
      const uint2 r = g.row2[v];
#pragma unroll
      for (uint32_t c = 0; c < 4u; ++c) {
        if (r.x + c < r.y) {
          const uint32_t av = g.adj[r.x + c];
          if (!(av & kEdgeDown)) o[c] = 4u * av;
        }
      }
      typedef __attribute__((address_space(3))) uint64_t lds_u64;
      *(lds_u64*)(size_t)(ebase + 8u * kMsThreads * i) =
          (uint64_t)(o[0] | (o[1] << 16)) | ((uint64_t)(o[2] | (o[3] << 16)) << 32);
      if (g.ovl[v]) sink |= 1u << i;
    }
  }
  __syncthreads();
  MsBases ab;
#pragma unroll
  for (uint32_t h = 0; h < 3u; ++h) {
    ab.eb[h] = ebase + 8u * kMsThreads * 8u * h;
    asm volatile("" : "+v"(ab.eb[h]));
  }
  ab.elast = tid + kMsThreads * (NPT - 1u) < V ? ebase + 8u * kMsThreads * (NPT - 1u) : Lay::kEll;
  ab.wb[0] = 4u * tid;
  ab.wb[1] = 4u * tid + Lay::kF1;
  asm volatile("" : "+v"(ab.elast), "+v"(ab.wb[0]), "+v"(ab.wb[1]));
  const uint32_t nbatch = (a.n + kMsBatch - 1u) / kMsBatch;
  for (uint32_t unit = blockIdx.x; unit < nbatch;) {
    const uint32_t k0 = unit * kMsBatch, nbk = min(kMsBatch, a.n - k0);
    // per-node addresses are re-derived from an opaque copy of tid in each phase: hoisted
    // out of the batch loop they would hold NPT more registers through the level loop
    uint32_t tb = tid;
    asm volatile("" : "+v"(tb));
    // level 0: the sources' own bits in F[0]
#pragma unroll
    for (uint32_t i = 0; i < NPT; ++i)
      if (tb + kMsThreads * i < V) ms_wr(4u * (tb + kMsThreads * i), 0u);
    if (tid < 3u) ctl[tid] = 0u;
    __syncthreads();
    if (tid < nbk) {
      const uint32_t src = a.sources[a.msperm[k0 + tid]];
      if (src < V) lds_or((lds_u32*)(size_t)(4u * src), 1u << tid);
    }
    __syncthreads();
    // levels as bit-planes; a source's own bit reads level 0xFF (all planes), a node >= V
    // is "visited" for every source so it never gains a bit
    uint32_t vis[NPT], p[8][NPT];
#pragma unroll
    for (uint32_t i = 0; i < NPT; ++i) {
      const uint32_t v = tb + kMsThreads * i;
      vis[i] = v < V ? ms_rd(4u * v) : ~0u;
#pragma unroll
      for (uint32_t b = 0; b < 8u; ++b) p[b][i] = vis[i];
    }
    uint32_t L = 0;
    bool ovf = false;
    uint32_t hm[8];
    auto masks = [&]() {  // the bits of the level the next step makes (L + 1)
#pragma unroll
      for (uint32_t b = 0; b < 8u; ++b) hm[b] = (((L + 1u) >> b) & 1u) ? ~0u : 0u;
    };
    // end of a level: did any node gain a bit? (flag per level, three in rotation: the one
    // cleared here was last read before the previous barrier)
    auto level_end = [&](uint32_t any) -> bool {
      if (__builtin_amdgcn_ballot_w64(any != 0u) != 0ull && lane == 0u) ctl[L % 3u] = 1u;
      lds_barrier();
      const uint32_t f = __builtin_amdgcn_readfirstlane(ctl[L % 3u]);
      if (tid == 0u) ctl[(L + 2u) % 3u] = 0u;
      ++L;
      return f != 0u;
    };
    for (;;) {
      if (L + 2u > 254u) {  // levels must stay below 255 (u8 rows, 0xFF = unreached)
        ovf = true;
        break;
      }
      masks();
      if (!level_end(ms_step<NPT, 0, Lay::kF1>(ab, sink, vis, p, hm))) break;
      masks();
      if (!level_end(ms_step<NPT, Lay::kF1, 0>(ab, sink, vis, p, hm))) break;
    }
    if (ovf) {
      if (tid < nbk) {
        const uint32_t k = a.msperm[k0 + tid];
        a.rowok[k] = 0u;
        a.ovf_list[atomicAdd(ovf_count, 1u)] = k;
      }
    } else {
      // rows out. Each node's planes are transposed in place (8 x 8 bit blocks): afterwards
      // p[c][i] holds the level bytes of sources 4c .. 4c+3 of node i (0xFF: not reached)
#pragma unroll
      for (uint32_t i = 0; i < NPT; ++i) {
        uint32_t lw[8];
#pragma unroll
        for (uint32_t kb = 0; kb < 4u; ++kb) {  // sources 8kb .. 8kb+7
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (uint32_t b = 0; b < 4u; ++b) {
            lo |= ((p[b][i] >> (8u * kb)) & 0xFFu) << (8u * b);
            hi |= ((p[b + 4u][i] >> (8u * kb)) & 0xFFu) << (8u * b);
          }
          uint64_t x = (uint64_t)lo | ((uint64_t)hi << 32);
          uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
          x = x ^ t ^ (t << 7);
          t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
          x = x ^ t ^ (t << 14);
          t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
          x = x ^ t ^ (t << 28);
          // byte 0 (no plane bit): not reached -> 0xFF; byte 0xFF (the source itself) -> 0
          uint32_t w0 = (uint32_t)x, w1 = (uint32_t)(x >> 32);
          w0 ^= ((swar_zero_hi(w0) | swar_zero_hi(~w0)) >> 7) * 0xFFu;
          w1 ^= ((swar_zero_hi(w1) | swar_zero_hi(~w1)) >> 7) * 0xFFu;
          lw[2u * kb] = w0;
          lw[2u * kb + 1u] = w1;
        }
#pragma unroll
        for (uint32_t c = 0; c < 8u; ++c) p[c][i] = lw[c];
      }
      uint32_t to = tid;
      asm volatile("" : "+v"(to));
#pragma unroll
      for (uint32_t j = 0; j < kMsBatch; ++j) {
        if (j >= nbk) continue;  // uniform
        const size_t k = a.msperm[k0 + j];
        uint8_t* lrow = a.lvl8 + k * rb;
        uint64_t* drow = a.dist + k * V;
#pragma unroll
        for (uint32_t i = 0; i < NPT; ++i) {
          const uint32_t v = to + kMsThreads * i;
          if (v >= V) continue;
          const uint32_t l = (p[j >> 2][i] >> (8u * (j & 3u))) & 0xFFu;
          lrow[v] = (uint8_t)l;
          if (dist_here) store_row<uint64_t>(&drow[v], l != 0xFFu ? (uint64_t)l * cost : ~0ull, nt);
        }
      }
      if (tid < nbk) {
        const uint32_t k = a.msperm[k0 + tid];
        a.rowok[k] = a.sources[k] < V ? 1u : 0u;
      }
    }
    __syncthreads();  // every lane is done with this batch's LDS and next_unit
    if (tid == 0) *next_unit = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = *next_unit;
  }
  retire_workgroup(ctr, nullptr);
}

// ---------------------------------------------------------------------------
// Tile-active multi-source BFS (msbfs_tile_kernel, round 3: the G100 all-sources path).
//
// Same closed form and bit-parallel state as msbfs_kernel, but a level no longer pulls over
// every node. Nodes are renumbered (DevGraph::tord) so that 64 consecutive internal ids —
// one wavefront slot — form a compact tile, and a level step only processes the tiles a
// node of which may gain a bit: tile T can gain at step L only if a node of a tile in
// N(T) (DevGraph::tmask) wrote a non-zero frontier word at step L-1. A processed tile whose
// wave sees any non-zero frontier word ORs its tmask row into the next step's activity
// bitmask (act[3][8] u32 in rotation, LDS); an empty bitmask ends the batch. For a
// 32-source cluster on G100 a level touches ~37 of 157 tiles (scripts/tile_sim.py).
//
// Frontier words of skipped tiles are not rewritten: the buffer then holds a frontier of an
// earlier level m <= L-1 of the same batch. Such bits are harmless: bit j of node x at level
// m (x expands: sinks write 0) puts every neighbour of x on level <= m + 1 <= L for source
// j, so the neighbour's visited word already holds j when it reads the stale word. Both
// buffers are zeroed at the start of a batch.
//
// Thread t owns internal nodes p = t + 512 i (slot i = tile 8i + wave, lane = position in
// the tile). A wave's active slots of a step are a bit mask in SGPRs; the pull row of the
// next active slot is read while the current slot's frontier reads are in flight.
// ---------------------------------------------------------------------------
// LDS layout (bytes) for vpad = ntiles * 64 internal ids: F[0] and F[1] frontier words
// (vpad + 4 each; word vpad is a zero word padding slots read), act[3][8] activity words,
// the next batch, the tiles' neighbour lists (u8 tile ids, kTileList per tile), pull rows.
struct MsTLayout {
  uint32_t f1, act, next, tl, ell, total;
  __host__ __device__ explicit MsTLayout(uint32_t ntiles) {
    const uint32_t vpad = ntiles * kTileNodes;
    f1 = (4u * (vpad + 4u) + 15u) & ~15u;
    act = 2u * f1;
    next = act + 96u;
    tl = act + 128u;
    ell = tl + ((ntiles * kTileList + 15u) & ~15u);
    total = ell + 8u * vpad;
  }
};

// The tile kernel's arguments, compact (fewer kernel-argument SGPRs than DevGraph + SolveArgs)
struct MsTileArgs {
  const uint32_t *tord, *tinv, *adj, *tmask, *sources, *msperm, *xcount;
  const uint2* row2;
  const uint8_t *ovl, *tlist;
  uint8_t *lvl8, *rowok;
  uint64_t* dist;
  uint32_t* ovf_list;
  uint32_t V, ntiles, n;
};

template <uint32_t NPT, bool PROF>
__global__ __launch_bounds__(kMsThreads, 1) void msbfs_tile_kernel(MsTileArgs t, uint64_t cost,
                                                                   uint32_t* ctr, uint32_t* ovf_count, uint32_t flags,
                                                                   unsigned long long* prof) {
  // tuning (OPENR_SPF_MS_PROF=1): wave 0's cycles per phase of every level step — [0] level
  // start (activity words, chunk mask), [1] a chunk's frontier reads, [2] its arithmetic and
  // frontier stores, [3] its emission marks, [4] the barrier — and [5] steps, [6] active
  // chunks, [7] batches. A stamp follows an asm use of the value the phase waits for.
  const bool pf = PROF && prof != nullptr && threadIdx.x < 64u;
  unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long ts = 0;
#define OPENR_MS_STAMP(i, dep)                                     \
  do {                                                             \
    if (pf) {                                                      \
      asm volatile("" ::"v"(dep));                                 \
      const long long tnow = (long long)__builtin_amdgcn_s_memtime(); \
      pacc[i] += (unsigned long long)(tnow - ts);                  \
      ts = tnow;                                                   \
    }                                                              \
  } while (0)
  typedef __attribute__((address_space(3))) uint64_t lds_u64;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = t.V, tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const MsTLayout lay(t.ntiles);
  lds_u32* const act = (lds_u32*)(size_t)lay.act;
  lds_u32* const next_unit = (lds_u32*)(size_t)lay.next;
  const bool nt = (flags & 1u) != 0, dist_here = (flags & 2u) == 0;
  const uint32_t rb = reach_row_bytes(V), vpad = t.ntiles * kTileNodes;
  const uint32_t ebase = lay.ell + 8u * tid;  // this thread's first pull row
  const uint32_t kZero = 4u * vpad;           // byte offset of the zero word
  const uint32_t F1 = lay.f1;
  // control words zero, neighbour lists staged; pull rows in internal ids (a down edge or a
  // missing slot reads the zero word); rows of padding ids (V <= p < vpad) read zero words
  for (uint32_t w = tid; w < 32u; w += kMsThreads) act[w] = 0u;
  for (uint32_t w = tid; w < (t.ntiles * kTileList + 3u) / 4u; w += kMsThreads)
    *(lds_u32*)(size_t)(lay.tl + 4u * w) = reinterpret_cast<const uint32_t*>(t.tlist)[w];
  if (tid == 0) {
    ms_wr(kZero, 0u);
    ms_wr(F1 + kZero, 0u);
  }
  uint32_t sink = 0;
#pragma unroll
  for (uint32_t i = 0; i < NPT; ++i) {
    const uint32_t p = tid + kMsThreads * i;
    if (p < vpad) {
      uint32_t o[4] = {kZero, kZero, kZero, kZero};
      if (p < V) {
        const uint32_t v = t.tord[p];
        const uint2 r = t.row2[v];
#pragma unroll
        for (uint32_t c = 0; c < 4u; ++c) {
          if (r.x + c < r.y) {
            const uint32_t av = t.adj[r.x + c];
            if (!(av & kEdgeDown)) o[c] = 4u * t.tinv[av];
          }
        }
        if (t.ovl[v]) sink |= 1u << i;
      }
      *(lds_u64*)(size_t)(ebase + 8u * kMsThreads * i) =
          (uint64_t)(o[0] | (o[1] << 16)) | ((uint64_t)(o[2] | (o[3] << 16)) << 32);
    }
  }
  // rows: the call's, then (extended batch) the halo rows
  const uint32_t ntot = t.xcount ? t.n + t.xcount[0] : t.n;
  const uint32_t nbatch = (ntot + kMsBatch - 1u) / kMsBatch;
  for (uint32_t unit = blockIdx.x; unit < nbatch;) {
    const uint32_t k0 = unit * kMsBatch, nbk = min(kMsBatch, ntot - k0);
    uint32_t tb = tid;
    asm volatile("" : "+v"(tb));
    // both frontier buffers zero over the owned ids, activity bitmasks zero
#pragma unroll
    for (uint32_t i = 0; i < NPT; ++i) {
      if (tb + kMsThreads * i < vpad) {
        ms_wr(4u * (tb + kMsThreads * i), 0u);
        ms_wr(F1 + 4u * (tb + kMsThreads * i), 0u);
      }
    }
    if (tid < 24u) act[tid] = 0u;
    __syncthreads();
    // level 0: the sources' own bits in F[0]; their tiles' neighbourhoods are active at step 0
    if (tid < nbk) {
      const uint32_t src = t.sources[t.msperm[k0 + tid]];
      if (src < V) {
        const uint32_t ps = t.tinv[src];
        lds_or((lds_u32*)(size_t)(4u * ps), 1u << tid);
        const uint32_t* m = t.tmask + (size_t)(ps / kTileNodes) * kTileMaskWords;
#pragma unroll
        for (uint32_t k = 0; k < kTileMaskWords; ++k)
          if (m[k]) lds_or(&act[k], m[k]);
      }
    }
    __syncthreads();
    // levels as bit-planes; the visited word of a node is the OR of its planes (every level
    // >= 1 has a bit set, level 0 is all ones); a node >= V is visited for every source
    uint32_t p[8][NPT];
#pragma unroll
    for (uint32_t i = 0; i < NPT; ++i) {
      const uint32_t q = tb + kMsThreads * i;
      const uint32_t v0 = q < V ? ms_rd(4u * q) : ~0u;
#pragma unroll
      for (uint32_t b = 0; b < 8u; ++b) p[b][i] = v0;
    }
    uint32_t L = 0;
    bool ovf = false;
    if (pf) {
      ts = (long long)__builtin_amdgcn_s_memtime();
      pacc[7] += 1;
    }
    for (;;) {
      // this step's activity: bit (8i + wave) of act[L % 3] for slot i; slots go in chunks
      // of kMsChunk (tile order makes a chunk's tiles neighbours: tile_order in spf_capi)
      const uint32_t cur_set = L % 3u;
      uint32_t aw[5];
#pragma unroll
      for (uint32_t k = 0; k < 5u; ++k) aw[k] = __builtin_amdgcn_readfirstlane(act[8u * cur_set + k]);
      uint32_t anyw = aw[0] | aw[1] | aw[2] | aw[3] | aw[4];
#pragma unroll
      for (uint32_t k = 5; k < kTileMaskWords; ++k) anyw |= __builtin_amdgcn_readfirstlane(act[8u * cur_set + k]);
      if (anyw == 0u) break;  // uniform: every wave read the same words after the barrier
      if (L + 2u > 254u) {  // levels must stay below 255 (u8 rows, 0xFF = unreached)
        ovf = true;
        break;
      }
      constexpr uint32_t NC = NPT / kMsChunk;
      // chunk c of this wave holds tiles 32c + 8r + wave (r < 4): bits wave + 8r of word c
      uint32_t C = 0;  // active chunks
#pragma unroll
      for (uint32_t c = 0; c < NC; ++c) C |= ((aw[c] & (0x01010101u << wave)) != 0u ? 1u : 0u) << c;
      if (pf) {
        pacc[5] += 1;
        pacc[6] += (unsigned long long)__builtin_popcount(C);
      }
      OPENR_MS_STAMP(0, C);
      if (tid < 8u) act[8u * ((L + 2u) % 3u) + tid] = 0u;  // last read one step ago
      lds_u32* const nact = act + 8u * ((L + 1u) % 3u);
      uint32_t hm[8];
#pragma unroll
      for (uint32_t b = 0; b < 8u; ++b) hm[b] = (((L + 1u) >> b) & 1u) ? ~0u : 0u;
      const uint32_t cur = (L & 1u) ? F1 : 0u, nxt = (L & 1u) ? 0u : F1;
      // pull rows of the first active chunk (a slot past the last tile has none: it reads zero
      // words and writes nothing)
      const uint32_t zrow = kZero | (kZero << 16);
      const uint64_t zer = (uint64_t)zrow | ((uint64_t)zrow << 32);
      uint64_t er[kMsChunk];
      {
        const uint32_t c0 = C ? (uint32_t)__builtin_ctz(C) : 0u;
        uint32_t eaddr = ebase + 8u * kMsThreads * kMsChunk * c0;
        asm volatile("" : "+v"(eaddr));
#pragma unroll
        for (uint32_t r = 0; r < kMsChunk; ++r)
          er[r] = (C && 8u * (kMsChunk * c0 + r) + wave < t.ntiles) ? *(const lds_u64*)(size_t)(eaddr + 8u * kMsThreads * r)
                                                                 : zer;
      }
      MsUnroll<0, NC>::run([&](auto ic) {
        constexpr uint32_t c = decltype(ic)::value;
        if ((C >> c) & 1u) {  // uniform
          uint32_t f[kMsChunk];
#pragma unroll
          for (uint32_t r = 0; r < kMsChunk; ++r) {
            const uint32_t lo = (uint32_t)er[r], hi = (uint32_t)(er[r] >> 32);
            f[r] = ms_rd(cur + (lo & 0xFFFFu)) | ms_rd(cur + (lo >> 16)) | ms_rd(cur + (hi & 0xFFFFu)) |
                   ms_rd(cur + (hi >> 16));
          }
          OPENR_MS_STAMP(1, f[0] | f[1] | f[2] | f[3]);
          const uint32_t rest = C & ~((2u << c) - 1u);
          if (rest) {  // the next active chunk's pull rows, in flight with this chunk's reads
            const uint32_t c1 = (uint32_t)__builtin_ctz(rest);
            uint32_t na = ebase + 8u * kMsThreads * kMsChunk * c1;
            asm volatile("" : "+v"(na));
#pragma unroll
            for (uint32_t r = 0; r < kMsChunk; ++r)
              er[r] = 8u * (kMsChunk * c1 + r) + wave < t.ntiles ? *(const lds_u64*)(size_t)(na + 8u * kMsThreads * r) : zer;
          }
          uint32_t em = 0;  // slots of the chunk that emit (a non-zero frontier word)
#pragma unroll
          for (uint32_t r = 0; r < kMsChunk; ++r) {
            constexpr uint32_t i0 = kMsChunk * c;
            const uint32_t i = i0 + r;
            if (8u * i + wave >= t.ntiles) continue;  // uniform: a slot past the last tile
            const uint32_t vis = p[0][i] | p[1][i] | p[2][i] | p[3][i] | p[4][i] | p[5][i] | p[6][i] | p[7][i];
            const uint32_t nw = f[r] & ~vis;
            const uint32_t fw = ((sink >> i) & 1u) ? 0u : nw;
            ms_wr(nxt + 4u * (tb + kMsThreads * i), fw);
#pragma unroll
            for (uint32_t b = 0; b < 8u; ++b) {
              p[b][i] |= nw & hm[b];
              asm volatile("" : "+v"(p[b][i]));  // updated here: not sunk past the barrier with nw live
            }
            em |= (__builtin_amdgcn_ballot_w64(fw != 0u) != 0ull ? 1u : 0u) << r;
          }
          OPENR_MS_STAMP(2, em);
          // emitting tiles mark their neighbourhoods (lists: lane j < kTileList holds the
          // j-th tile, the tile itself included) active for the next step
          const uint32_t lane = __lane_id();
          for (uint32_t m = em; m; m &= m - 1u) {
            const uint32_t tile = 8u * (kMsChunk * c + (uint32_t)__builtin_ctz(m)) + wave;
            const uint32_t nbt = lane < kTileList ? *(const lds_u8*)(size_t)(lay.tl + kTileList * tile + lane) : 0xFFu;
            if (nbt < 0xFEu) lds_or(&nact[nbt >> 5], 1u << (nbt & 31u));
            // more than kTileList neighbour tiles (list head 0xFE): every tile
            if (__builtin_amdgcn_readfirstlane(nbt) == 0xFEu && lane < kTileMaskWords) lds_or(&nact[lane], ~0u);
          }
          OPENR_MS_STAMP(3, em);
        }
      });
      lds_barrier();
      OPENR_MS_STAMP(4, L);
      ++L;
    }
    if (ovf) {
      if (tid < nbk) {
        const uint32_t k = t.msperm[k0 + tid];
        t.rowok[k] = 0u;
        // a halo row is no call row: the sources that need it are listed by the next-hop pass
        if (k < t.n) t.ovf_list[atomicAdd(ovf_count, 1u)] = k;
      }
    } else {
      // rows out: planes -> level bytes (as msbfs_kernel), stored at the node's own id
#pragma unroll
      for (uint32_t i = 0; i < NPT; ++i) {
        uint32_t lw[8];
#pragma unroll
        for (uint32_t kb = 0; kb < 4u; ++kb) {
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (uint32_t b = 0; b < 4u; ++b) {
            lo |= ((p[b][i] >> (8u * kb)) & 0xFFu) << (8u * b);
            hi |= ((p[b + 4u][i] >> (8u * kb)) & 0xFFu) << (8u * b);
          }
          uint64_t x = (uint64_t)lo | ((uint64_t)hi << 32);
          uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
          x = x ^ t ^ (t << 7);
          t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
          x = x ^ t ^ (t << 14);
          t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
          x = x ^ t ^ (t << 28);
          uint32_t w0 = (uint32_t)x, w1 = (uint32_t)(x >> 32);
          w0 ^= ((swar_zero_hi(w0) | swar_zero_hi(~w0)) >> 7) * 0xFFu;
          w1 ^= ((swar_zero_hi(w1) | swar_zero_hi(~w1)) >> 7) * 0xFFu;
          lw[2u * kb] = w0;
          lw[2u * kb + 1u] = w1;
        }
#pragma unroll
        for (uint32_t c = 0; c < 8u; ++c) p[c][i] = lw[c];
      }
      uint32_t orig[NPT];  // internal -> node id (the visited words' registers are free now)
#pragma unroll
      for (uint32_t i = 0; i < NPT; ++i) {
        const uint32_t q = tb + kMsThreads * i;
        orig[i] = q < V ? t.tord[q] : ~0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < kMsBatch; ++j) {
        if (j >= nbk) continue;  // uniform
        const size_t k = t.msperm[k0 + j];
        uint8_t* lrow = t.lvl8 + k * rb;
        uint64_t* drow = t.dist + k * V;
#pragma unroll
        for (uint32_t i = 0; i < NPT; ++i) {
          const uint32_t v = orig[i];
          if (v >= V) continue;
          const uint32_t l = (p[j >> 2][i] >> (8u * (j & 3u))) & 0xFFu;
          lrow[v] = (uint8_t)l;
          if (dist_here) store_row<uint64_t>(&drow[v], l != 0xFFu ? (uint64_t)l * cost : ~0ull, nt);
        }
      }
      if (tid < nbk) {
        const uint32_t k = t.msperm[k0 + tid];
        t.rowok[k] = t.sources[k] < V ? 1u : 0u;
      }
    }
    __syncthreads();  // every lane is done with this batch's LDS and next_unit
    if (tid == 0) *next_unit = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = *next_unit;
  }
#undef OPENR_MS_STAMP
  if (pf && __lane_id() == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&prof[i], pacc[i]);
  retire_workgroup(ctr, nullptr);
}

template <uint32_t NPT>
hipError_t launch_msbfs_tile_npt(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t* blk, int num_cus,
                                 hipStream_t s, uint32_t flags) {
  const bool want_prof = env_u32("OPENR_SPF_MS_PROF", 0u, 0u, 1u) != 0;
  auto k = want_prof ? msbfs_tile_kernel<NPT, true> : msbfs_tile_kernel<NPT, false>;
  const uint32_t lds = MsTLayout(g.ntiles).total;
  MsTileArgs t;
  t.tord = g.tord;
  t.tinv = g.tinv;
  t.adj = g.adj;
  t.tmask = g.tmask;
  t.sources = a.sources;
  t.msperm = a.msperm;
  t.xcount = a.xcount;
  t.row2 = g.row2;
  t.ovl = g.ovl;
  t.tlist = g.tlist;
  t.lvl8 = a.lvl8;
  t.rowok = a.rowok;
  t.dist = a.dist;
  t.ovf_list = a.ovf_list;
  t.V = g.V;
  t.ntiles = g.ntiles;
  t.n = a.n;
  hipError_t err =
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  // an extended batch holds at most the halo bound more rows (ms_ext_rows)
  const uint32_t nbatch = ((a.xcount ? ms_ext_rows(g, a.n) : a.n) + kMsBatch - 1u) / kMsBatch;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>(nbatch, (uint32_t)num_cus));
  static unsigned long long* prof_buf = nullptr;  // tuning aid: per-phase cycle sums, printed
  unsigned long long* prof = nullptr;
  if (want_prof) {
    if (!prof_buf && hipMalloc(&prof_buf, 8 * sizeof(unsigned long long)) != hipSuccess) prof_buf = nullptr;
    prof = prof_buf;
    if (prof) (void)hipMemsetAsync(prof, 0, 8 * sizeof(unsigned long long), s);
  }
  note_launch("msbfs_tile_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(kMsThreads), lds, s, t, cost, blk, blk + 4, flags, prof);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && prof) {
    unsigned long long h[8];
    if (hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess) {
      const double st = h[5] ? (double)h[5] : 1.0, ch = h[6] ? (double)h[6] : 1.0;
      std::fprintf(stderr,
                   "msbfs_tile: grid=%u batches(wave0)=%llu steps/batch=%.1f active chunks/step=%.2f | cycles/step: "
                   "start %.0f barrier %.0f | cycles/chunk: reads %.0f compute %.0f marks %.0f\n",
                   grid, h[7], h[7] ? st / (double)h[7] : 0.0, ch / st, h[0] / st, h[4] / st, h[1] / ch, h[2] / ch,
                   h[3] / ch);
    }
  }
  return e;
}

template <uint32_t NPT>
hipError_t launch_msbfs_npt(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t* blk, int num_cus,
                            hipStream_t s, uint32_t flags) {
  using Lay = MsLayout<NPT>;
  auto k = msbfs_kernel<NPT>;
  const uint32_t lds = Lay::bytes(g.V);
  hipError_t err =
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  const uint32_t nbatch = (a.n + kMsBatch - 1u) / kMsBatch;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>(nbatch, (uint32_t)num_cus));
  note_launch("msbfs_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(kMsThreads), lds, s, g, a, cost, blk, blk + 4, flags);
  return hipGetLastError();
}

}  // namespace

// Which level pass an all-sources batch takes (0: none, 1: reach pass, 2: msbfs).
// Knobs: OPENR_SPF_BFS_MSBFS (0 off, 1 whenever it applies, 2 = auto) and
// OPENR_SPF_BFS_REACH (0 off, 1 whenever it applies, 2 = auto); auto = batches of >= V
// sources, where every neighbour of a source is likely in the batch.
// rows of an extended batch of n sources: the call's plus at most one halo row per
// usable neighbour slot, and never more halo rows than nodes outside the call
uint32_t ms_ext_rows(const DevGraph& g, uint32_t n) {
  return n + std::min<uint32_t>(g.V, (uint32_t)std::min<uint64_t>((uint64_t)n * g.max_deg, 0xFFFFFFFFu));
}

// the tile-active multi-source BFS serves the graph (tile order built, layout fits)
bool ms_tile_ok(const DevGraph& g) {
  return g.tord && g.tinv && g.tmask && g.tlist && g.ntiles <= 32u * kTileMaskWords &&
         g.ntiles * kTileNodes <= 20u * kMsThreads && MsTLayout(g.ntiles).total <= kMaxLds &&
         env_u32("OPENR_SPF_MSBFS_TILE", 1u, 0u, 1u) != 0u;
}

// wave-reach knob: 0 off, 1 whenever it applies, 2 auto
static uint32_t wreach_knob() { return env_u32("OPENR_SPF_BFS_WREACH", 0u, 0u, 2u); }

// queue half: the widest sampled level with a quarter's margin (OPENR_SPF_REACH_QHALF, tests:
// a smaller half, so wide levels take the u16 re-run)
uint32_t allsrc_qhalf(const DevGraph& g) {
  const uint32_t need1 = std::max<uint32_t>(g.max_deg + 1u, g.est_width1 + g.est_width1 / 4u);
  const uint32_t qforce = env_u32("OPENR_SPF_REACH_QHALF", 0u, 0u, 65535u);
  return qforce ? (std::max<uint32_t>(qforce, g.max_deg + 1u) + 15u) & ~15u : (std::max<uint32_t>(64u, need1) + 15u) & ~15u;
}

bool allsrc_ext_ok(const DevGraph& g) {
  return g.crank && (ms_tile_ok(g) || (g.elld && wreach_knob() != 0u)) && env_u32("OPENR_SPF_MSBFS_HALO", 1u, 0u, 1u);
}

int allsrc_pass(const DevGraph& g, const SolveArgs& a) {
  if (!a.lvl8 || !a.rowmap || !a.rowok || a.out_row || a.perm || a.tight || a.ign_ptr || g.max_deg > 4u) return 0;
  // the wave-reach pass: a full batch, or a partial one extended with halo rows
  const uint32_t wr = wreach_knob();
  if (wr != 0u && wreach_lds_bytes(g, allsrc_qhalf(g)) &&
      (a.n >= g.V || (a.xsrc && a.xcount && a.xslot && a.xdup && g.crank)))
    return 3;
  const bool ms_ok = a.msperm && a.mscnt;
  const uint32_t ms = env_u32("OPENR_SPF_BFS_MSBFS", 0u, 0u, 2u);
  if (ms != 0u && ms_ok && (ms_tile_ok(g) || (MsLayout<20>::bytes(g.V) <= kMaxLds && g.V <= MsLayout<20>::kMaxV)) &&
      (ms == 1u || a.n >= g.V))
    return 2;
  const uint32_t rk = env_u32("OPENR_SPF_BFS_REACH", 0u, 0u, 2u);  // opt-in, as above
  if (rk != 0u && (rk == 1u || a.n >= g.V)) return 1;
  return 0;
}

hipError_t launch_allsrc(int pass, const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t half, uint32_t* blk,
                         int num_cus, hipStream_t s, LaunchInfo* info) {
  // OPENR_SPF_REACH_DIST=2: the next-hop pass writes the distance rows (streaming) instead
  const bool dist2 = env_u32("OPENR_SPF_REACH_DIST", 1u, 1u, 2u) == 2u;
  uint32_t flags = nt_stores() | (dist2 ? 2u : 0u);
  const uint32_t mgrid = std::max<uint32_t>(1u, std::min<uint32_t>((g.V + 255u) / 256u, 4u * (uint32_t)num_cus));
  const uint32_t ngrid = std::max<uint32_t>(1u, std::min<uint32_t>((a.n + 255u) / 256u, 4u * (uint32_t)num_cus));
  // a partial batch on the tile-active pass: extended with halo rows (ms_ext_*)
  const bool ext = (pass == 3 || (pass == 2 && ms_tile_ok(g))) && a.n < g.V && a.xsrc && a.xcount && a.xslot &&
                   a.xdup && g.crank && env_u32("OPENR_SPF_MSBFS_HALO", 1u, 0u, 1u);
  hipError_t err;
  if (pass == 3 && a.n < g.V && !ext) return hipErrorInvalidValue;  // allsrc_pass checked the scratch
  if (ext) {
    note_launch("ms_ext");
    hipLaunchKernelGGL(ms_ext_clear_kernel, dim3(mgrid), dim3(256), 0, s, a.rowmap, a.xslot, g.V, a.xcount);
    hipLaunchKernelGGL(ms_ext_fill_kernel, dim3(ngrid), dim3(256), 0, s, a.sources, a.n, g.V, g.crank, a.rowmap,
                       a.xslot, a.xsrc, a.xdup, a.xcount);
    hipLaunchKernelGGL(ms_ext_halo_kernel, dim3(ngrid), dim3(256), 0, s, g, a.sources, a.n, a.rowmap, a.xslot, a.xsrc,
                       a.xcount);
    if (pass == 2)  // batch order of the multi-source pass (the wave-reach pass takes rows as they are)
      hipLaunchKernelGGL(ms_ext_order_kernel, dim3(1), dim3(1024), 0, s, a.xslot, g.V, a.xdup, a.xcount, a.msperm);
  } else {
    note_launch("reach_map");
    hipLaunchKernelGGL(reach_map_clear_kernel, dim3(mgrid), dim3(256), 0, s, a.rowmap, g.V);
    hipLaunchKernelGGL(reach_map_fill_kernel, dim3(ngrid), dim3(256), 0, s, a.rowmap, a.sources, a.n, g.V);
  }
  if (pass == 3) {
    SolveArgs b = a;  // the level pass solves [sources | halo]; the next-hop pass the call's rows
    if (ext) b.sources = a.xsrc;
    else b.xcount = nullptr;
    err = launch_wreach(g, b, half, blk, num_cus, s, info);
  } else if (ext) {
    SolveArgs b = a;  // the multi-source pass solves [sources | halo]; the next-hop pass the call's rows
    b.sources = a.xsrc;
    if (info) info->kernel = "msbfs_tile_kernel";
    const uint32_t need = (g.ntiles * kTileNodes + kMsThreads - 1u) / kMsThreads;
    if (need <= 4u) err = launch_msbfs_tile_npt<4>(g, b, cost, blk, num_cus, s, flags);
    else if (need <= 8u) err = launch_msbfs_tile_npt<8>(g, b, cost, blk, num_cus, s, flags);
    else if (need <= 12u) err = launch_msbfs_tile_npt<12>(g, b, cost, blk, num_cus, s, flags);
    else if (need <= 16u) err = launch_msbfs_tile_npt<16>(g, b, cost, blk, num_cus, s, flags);
    else err = launch_msbfs_tile_npt<20>(g, b, cost, blk, num_cus, s, flags);
  } else if (pass == 2) {
    if (!a.msperm || !a.mscnt) return hipErrorInvalidValue;
    const uint32_t pgrid = ngrid;
    err = hipMemsetAsync(a.mscnt, 0, sizeof(uint32_t), s);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(ms_perm_count_kernel, dim3(pgrid), dim3(256), 0, s, a.sources, a.n, a.rowmap, g.V, a.mscnt);
    hipLaunchKernelGGL(ms_perm_fill_kernel, dim3(pgrid), dim3(256), 0, s, g.corder, a.rowmap, a.n, g.V, a.mscnt,
                       a.msperm);
    SolveArgs b = a;
    b.xcount = nullptr;  // every neighbour row is in the call
    if (ms_tile_ok(g)) {  // tile-active variant (OPENR_SPF_MSBFS_TILE=0: the dense pull)
      const uint32_t need = (g.ntiles * kTileNodes + kMsThreads - 1u) / kMsThreads;  // internal ids per thread
      if (info) info->kernel = "msbfs_tile_kernel";
      if (need <= 4u) err = launch_msbfs_tile_npt<4>(g, b, cost, blk, num_cus, s, flags);
      else if (need <= 8u) err = launch_msbfs_tile_npt<8>(g, b, cost, blk, num_cus, s, flags);
      else if (need <= 12u) err = launch_msbfs_tile_npt<12>(g, b, cost, blk, num_cus, s, flags);
      else if (need <= 16u) err = launch_msbfs_tile_npt<16>(g, b, cost, blk, num_cus, s, flags);
      else err = launch_msbfs_tile_npt<20>(g, b, cost, blk, num_cus, s, flags);
    } else {
      const uint32_t need = (g.V + kMsThreads - 1u) / kMsThreads;  // nodes per thread
      if (info) info->kernel = "msbfs_kernel";
      if (need <= 4u) err = launch_msbfs_npt<4>(g, a, cost, blk, num_cus, s, flags);
      else if (need <= 8u) err = launch_msbfs_npt<8>(g, a, cost, blk, num_cus, s, flags);
      else if (need <= 12u) err = launch_msbfs_npt<12>(g, a, cost, blk, num_cus, s, flags);
      else if (need <= 16u) err = launch_msbfs_npt<16>(g, a, cost, blk, num_cus, s, flags);
      else err = launch_msbfs_npt<20>(g, a, cost, blk, num_cus, s, flags);
    }
  } else {
    constexpr int BLOCK = 128;
    // queue reads of lanes past a level's end land up to BLOCK entries past the halves
    const uint32_t ring_alloc = 2u * half + (uint32_t)BLOCK;
    const uint32_t lds = reach_layout(g.V, ring_alloc).total;
    if (lds > kMaxLds) return hipErrorInvalidValue;
    auto k = bfs_reach_kernel<BLOCK>;
    err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    if (info) {
      info->lds_bytes = lds;
      info->grid = blocks_for(a.n, lds, num_cus, BLOCK);
      info->kernel = "bfs_reach_kernel";
    }
    note_launch("bfs_reach_kernel");
    hipLaunchKernelGGL(k, dim3(blocks_for(a.n, lds, num_cus, BLOCK)), dim3(BLOCK), lds, s, g, a, cost, half, ring_alloc,
                       blk, blk + 4, flags);
    err = hipGetLastError();
  }
  if (err != hipSuccess) return err;
  if (pass == 3) flags |= 2u;  // the wave-reach pass writes level rows only
  if (a.nh || (flags & 2u)) {
    // 8 workgroups of 4 waves per CU, a multiple of the 8 XCDs
    const uint32_t grid2 = 8u * std::max<uint32_t>(1u, std::min<uint32_t>((a.n + 8u * kNhlWaves - 1u) / (8u * kNhlWaves),
                                                                           (uint32_t)num_cus));
    note_launch("nh_from_levels_kernel");
    hipLaunchKernelGGL(nh_from_levels_kernel, dim3(grid2), dim3(64 * kNhlWaves), 0, s, g, a, cost, blk + 4, flags);
    err = hipGetLastError();
  }
  return err;
}

}  // namespace openr_spf
