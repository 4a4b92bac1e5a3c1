// spf_bfs_lvl.hip — uniform-cost SPF kernel, "lvl" family: exact level bytes in LDS.
//
// Same semantics as spf_bfs.hip (LinkState::runSpf closed form for uniform cost,
// /root/reference/openr/decision/LinkState.cpp:808-882): dist = c * level, next hops =
// OR over tight in-edges. Chosen for DEEP graphs (grids: ~150 levels of ~70 nodes): the
// per-solve LDS holds lvl[v] (u8) and the packed next-hop sets, and the u64 distance
// row is written coalesced from lvl at the end — the code family's per-node scattered
// distance stores cost more than they save there (G100: 1.42 vs 1.19 ms).
//
// Level L: an arrival on edge u->v is tight iff lvl[v] > L; it ORs nh(u) into nh(v)
// and stores lvl[v] = L+1. The arrival whose atomicOr finds v's (single-dword) set empty
// appends v (every reached node's set is non-empty); sliced classes (> 32 neighbours,
// one 32-bit slice of the set per workgroup pass) elect by a visited bitmap instead.
// One 256-thread workgroup per solve, persistent and dynamically scheduled; K=4 edges
// per lane with their LDS reads, then their atomics, issued together.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;
using namespace bfs;

template <typename LT>
struct LvlLayout {
  uint32_t lvl, vis, nh, ring, ign, dummy, total;
};

// ring = frontier queue (power of two, wraps) in the fast path, or the full BFS-order
// array (capacity V, never wraps) in the fallback path.
template <typename LT>
__host__ __device__ inline LvlLayout<LT> lvl_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t nh_words,
                                                    bool need_vis, uint32_t ring_cap) {
  LvlLayout<LT> l;
  uint32_t off = 32;  // control: append counters [0..3], overflow flag [4]
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.lvl = take((uint32_t)sizeof(LT) * (V + 4u));
  l.vis = need_vis ? take(4u * ((V + 31u) / 32u)) : 0u;
  l.nh = take(4u * nh_words);
  l.ring = take(2u * ring_cap);
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.dummy = take(4u * 64u);  // per-lane sink for the no-op atomics of non-tight edges
  l.total = off;
  return l;
}

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

int lvl_class_mode(int cls) {
  switch (cls) {
    case kLvl4: return kNhNibble;
    case kLvl8: return kNhByte;
    case kLvl16: return kNhHalf;
    default: return kNhW1;  // kLvl32, and each 32-bit slice of kLvlSliced
  }
}

// The distance part of a solve's rows from its levels: u64 distances (level x cost,
// UINT64_MAX unreached) or, when SolveArgs::lvl_rows is set, the levels themselves (u8 / u16,
// all ones unreached: the compact form a strong-scaling rank all-gathers),
// coalesced. Lanes t, t + stride, ... of the writing group.
template <typename LT>
__device__ __forceinline__ void store_dist_row(const SolveArgs& a, uint32_t sid, uint32_t V, const LT* lvl,
                                               uint64_t cost, bool nt, uint32_t t, uint32_t stride) {
  constexpr uint32_t kUnset = LvlOps<LT>::kUnset;
  const size_t row = out_row_of(a, sid);
  if (a.lvl_rows) {
    if (a.lvl_bytes == 1) {
      uint8_t* lrow = a.lvl_rows + row * V;
      if (sizeof(LT) == 1 && ((reinterpret_cast<uintptr_t>(lrow) | V) & 3u) == 0) {
        const uint32_t* l4 = reinterpret_cast<const uint32_t*>(lvl);  // four u8 levels per dword, as stored
        uint32_t* o4 = reinterpret_cast<uint32_t*>(lrow);
        for (uint32_t i = t; i < V / 4u; i += stride) store_row<uint32_t>(&o4[i], l4[i], nt);
      } else {
        bool over = false;
        for (uint32_t v = t; v < V; v += stride) {
          const uint32_t l = lvl[v];
          const bool big = l != kUnset && l > 0xFEu;
          over |= big;
          lrow[v] = (uint8_t)(l == kUnset ? 0xFFu : big ? 0xFEu : l);
        }
        if (over) atomicOr(a.status, kStatusLevelOverflow);
      }
    } else {
      uint16_t* lrow = reinterpret_cast<uint16_t*>(a.lvl_rows) + row * V;
      for (uint32_t v = t; v < V; v += stride) {
        const uint32_t l = lvl[v];
        lrow[v] = (uint16_t)(l == kUnset ? 0xFFFFu : l);
      }
    }
    return;
  }
  uint64_t* drow = a.dist + row * V;
  if (((reinterpret_cast<uintptr_t>(drow) & 15u) | (V & 1u)) == 0) {
    // two nodes per lane: 16-byte stores
    ulonglong2* d2 = reinterpret_cast<ulonglong2*>(drow);
    for (uint32_t i = t; i < V / 2u; i += stride) {
      const uint32_t l0 = lvl[2u * i], l1 = lvl[2u * i + 1u];
      const uint64_t x0 = l0 != kUnset ? (uint64_t)l0 * cost : ~0ull;
      const uint64_t x1 = l1 != kUnset ? (uint64_t)l1 * cost : ~0ull;
      if (nt) {
        __builtin_nontemporal_store(x0, &d2[i].x);
        __builtin_nontemporal_store(x1, &d2[i].y);
      } else {
        d2[i] = make_ulonglong2(x0, x1);
      }
    }
  } else {
    for (uint32_t v = t; v < V; v += stride) {
      const uint32_t l = lvl[v];
      store_row<uint64_t>(&drow[v], l != kUnset ? (uint64_t)l * cost : ~0ull, nt);
    }
  }
}

// Writes this solve's dist row (u64, or level row) and next-hop row from LDS, coalesced.
// Sliced classes: slice s owns next-hop bytes [4s, 4s + 4); slice 0 also writes the
// distance row and zero-fills the bytes past the last slice.
template <int MODE, typename LT, int BLOCK, bool SLICED>
__device__ __forceinline__ void write_rows(const SolveArgs& a, uint32_t sid, uint32_t slice, uint32_t V,
                                           const LT* lvl, const uint32_t* nh, uint64_t cost, bool nt) {
  using N = Nh<MODE>;
  const uint32_t tid = threadIdx.x;
  if (SLICED) {
    if (a.nh) {
      const uint32_t nb = a.nh_bytes, j0 = 4u * slice, zero0 = 4u * a.nsl;
      uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
      for (uint32_t v = tid; v < V; v += BLOCK) {
        const uint32_t w = nh[v];
        uint8_t* o = nrow + (size_t)v * nb;
#pragma unroll
        for (uint32_t jj = 0; jj < 4u; ++jj)
          if (j0 + jj < nb) o[j0 + jj] = (uint8_t)(w >> (8u * jj));
        if (slice == 0)
          for (uint32_t j = zero0; j < nb; ++j) o[j] = 0;
      }
    }
    if (slice != 0) return;
  }
  store_dist_row<LT>(a, sid, V, lvl, cost, nt, tid, (uint32_t)BLOCK);
  if (SLICED || !a.nh) return;
  const uint32_t nb = a.nh_bytes;
  uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
  const bool aligned4 = ((reinterpret_cast<uintptr_t>(nrow) | V) & 3u) == 0;
  if (MODE == kNhNibble && nb == 1 && aligned4) {
    // four nodes (four nibbles of one half-dword) per lane -> one u32 of four bytes
    uint32_t* nrow32 = reinterpret_cast<uint32_t*>(nrow);
    for (uint32_t i = tid; i < V / 4u; i += BLOCK) {
      const uint32_t h = (nh[i >> 1] >> ((i & 1u) * 16u)) & 0xFFFFu;
      store_row<uint32_t>(&nrow32[i], (h & 0xFu) | ((h & 0xF0u) << 4) | ((h & 0xF00u) << 8) | ((h & 0xF000u) << 12),
                          nt);
    }
  } else if (MODE == kNhByte && nb == 1 && aligned4) {
    uint32_t* nrow32 = reinterpret_cast<uint32_t*>(nrow);
    for (uint32_t i = tid; i < V / 4u; i += BLOCK) store_row<uint32_t>(&nrow32[i], nh[i], nt);
  } else {
    const uint32_t total = V * nb;
    for (uint32_t i = tid; i < total; i += BLOCK) {
      const uint32_t v = i / nb, j = i - v * nb;
      nrow[i] = (uint8_t)N::byte(nh, v, j);
    }
  }
}

// ELLM: 0 = CSR rows only; 1 = the first 4 edges of a row from one 16-byte ELL load,
// the rest from CSR (G == 1); 2 = ELL only (every row has <= 4 edges, no ignore set,
// no tight-edge output).
// RING = true : LT = u8, queue = power-of-two ring; a (solve, slice) unit whose two
//               adjacent levels exceed the ring, or whose depth exceeds 253, is appended
//               to a.ovf_list (count *ovf_count).
// RING = false: LT = u16, full BFS order (never overflows). from_list != 0: the units of
//               a.ovf_list only (the re-run of what the ring variant flagged).
// SLICED: one unit = (solve, 32-bit slice of the next-hop set).
// GENERIC = false: no ignore set and no tight-edge output (compile time).
template <int MODE, int BLOCK, typename LT, bool RING, int ELLM, bool GENERIC, bool SLICED>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void bfs_lvl_kernel(
    DevGraph g, SolveArgs a, uint64_t cost, uint32_t glog, uint32_t has_ign_rt, uint32_t ring_cap, uint32_t from_list,
    uint32_t* ctr, uint32_t* ovf_count, uint32_t flags) {
  constexpr int K = (int)kBfsEdgesPerLane;
  const uint32_t nt = flags & 1u;
  const bool fresh_lvl = (flags & 2u) != 0;  // level stored by the appending arrival only
  constexpr bool ELECT = Nh<MODE>::kSingle && !SLICED;
  const bool has_ign = GENERIC && has_ign_rt != 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t s_next;
  using N = Nh<MODE>;
  using O = LvlOps<LT>;
  const uint32_t V = g.V, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = __lane_id();
  const uint32_t nh_words = N::words(V);
  const LvlLayout<LT> lay = lvl_layout<LT>(V, g.L, has_ign, nh_words, !ELECT, ring_cap);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  LT* lvl = reinterpret_cast<LT*>(base + lay.lvl);
  uint32_t* lvl_w = reinterpret_cast<uint32_t*>(base + lay.lvl);
  uint32_t* vis = reinterpret_cast<uint32_t*>(base + lay.vis);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint16_t* ring = reinterpret_cast<uint16_t*>(base + lay.ring);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  uint32_t* dummy = reinterpret_cast<uint32_t*>(base + lay.dummy);
  const uint32_t bit_words = (V + 31u) / 32u;
  const uint32_t lvl_words = ((uint32_t)sizeof(LT) * (V + 4u)) / 4u;
  const uint32_t ign_words = (g.L + 31u) / 32u;
  const uint32_t G = 1u << glog, ngroups = BLOCK >> glog, groups_per_wave = 64u >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  const uint32_t tight_words = (g.E + 63u) / 64u;
  const uint32_t rmask = ring_cap - 1u;  // RING: ring_cap is a power of two
  const uint32_t nsl = SLICED ? a.nsl : 1u;
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  // a re-run launch with nothing flagged does no work
  const uint32_t units = from_list ? *ovf_count : count * nsl;
  // nothing flagged: every workgroup leaves at once (no unit is taken, so the scheduling
  // counters stay at rest and no workgroup needs to retire; saves the 256 retire atomics)
  if (from_list && units == 0u) return;
#ifdef OPENR_SPF_PROFILE
  // [0] load (ring + ELL/row), [1] level reads, [2] atomics, [3] append, [4] barrier,
  // [5] init + level 0, [6] write rows, [7] passes, [8] levels, [9] solves
  uint64_t pc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
#endif

  for (uint32_t unit = blockIdx.x; unit < units;) {
    const uint32_t uid = from_list ? a.ovf_list[unit] : unit;  // class-local (solve, slice) index
    const uint32_t k = SLICED ? uid / nsl : uid, slice = SLICED ? uid - k * nsl : 0u;
    const uint32_t sid = a.perm ? a.perm[first + k] : k;
    const uint32_t src = a.sources[sid];
    if (src < V) {  // block-uniform
      OPENR_PROF_STAMP(t0);
      for (uint32_t i = tid; i < lvl_words; i += BLOCK) lvl_w[i] = 0xFFFFFFFFu;
      if (!ELECT)
        for (uint32_t i = tid; i < bit_words; i += BLOCK) vis[i] = 0;
      for (uint32_t i = tid; i < nh_words; i += BLOCK) nh[i] = 0;
      if (has_ign)
        for (uint32_t i = tid; i < ign_words; i += BLOCK) ign[i] = 0;
      if (tid < 8) ctl[tid] = 0;
      __syncthreads();
      if (has_ign) load_ignore(ign, ign_words, a, sid, g.L);
      if (tid == 0) {
        lvl[src] = 0;
        lvl[V] = 0;  // ELL sentinel (ellv): level 0 is never > L, so a sentinel slot is never tight
        if (!ELECT) vis[src >> 5] = 1u << (src & 31u);
      }
      __syncthreads();
      uint64_t* trow = (GENERIC && a.tight) ? a.tight + out_row_of(a, sid) * tight_words : nullptr;

      // level 0: expand the source (even when overloaded); a directly connected
      // node's next hop is the node itself (LinkState.cpp:867-872)
      {
        const uint2 rs = g.row2[src];
        for (uint32_t e0 = rs.x; e0 < rs.y; e0 += BLOCK) {
          const uint32_t e = e0 + tid;
          bool fresh = false;
          uint32_t v = 0;
          if (e < rs.y) {
            const uint32_t av = g.adj[e];
            v = av & ~kEdgeDown;
            if (!(av & kEdgeDown) && !(has_ign && test_bit(ign, g.lid[e])) && v != src) {
              if constexpr (ELECT) {
                fresh = N::fetch_or_bit(nh, v, g.nbr[e]) == 0u;
              } else {
                const uint32_t bit = 1u << (v & 31u);
                fresh = !(atomicOr(&vis[v >> 5], bit) & bit);
                const uint32_t b = g.nbr[e];
                if (!SLICED) N::or_bit(nh, v, b);
                else if ((b >> 5) == slice) N::or_bit(nh, v, b & 31u);
              }
              lvl[v] = (LT)1;
              if (trow) atomicOr(reinterpret_cast<unsigned long long*>(&trow[e >> 6]), 1ull << (e & 63u));
            }
          }
          // level-0 appends count in ctl[0]; level L >= 1 uses ctl[L & 3]
          const uint32_t slot = 1u + wave_append(fresh, &ctl[0]);
          if (fresh) ring[slot] = (uint16_t)v;  // slot < 1 + deg(src) <= ring_cap checked by the host
        }
      }
      __syncthreads();
#ifdef OPENR_SPF_PROFILE
      OPENR_PROF_STAMP(t1);
      OPENR_PROF_ADD(5, t0, t1);
      pc[9] += 1;
#endif

      uint32_t head = 1, tail = 1u + ctl[0], L = 1;
      bool overflow = false;  // block-uniform
      while (head < tail) {
        if (RING && L + 1u >= O::kUnset) {  // next level not representable in u8
          overflow = true;
          break;
        }
        uint32_t* cnt = &ctl[L & 3u];
        if (tid == 0) ctl[(L + 1u) & 3u] = 0;  // last read three barriers ago
        for (uint32_t fb = head; fb < tail; fb += ngroups) {
          if (fb + wave * groups_per_wave >= tail) continue;  // this wave has no slice (uniform)
          OPENR_PROF_STAMP(t0);
          const uint32_t idx = fb + group;
          const bool live = idx < tail;
          uint32_t u = 0, beg = 0, end = 0;
          uint4 ell = ELLM == 2 ? make_uint4(V, V, V, V) : make_uint4(kEdgeDown, kEdgeDown, kEdgeDown, kEdgeDown);
          if (live) {
            u = ring[RING ? (idx & rmask) : idx];
            if (ELLM == 2) {
              ell = g.ellv[u];  // down / padding / sink-row slots hold the sentinel V
            } else {
              const uint2 r = g.row2t[u];  // empty (begin flagged) for overloaded nodes (sinks)
              beg = r.x;
              end = r.y;
              if (ELLM == 1) ell = g.ellt[u];
            }
          }
          const typename N::Val nhu = N::load(nh, u);  // final: u was reached a level ago
#ifdef OPENR_SPF_PROFILE
          OPENR_PROF_STAMP(t1);
          OPENR_PROF_ADD(0, t0, t1);
          pc[7] += 1;
#endif
          // ELL-only: one pass over the 4 slots (a lane with no frontier node holds the
          // sentinel row, which is never tight)
          for (uint32_t e0 = (ELLM == 2 ? 0u : beg) + lane_g; ELLM == 2 ? e0 == 0u : __any(e0 < end); e0 += G * K) {
            uint32_t av[K], lv[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j * G;
              if (ELLM == 2) {
                av[j] = j == 0 ? ell.x : j == 1 ? ell.y : j == 2 ? ell.z : ell.w;
              } else if (ELLM == 1 && e0 == beg) {
                av[j] = j == 0 ? ell.x : j == 1 ? ell.y : j == 2 ? ell.z : ell.w;
              } else {
                av[j] = e < end ? g.adj[e] : kEdgeDown;
              }
              lv[j] = (has_ign && e < end) ? g.lid[e] : 0u;
            }
#ifdef OPENR_SPF_PROFILE
            OPENR_PROF_STAMP(t1);
#endif
            // (1) tight test: the K level reads are issued together (no branches)
            bool tight[K];
            uint32_t vv[K], lold[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j * G;
              if (ELLM == 2) {  // ellv: a node id or the sentinel V (lvl[V] == 0); ELLM 2 is never GENERIC
                vv[j] = av[j];
                lold[j] = lvl[vv[j]];
                tight[j] = lold[j] > L;
                continue;
              }
              vv[j] = av[j] & ~(kEdgeDown | kNodeSink);  // always a valid node id
              const bool ok = !(av[j] & kEdgeDown) && e < end && !(has_ign && test_bit(ign, lv[j]));
              const uint32_t l = lvl[ok ? vv[j] : V];  // lvl[V] is padding (0: never tight)
              tight[j] = ok && l > L;  // first or equal-cost arrival (LinkState.cpp:857-873)
            }
#ifdef OPENR_SPF_PROFILE
            OPENR_PROF_STAMP(t2);
            OPENR_PROF_ADD(1, t1, t2);
#endif
            // (2) addNextHops(nh(u)) + election of the appending arrival: K atomics in
            //     flight together; non-tight edges OR 0 into the lane's own dummy word
            bool fresh[K];  // this arrival appends v (kept as lane masks: ballots read them directly)
            if constexpr (ELECT) {
              const uint32_t x = nhu.x;
              uint32_t old[K];
#pragma unroll
              for (int j = 0; j < K; ++j)
                old[j] = atomicOr(tight[j] ? &nh[N::word(vv[j])] : &dummy[lane], tight[j] ? x << N::shift(vv[j]) : 0u);
#pragma unroll
              for (int j = 0; j < K; ++j)
                fresh[j] = tight[j] && ((old[j] >> N::shift(vv[j])) & N::kMask) == 0u;
            } else {
              uint32_t old[K];
#pragma unroll
              for (int j = 0; j < K; ++j)
                old[j] = atomicOr(tight[j] ? &vis[vv[j] >> 5] : &dummy[lane], tight[j] ? 1u << (vv[j] & 31u) : 0u);
#pragma unroll
              for (int j = 0; j < K; ++j) {
                fresh[j] = tight[j] && !((old[j] >> (vv[j] & 31u)) & 1u);
                if (tight[j]) N::or_val(nh, vv[j], nhu);
              }
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
              // ELL-only path: store unconditionally (no branch). A non-tight v has a level
              // <= L that no arrival of this level changes, so writing it back is race-free.
              if (!fresh_lvl) {
                if (ELLM == 2) lvl[vv[j]] = (LT)(tight[j] ? L + 1u : lold[j]);
                else if (tight[j]) lvl[vv[j]] = (LT)(L + 1u);
              }
              if (trow && tight[j]) {
                const uint32_t e = e0 + j * G;
                atomicOr(reinterpret_cast<unsigned long long*>(&trow[e >> 6]), 1ull << (e & 63u));
              }
            }
#ifdef OPENR_SPF_PROFILE
            OPENR_PROF_STAMP(t3);
            OPENR_PROF_ADD(2, t2, t3);
#endif
            // (3) wave-aggregated append: one ballot per edge slot j, one ds_add per wave;
            //     arrival (lane, j) takes slot base + (fresh arrivals of slots < j) +
            //     (fresh arrivals of slot j in lower lanes)
            unsigned long long bj[K];
            uint32_t off[K + 1];
            off[0] = 0;
#pragma unroll
            for (int j = 0; j < K; ++j) {
              bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
              off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
            }
            const uint32_t total = off[K];
            if (total) {  // wave-uniform
              const int leader = __ffsll((long long)__ballot(1)) - 1;
              uint32_t wbase = 0;
              if ((int)lane == leader) wbase = atomicAdd(cnt, total);
              const uint32_t base = tail + __builtin_amdgcn_readfirstlane(wbase);
              // the wave's slots are [base, base + total): one wave-uniform test tells
              // whether all of them fit the ring (two adjacent levels); if not, the
              // solve is flagged and re-run, so none of them needs storing
              if (!RING || base + total - head <= ring_cap) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                  if (fresh[j]) {
                    const uint32_t slot = base + off[j] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                    ring[RING ? (slot & rmask) : slot] = (uint16_t)vv[j];
                    // fresh_lvl: only the appending arrival stores v's level. Another
                    // arrival of this level that reads lvl[v] before the store sees
                    // "unset" (> L), i.e. tight, which is what v's level L+1 reads too.
                    if (fresh_lvl) lvl[vv[j]] = (LT)(L + 1u);
                  }
                }
              } else if ((int)lane == leader) {
                ctl[4] = 1;  // two adjacent levels exceed the ring
              }
            }
#ifdef OPENR_SPF_PROFILE
            OPENR_PROF_STAMP(t4);
            OPENR_PROF_ADD(3, t3, t4);
#endif
          }
        }
#ifdef OPENR_SPF_PROFILE
        OPENR_PROF_STAMP(t0);
#endif
        lds_barrier();
#ifdef OPENR_SPF_PROFILE
        OPENR_PROF_STAMP(t1);
        OPENR_PROF_ADD(4, t0, t1);
        pc[8] += 1;
#endif
        head = tail;
        tail += *cnt;
        ++L;
        if (RING && ctl[4]) {  // ring overflow; ctl[4] is uniform after the barrier
          overflow = true;
          break;
        }
        // every node is reached: no edge out of level [head, tail) can be tight (its
        // heads have levels <= L), and the level's levels / next hops are final
        if (tail == V) break;
      }
      if (RING && overflow) {  // re-run by the full-order variant (from the list)
        if (tid == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = uid;
      } else {
#ifdef OPENR_SPF_PROFILE
        OPENR_PROF_STAMP(t0);
#endif
        write_rows<MODE, LT, BLOCK, SLICED>(a, sid, slice, V, lvl, nh, cost, nt != 0);
#ifdef OPENR_SPF_PROFILE
        OPENR_PROF_STAMP(t1);
        OPENR_PROF_ADD(6, t0, t1);
#endif
      }
    }
    // next unit: dynamic scheduling (the first gridDim.x units are static)
    __syncthreads();  // every lane is done with this unit's LDS and s_next
    if (tid == 0) s_next = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = s_next;
  }
  // the re-run consumed the flags of its class: its last workgroup clears the count
  retire_workgroup(ctr, (!RING && from_list) ? ovf_count : nullptr);
#ifdef OPENR_SPF_PROFILE
  if (lane == 0 && a.prof)
    for (int i = 0; i < 10; ++i) atomicAdd(&a.prof[i], (unsigned long long)pc[i]);
#endif
}

// ---------------------------------------------------------------------------
// Lean level pass (the grid configuration): every transit row fits the 4 ELL slots, no
// ignore set, no tight-edge output, one next-hop field per node inside one dword, u8
// levels. Same semantics as bfs_lvl_kernel<MODE, *, u8, true, 2, false, false>
// (LinkState::runSpf closed form for uniform cost, LinkState.cpp:808-882); the pass is
// restated so that an edge slot costs ~11 vector instructions instead of ~30:
//  * LDS is addressed through address-space-3 pointers: the level array sits at the
//    constant byte offset 32, folded into the ds instruction;
//  * a lane whose edge is not tight ORs its value into its own dummy word, which is all
//    ones, so "first arrival" is one test of the returned field for every slot (a dummy
//    field is never zero), and that test's compare mask is the slot's ballot;
//  * the frontier queue is two halves of ring_cap / 2 entries, level L in half L & 1, so
//    an append slot is base + mbcnt (no wrap mask); a level wider than a half flags the
//    solve for the u16 full-order re-run of bfs_lvl_kernel, as a deeper-than-253 solve;
//  * lanes past the frontier read the sentinel row ellv[V] (every slot V, lvl[V] = 0:
//    never tight), so the pass has no divergent prologue.
// ---------------------------------------------------------------------------
struct LeanLayout {
  uint32_t nh, ring, dummy, total;
};
// [0, 32) control, [32, 32 + V + 4) u8 levels, next-hop words, two queue halves, dummies
__host__ __device__ inline LeanLayout lean_layout(uint32_t V, uint32_t nh_words, uint32_t ring_cap) {
  LeanLayout l;
  uint32_t off = 32u + ((V + 4u + 15u) & ~15u);
  l.nh = off;
  off += (4u * nh_words + 15u) & ~15u;
  l.ring = off;
  off += (2u * ring_cap + 15u) & ~15u;
  l.dummy = off;
  off += 4u * 64u;
  l.total = off;
  return l;
}

// DELTA: the transit rows are read as four signed byte deltas (DevGraph::elld, 4 bytes per
// node instead of the 16-byte ellv row: G100's rows in 40 KB instead of 160 KB, so they stay
// in the CU's L1); a zero delta (no edge, down link, overloaded row) and a lane past the
// level resolve to a node whose level is <= L, never tight.
// WPE: the waves-per-SIMD target the compiler allocates registers for. LDS caps G100 at
// 10 workgroups of 2 waves per CU (5 per SIMD), and 5 is the default since round 6.
template <int MODE, int BLOCK, bool PROF, bool DELTA, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void bfs_ell_kernel(
    DevGraph g, SolveArgs a, uint64_t cost, uint32_t ring_cap, uint32_t* ctr, uint32_t* ovf_count, uint32_t nt,
    unsigned long long* prof) {
  using N = Nh<MODE>;
  static_assert(N::kSingle, "single-dword next-hop fields only");
  constexpr uint32_t kBits = 32u / N::kPer;
  constexpr uint32_t kLog = kBits == 4 ? 3 : kBits == 8 ? 2 : kBits == 16 ? 1 : 0;  // log2 nodes per dword
  constexpr uint32_t kShl = 5u - kLog;  // field shift = v << kShl (low 5 bits used by v_lshlrev / v_bfe)
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar loop bounds)
  const uint32_t nh_words = N::words(V);
  const LeanLayout lay = lean_layout(V, nh_words, ring_cap);
  lds_u32* const ctl = (lds_u32*)(size_t)0u;  // [0..3] append counters, [4] overflow flag, [7] next unit
  lds_u8* const lvl = (lds_u8*)(size_t)32u;
  lds_u32* const lvl_w = (lds_u32*)(size_t)32u;
  lds_u32* const nh = (lds_u32*)(size_t)lay.nh;
  lds_u16* const ring = (lds_u16*)(size_t)lay.ring;
  lds_u32* const my_dummy = (lds_u32*)(size_t)(lay.dummy + 4u * lane);
  // generic views for the shared row writer
  const uint8_t* lvl_g = reinterpret_cast<const uint8_t*>(reinterpret_cast<char*>(smem) + 32);
  const uint32_t* nh_g = reinterpret_cast<const uint32_t*>(reinterpret_cast<char*>(smem) + lay.nh);
  const uint32_t lvl_words = (V + 4u) / 4u;
  const uint32_t half = ring_cap / 2u;
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  *my_dummy = 0xFFFFFFFFu;  // only ever ORed afterwards: its fields are never zero
  // tuning (OPENR_SPF_PROF): wave 0's cycles per phase of its first pass of every
  // level: [0] barrier -> queue entry, [1] ELL row load, [2] level / set reads, [3] atomics,
  // [4] append, [5] drain + barrier, [6] levels, [7] solves. A stamp follows an asm use of
  // the value the phase waits for, so it is taken once that value has arrived.
  const bool pf = PROF && prof != nullptr && wave == 0;
  unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long ts = 0;
#define OPENR_LEAN_STAMP(i, dep)                             \
  do {                                                       \
    if (pf) {                                                \
      asm volatile("" ::"v"(dep));                           \
      const long long t = (long long)__builtin_amdgcn_s_memtime(); \
      pacc[i] += (unsigned long long)(t - ts);               \
      ts = t;                                                \
    }                                                        \
  } while (0)

  for (uint32_t unit = blockIdx.x; unit < count;) {
    const uint32_t sid = a.perm ? a.perm[first + unit] : unit;
    const uint32_t src = a.sources[sid];
    if (src < V) {  // block-uniform
      for (uint32_t i = tid; i < lvl_words; i += BLOCK) lvl_w[i] = 0xFFFFFFFFu;
      for (uint32_t i = tid; i < nh_words; i += BLOCK) nh[i] = 0;
      if (tid < 5) ctl[tid] = 0;
      __syncthreads();
      if (tid == 0) {
        lvl[src] = 0;
        lvl[V] = 0;  // ELL sentinel: level 0 is never > L, so a sentinel slot is never tight
      }
      __syncthreads();
      // level 0: the source expands even when overloaded; a directly connected node's
      // next hop is the node itself (LinkState.cpp:867-872). Level 1 goes to half 1.
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
              const uint32_t sh = (v << kShl) & 31u;
              fresh = ((lds_or(&nh[v >> kLog], (1u << g.nbr[e]) << sh) >> sh) & N::kMask) == 0u;
              lvl[v] = 1;
            }
          }
          const uint32_t slot = wave_append(fresh, reinterpret_cast<uint32_t*>(smem) + 1);
          if (fresh) ring[half + slot] = (uint16_t)v;  // slot < deg(src) <= half (host-checked)
        }
      }
      __syncthreads();

      uint32_t cur = __builtin_amdgcn_readfirstlane(ctl[1]), L = 1, reached = 1u + cur;
      bool overflow = false;  // block-uniform
      if (pf) {
        ts = (long long)__builtin_amdgcn_s_memtime();
        pacc[7] += 1;
      }
      // one lane per frontier node, its K = 4 ELL slots; NPP nodes per wave pass
      // (4 lanes per node, one slot each, measured no faster on strong-scaling shards:
      // the level then waits for every wave's shorter chain at the barrier instead)
      constexpr uint32_t K = 4u, NPP = 64u, NPB = (uint32_t)BLOCK;
      const uint32_t lnode = lane;
      uint32_t q = ring[half + wave * NPP + lnode];  // first pass's queue entry of level 1
      while (cur) {
        if (L + 1u >= 0xFFu) {  // next level not representable in u8
          overflow = true;
          break;
        }
        // level L: entries [0, cur) of half L & 1; level L+1 appends to the other half,
        // counted in ctl[(L + 1) & 3] (zeroed here: last read three barriers ago); bit 31
        // of that count flags a level that outgrew its half
        lds_u32* const cnt = &ctl[(L + 1u) & 3u];
        if (tid == 0) ctl[(L + 2u) & 3u] = 0;
        const uint32_t rd = (L & 1u) * half, wr = half - rd;
        const uint8_t lnext = (uint8_t)(L + 1u);
        for (uint32_t fb = wave * NPP; fb < cur; fb += NPB) {
          const uint32_t idx = fb + lnode;
          if (fb != wave * NPP) q = ring[rd + idx];  // the first pass's entry was read with the count
          const uint32_t u = idx < cur ? q : V;  // past the level: the sentinel row
          const bool st = pf && fb == 0u;        // stamps: wave 0's first pass of the level
          if (st) OPENR_LEAN_STAMP(0, u);
          uint32_t vv[K];
          if constexpr (DELTA) {
            const bool live = idx < cur;
            const uint32_t d4 = g.elld[live ? u : 0u];
            const uint32_t dd = live ? d4 : 0u;  // past the level: every slot is the sentinel V
#pragma unroll
            for (uint32_t j = 0; j < K; ++j) vv[j] = u + (uint32_t)__builtin_amdgcn_sbfe((int32_t)dd, 8u * j, 8u);
          } else {
            const uint4 ell = g.ellv[u];  // ellv[V] = sentinel row
            vv[0] = ell.x;
            vv[1] = ell.y;
            vv[2] = ell.z;
            vv[3] = ell.w;
          }
          if (st) OPENR_LEAN_STAMP(1, vv[0]);
          const uint32_t x = __builtin_amdgcn_ubfe(nh[u >> kLog], u << kShl, kBits);  // final since L-1
          // the level reads issue together, then the atomics
          uint32_t lv[K], old[K];
#pragma unroll
          for (uint32_t j = 0; j < K; ++j) lv[j] = lvl[vv[j]];
          if (st) OPENR_LEAN_STAMP(2, lv[0] + x);
#pragma unroll
          for (uint32_t j = 0; j < K; ++j) {
            const uint32_t v = vv[j];
            const bool tight = lv[j] > L;  // first or equal-cost arrival (LinkState.cpp:857-873)
            old[j] = lds_or(tight ? &nh[v >> kLog] : my_dummy, x << ((v << kShl) & 31u));
          }
          __builtin_amdgcn_sched_barrier(0);  // all atomics in flight before their results are used
          if (st) OPENR_LEAN_STAMP(3, old[0]);
          unsigned long long bj[K];
          bool fresh[K];
          uint32_t off[K + 1];
          off[0] = 0;
#pragma unroll
          for (uint32_t j = 0; j < K; ++j) {
            // v's field was empty: this is the first arrival (a dummy field never is)
            fresh[j] = __builtin_amdgcn_ubfe(old[j], vv[j] << kShl, kBits) == 0u;
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
                  // only the appending arrival stores v's level; another arrival of this
                  // level that reads it earlier sees "unset" (> L), i.e. tight, as it is
                  lvl[vv[j]] = lnext;
                }
              }
            } else if (lane == leader) {
              lds_or(cnt, 0x80000000u);  // the level outgrows its half
            }
          }
          if (st) OPENR_LEAN_STAMP(4, total);
        }
        lds_barrier();
        // the next level's count and its first pass's queue entry, read together
        const uint32_t c = __builtin_amdgcn_readfirstlane(*cnt);
        q = ring[wr + wave * NPP + lnode];
        if (pf) {
          OPENR_LEAN_STAMP(5, c);
          pacc[6] += 1;
        }
        ++L;
        if (c >> 31) {  // uniform after the barrier
          overflow = true;
          break;
        }
        cur = c;
        reached += cur;
        if (reached == V) break;  // every node reached: the newest level cannot expand tightly
      }
      if (overflow) {
        if (tid == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = unit;
      } else {
        write_rows<MODE, uint8_t, BLOCK, false>(a, sid, 0, V, lvl_g, nh_g, cost, nt != 0);
      }
    }
    __syncthreads();  // every lane is done with this unit's LDS and ctl[7]
    if (tid == 0) ctl[7] = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = ctl[7];
  }
#undef OPENR_LEAN_STAMP
  if (pf && lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&prof[i], pacc[i]);
  retire_workgroup(ctr, nullptr);
}

// Occupancy first (target workgroups per CU, 8 by default): the full-order u16 variant
// when it fits the per-workgroup budget, else the u8 ring when a ring wide enough for the
// estimated two-level frontier fits and the estimated depth stays under the u8 limit;
// then lower occupancy.
struct LvlShape {
  uint32_t ring_cap = 0, per_cu = 1;  // ring_cap == 0: full order
};
LvlShape lvl_shape(const DevGraph& g, bool has_ign, int mode, bool vis, uint32_t target) {
  LvlShape sh;
  const uint32_t nw = nh_words_for(mode, g.V);
  const uint32_t fixed = lvl_layout<uint8_t>(g.V, g.L, has_ign, nw, vis, 0).total;
  const uint32_t full = lvl_layout<uint16_t>(g.V, g.L, has_ign, nw, vis, g.V).total;
  const uint32_t need = std::max<uint32_t>(std::max<uint32_t>(256u, g.max_deg + 2u), g.est_width2 + g.est_width2 / 4u);
  const bool ring_ok = !env_u32("OPENR_SPF_BFS_FULL", 0u, 0u, 1u) && g.est_depth + 8u < LvlOps<uint8_t>::kUnset;
  for (uint32_t want = target; want >= 1; --want) {
    const uint32_t budget = kMaxLds / want;
    sh.per_cu = want;
    if (full <= budget) {
      sh.ring_cap = 0;
      break;
    }
    if (!ring_ok || budget <= fixed) continue;
    uint32_t cap = 1;
    while (cap * 2u <= (budget - fixed) / 2u && cap < 8192u) cap *= 2u;
    if (cap >= need) {
      sh.ring_cap = cap;
      break;
    }
  }
  // test hook: force a (too small) ring so the overflow -> re-run-list path runs
  const uint32_t forced = env_u32("OPENR_SPF_RING_CAP", 0u, 0u, 65536u);
  if (forced && (forced & (forced - 1u)) == 0u && forced >= g.max_deg + 2u &&
      fixed + 2u * forced <= kMaxLds / sh.per_cu)
    sh.ring_cap = forced;
  return sh;
}

template <int MODE, int BLOCK, typename LT, bool RING, int ELLM, bool SLICED>
hipError_t launch_lvl_variant(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                              uint32_t ring_cap, bool from_list, uint32_t* ctr, uint32_t* ovf_count, int num_cus,
                              hipStream_t s, LaunchInfo* info) {
  const bool vis = SLICED || !Nh<MODE>::kSingle;
  const uint32_t lds = lvl_layout<LT>(g.V, g.L, has_ign, nh_words_for(MODE, g.V), vis, ring_cap).total;
  // a re-run covers only the listed units (usually none): one workgroup per CU is plenty
  const uint32_t grid = from_list ? std::min<uint32_t>(blocks_for(a.n * (SLICED ? a.nsl : 1u), lds, num_cus, BLOCK),
                                                       (uint32_t)num_cus)
                                  : blocks_for(a.n * (SLICED ? a.nsl : 1u), lds, num_cus, BLOCK);
  const bool generic = has_ign || a.tight != nullptr;
  auto k = generic ? bfs_lvl_kernel<MODE, BLOCK, LT, RING, ELLM == 2 ? 1 : ELLM, true, SLICED>
                   : bfs_lvl_kernel<MODE, BLOCK, LT, RING, ELLM, false, SLICED>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  if (info && !from_list) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = RING ? "bfs_lvl_kernel<ring,u8>" : "bfs_lvl_kernel<full,u16>";
  }
  const uint32_t flags = nt_stores() | (1u << 1);
  note_launch(RING ? "bfs_lvl_kernel<ring,u8>" : from_list ? "bfs_lvl_kernel<full,u16>:rerun" : "bfs_lvl_kernel<full,u16>");
  hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), lds, s, g, a, cost, glog, (uint32_t)has_ign, ring_cap,
                     (uint32_t)from_list, ctr, ovf_count, flags);
  return hipGetLastError();
}

template <int MODE, int BLOCK>
hipError_t launch_lvl_lean(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t ring_cap, uint32_t* ctr,
                           uint32_t* ovf_count, int num_cus, hipStream_t s, LaunchInfo* info) {
  const uint32_t lds = lean_layout(g.V, nh_words_for(MODE, g.V), ring_cap).total;
  uint32_t grid = blocks_for(a.n, lds, num_cus, BLOCK);
  const bool want_prof = prof_enabled();
  // OPENR_SPF_LEAN_DELTA=0: 16-byte ellv rows even when the delta rows exist
  const bool delta = g.elld && env_u32("OPENR_SPF_LEAN_DELTA", 1u, 0u, 1u) != 0;
  // registers for 5 waves per SIMD, the occupancy LDS allows G100 (10 workgroups of 2 waves
  // per CU): 89 VGPRs, no scratch, 31 SGPR spills; a target of 8 spilled 21 VGPRs to
  // scratch and 50 SGPRs (r06, interleaved A/B: 0.707 vs 0.715 ms median)
  auto k = want_prof ? (delta ? bfs_ell_kernel<MODE, BLOCK, true, true, 5> : bfs_ell_kernel<MODE, BLOCK, true, false, 5>)
                     : (delta ? bfs_ell_kernel<MODE, BLOCK, false, true, 5> : bfs_ell_kernel<MODE, BLOCK, false, false, 5>);
  hipError_t err =
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = delta ? "bfs_ell_kernel<halves,u8,delta>" : "bfs_ell_kernel<halves,u8>";
  }
  // tuning aid: per-phase cycle sums of the level loop, printed after the launch
  static unsigned long long* prof_buf = nullptr;
  unsigned long long* prof = nullptr;
  if (want_prof) {
    if (!prof_buf && hipMalloc(&prof_buf, 8 * sizeof(unsigned long long)) != hipSuccess) prof_buf = nullptr;
    prof = prof_buf;
    if (prof) (void)hipMemsetAsync(prof, 0, 8 * sizeof(unsigned long long), s);
  }
  note_launch("bfs_ell_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), lds, s, g, a, cost, ring_cap, ctr, ovf_count, nt_stores(), prof);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && prof) {
    unsigned long long h[8];
    if (hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess) {
      const double lv = h[6] ? (double)h[6] : 1.0;
      std::fprintf(stderr,
                   "bfs_ell: block=%d grid=%u n=%u solves=%llu levels/solve=%.1f | cycles/level: entry %.0f row %.0f "
                   "reads %.0f atomics %.0f append %.0f barrier %.0f\n",
                   BLOCK, grid, a.n, h[7], h[7] ? lv / (double)h[7] : 0.0, h[0] / lv, h[1] / lv, h[2] / lv, h[3] / lv,
                   h[4] / lv, h[5] / lv);
    }
  }
  return e;
}

// ---------------------------------------------------------------------------
// Wave pass (graph in LDS): the lean pass with ONE wavefront per solve and the transit
// rows staged in LDS. When every row has <= 4 edges and every neighbour id lies within
// 127 of its row's node (a row-major grid: +-1, +-n), a row is four signed byte deltas
// (`elld`, 4 bytes per node: a 100 x 100 grid in 40 KB), so one workgroup per CU stages
// the whole graph once and its W wavefronts each own a solve slot [u8 levels | next-hop
// words | two queue halves]. A solve's level loop then reads no global memory and has no
// barrier: a wavefront's LDS operations complete in issue order, so the next level reads
// the previous level's appends directly, and the append cursor is a scalar. Per level the
// dependent chain is queue entry -> delta row + nh(u) -> levels -> atomics (four LDS round
// trips, no L2 load, no ds_add, no s_barrier). Semantics as bfs_ell_kernel (closed form of
// LinkState::runSpf for uniform cost, LinkState.cpp:808-882): a delta of 0 (no edge) or a
// lane past the frontier resolves to a node whose level is <= L, never tight. A level
// wider than a half or a solve deeper than 253 levels is listed for the u16 re-run.
// ---------------------------------------------------------------------------
struct WaveLayout {
  uint32_t dummy, slot0, nh, q, per_slot, total;
};
// [0, 4V) delta rows, 64 all-ones dummy words, then W solve slots
__host__ __device__ inline WaveLayout wave_layout(uint32_t V, uint32_t nh_words, uint32_t qhalf, uint32_t waves) {
  WaveLayout l;
  l.dummy = (4u * V + 15u) & ~15u;
  l.slot0 = l.dummy + 256u;
  l.nh = (V + 15u) & ~15u;  // within a slot: levels at 0
  l.q = l.nh + ((4u * nh_words + 15u) & ~15u);
  l.per_slot = l.q + ((4u * qhalf + 15u) & ~15u);
  l.total = l.slot0 + waves * l.per_slot;
  return l;
}

// A wave-pass solve's rows out (lanes t, t + stride, ...): u64 distances (or level rows)
// from the slot's u8 levels at LDS byte `slot` (`lvl8`: the same bytes through smem), then the next-hop bytes.
template <int MODE>
__device__ __forceinline__ void wave_rows_out(const SolveArgs& a, uint32_t sid, uint32_t V, uint32_t slot,
                                              const uint8_t* lvl8, const lds_u32* nh, uint64_t cost, bool nt, uint32_t t,
                                              uint32_t stride) {
  using N = Nh<MODE>;
  constexpr uint32_t kBits = 32u / N::kPer;
  constexpr uint32_t kLog = kBits == 4 ? 3 : kBits == 8 ? 2 : kBits == 16 ? 1 : 0;
  constexpr uint32_t kShl = 5u - kLog;
  const lds_u32* const lvl_w = (const lds_u32*)(size_t)slot;
  uint64_t* drow = a.dist ? a.dist + out_row_of(a, sid) * V : nullptr;
  if (!a.lvl_rows && ((reinterpret_cast<uintptr_t>(drow) & 15u) | (V & 3u)) == 0) {
    ulonglong2* d2 = reinterpret_cast<ulonglong2*>(drow);
    for (uint32_t i = t; i < V / 4u; i += stride) {
      const uint32_t w = lvl_w[i];
      uint64_t xd[4];
#pragma unroll
      for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t l = (w >> (8u * k)) & 0xFFu;
        xd[k] = l != 0xFFu ? (uint64_t)l * cost : ~0ull;
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
    store_dist_row<uint8_t>(a, sid, V, lvl8, cost, nt, t, stride);
  }
  if (!a.nh) return;
  const uint32_t nb = a.nh_bytes;
  uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
  const bool aligned4 = ((reinterpret_cast<uintptr_t>(nrow) | V) & 3u) == 0;
  if (MODE == kNhNibble && nb == 1 && aligned4) {
    uint32_t* nrow32 = reinterpret_cast<uint32_t*>(nrow);
    for (uint32_t i = t; i < V / 4u; i += stride) {
      const uint32_t h = (nh[i >> 1] >> ((i & 1u) * 16u)) & 0xFFFFu;
      store_row<uint32_t>(&nrow32[i], (h & 0xFu) | ((h & 0xF0u) << 4) | ((h & 0xF00u) << 8) | ((h & 0xF000u) << 12),
                          nt);
    }
  } else if (MODE == kNhByte && nb == 1 && aligned4) {
    uint32_t* nrow32 = reinterpret_cast<uint32_t*>(nrow);
    for (uint32_t i = t; i < V / 4u; i += stride) store_row<uint32_t>(&nrow32[i], (uint32_t)nh[i], nt);
  } else {
    for (uint32_t i = t; i < V * nb; i += stride) {
      const uint32_t v = i / nb, j = i - v * nb;
      const uint32_t f = __builtin_amdgcn_ubfe(nh[v >> kLog], v << kShl, kBits);
      nrow[i] = 8u * j < kBits ? (uint8_t)(f >> (8u * j)) : (uint8_t)0;
    }
  }
}

template <int MODE, uint32_t U>
__global__ __launch_bounds__(512) void bfs_wave_kernel(DevGraph g, SolveArgs a, uint64_t cost, uint32_t qhalf,
                                                       uint32_t waves, uint32_t* ctr, uint32_t* ovf_count, uint32_t nt) {
  using N = Nh<MODE>;
  static_assert(N::kSingle, "single-dword next-hop fields only");
  constexpr uint32_t kBits = 32u / N::kPer;
  constexpr uint32_t kLog = kBits == 4 ? 3 : kBits == 8 ? 2 : kBits == 16 ? 1 : 0;
  constexpr uint32_t kShl = 5u - kLog;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nh_words = N::words(V);
  const WaveLayout lay = wave_layout(V, nh_words, qhalf, waves);
  const uint32_t slot = lay.slot0 + wave * lay.per_slot;
  lds_u32* const rows = (lds_u32*)(size_t)0u;
  lds_u8* const lvl = (lds_u8*)(size_t)slot;
  lds_u32* const lvl_w = (lds_u32*)(size_t)slot;
  lds_u32* const nh = (lds_u32*)(size_t)(slot + lay.nh);
  lds_u16* const q = (lds_u16*)(size_t)(slot + lay.q);
  lds_u32* const my_dummy = (lds_u32*)(size_t)(lay.dummy + 4u * lane);
  for (uint32_t i = tid; i < V; i += blockDim.x) rows[i] = g.elld[i];
  if (wave == 0) *my_dummy = 0xFFFFFFFFu;  // only ever ORed afterwards: its fields are never zero
  __syncthreads();
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  const uint32_t lvl_words = (V + 3u) / 4u;
  uint32_t unit = blockIdx.x * waves + wave;  // the first grid x W units are static, then dynamic
  while (unit < count) {
    const uint32_t sid = a.perm ? a.perm[first + unit] : unit;
    const uint32_t src = a.sources[sid];
    if (src < V) {  // wave-uniform
      for (uint32_t i = lane; i < lvl_words; i += 64u) lvl_w[i] = 0xFFFFFFFFu;
      for (uint32_t i = lane; i < nh_words; i += 64u) nh[i] = 0u;
      if (lane == 0) lvl[src] = 0;
      // level 0: the source expands even when overloaded (its full CSR row); a directly
      // connected node's next hop is the node itself (LinkState.cpp:867-872)
      uint32_t cur = 0;
      {
        const uint2 rs = g.row2[src];
        for (uint32_t e0 = rs.x; e0 < rs.y; e0 += 64u) {
          const uint32_t e = e0 + lane;
          bool fresh = false;
          uint32_t v = 0;
          if (e < rs.y) {
            const uint32_t av = g.adj[e];
            v = av & ~kEdgeDown;
            if (!(av & kEdgeDown) && v != src) {
              const uint32_t sh = (v << kShl) & 31u;
              fresh = ((lds_or(&nh[v >> kLog], (1u << g.nbr[e]) << sh) >> sh) & N::kMask) == 0u;
              lvl[v] = 1;
            }
          }
          const unsigned long long b = __builtin_amdgcn_ballot_w64(fresh);
          if (fresh)  // slot < deg(src) < qhalf (host-checked)
            q[qhalf + cur + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] =
                (uint16_t)v;
          cur += (uint32_t)__popcll(b);
        }
      }
      uint32_t L = 1, reached = 1u + cur;
      bool overflow = false;  // wave-uniform
      while (cur) {
        if (L + 1u >= 0xFFu) {  // next level not representable in u8
          overflow = true;
          break;
        }
        const uint32_t rd = (L & 1u) * qhalf, wr = qhalf - rd;
        const uint8_t lnext = (uint8_t)(L + 1u);
        uint32_t nxt = 0;  // scalar append cursor of level L+1
        // U frontier chunks of 64 per step, their dependent chains interleaved (U = 2: a
        // level of 65-128 nodes takes one chain instead of two)
        for (uint32_t fb = 0; fb < cur; fb += 64u * U) {
          constexpr uint32_t S = 4u * U;
          uint32_t vv[S], lv[S], old[S], xu[U];
#pragma unroll
          for (uint32_t h = 0; h < U; ++h) {
            const uint32_t idx = fb + 64u * h + lane;
            const bool live = idx < cur;
            const uint32_t qe = q[rd + (live ? idx : 0u)];
            const uint32_t u = live ? qe : src;             // past the level: the source (level 0)
            const uint32_t r4 = rows[u];                    // issued with the nh(u) read below
            const uint32_t d4 = live ? r4 : 0u;             // no slots: every slot resolves to u
            xu[h] = __builtin_amdgcn_ubfe(nh[u >> kLog], u << kShl, kBits);  // final since L-1
#pragma unroll
            for (uint32_t j = 0; j < 4u; ++j) vv[4u * h + j] = u + (uint32_t)__builtin_amdgcn_sbfe((int32_t)d4, 8u * j, 8u);
          }
#pragma unroll
          for (uint32_t j = 0; j < S; ++j) lv[j] = lvl[vv[j]];
#pragma unroll
          for (uint32_t j = 0; j < S; ++j) {
            const uint32_t v = vv[j];
            const bool tight = lv[j] > L;  // first or equal-cost arrival (LinkState.cpp:857-873)
            old[j] = lds_or(tight ? &nh[v >> kLog] : my_dummy, xu[j / 4u] << ((v << kShl) & 31u));
          }
          __builtin_amdgcn_sched_barrier(0);  // all atomics in flight before their results are used
          unsigned long long bj[S];
          bool fresh[S];
          uint32_t off[S + 1];
          off[0] = 0;
#pragma unroll
          for (uint32_t j = 0; j < S; ++j) {
            fresh[j] = __builtin_amdgcn_ubfe(old[j], vv[j] << kShl, kBits) == 0u;  // a dummy field never is
            bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
            off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
          }
          const uint32_t total = off[S];
          if (total) {  // wave-uniform
            if (nxt + total <= qhalf) {
#pragma unroll
              for (uint32_t j = 0; j < S; ++j) {
                if (fresh[j]) {
                  const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                  q[wr + nxt + off[j] + k] = (uint16_t)vv[j];
                  lvl[vv[j]] = lnext;  // only the appending arrival stores v's level
                }
              }
            } else {
              overflow = true;  // the level outgrows its half
            }
            nxt += total;
          }
        }
        if (overflow) break;
        ++L;
        cur = nxt;
        reached += cur;
        if (reached == V) break;  // every node reached: the newest level cannot expand tightly
      }
      if (overflow) {
        if (lane == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = unit;
      } else {
        wave_rows_out<MODE>(a, sid, V, slot, reinterpret_cast<const uint8_t*>(smem) + slot, nh, cost, nt != 0, lane, 64u);
      }
    }
    uint32_t nx = 0;
    if (lane == 0) nx = gridDim.x * waves + atomicAdd(&ctr[0], 1u);
    unit = __builtin_amdgcn_readfirstlane(nx);
  }
  __syncthreads();  // no wave of this workgroup takes units any more
  retire_workgroup(ctr, nullptr);
}

// Wavefronts per workgroup for the wave pass, 0 when it does not apply. One workgroup per
// CU holds the delta rows plus up to W solve slots (W >= 4 by LDS), spread so every CU
// gets work. Auto (OPENR_SPF_BFS_WAVE unset / 2): batches of at most three rounds of W
// solves per CU — the strong-scaling shards, where a solve's latency is exposed (G100,
// 1 250 sources: 0.165 vs 0.194 ms; 2 500: 0.273 vs 0.313; 5 000: 0.428 vs 0.460) —
// while a full batch stays on the lean pass, whose two-wave workgroups keep 10 solves per
// CU in flight (10 000 sources: 0.750 vs 0.804 ms). 1 = whenever it applies (tests), 0 =
// never.
uint32_t wave_pass_waves(const DevGraph& g, int mode, uint32_t qhalf, uint32_t n, int num_cus) {
  const uint32_t knob = env_u32("OPENR_SPF_BFS_WAVE", 2u, 0u, 2u);
  if (!g.elld || knob == 0u) return 0;
  const WaveLayout one = wave_layout(g.V, nh_words_for(mode, g.V), qhalf, 0);
  if (one.slot0 >= kMaxLds) return 0;
  const uint32_t w = std::min<uint32_t>(8u, (kMaxLds - one.slot0) / one.per_slot);
  if (w < 4u) return 0;  // fewer than 4 solve slots per CU: the lean pass
  const uint64_t cus = (uint64_t)std::max(num_cus, 1);
  if (knob == 2u && (uint64_t)n > 3ull * cus * w) return 0;
  return (uint32_t)std::min<uint64_t>(w, std::max<uint64_t>(1, ((uint64_t)n + cus - 1) / cus));
}

template <int MODE>
hipError_t launch_lvl_wave(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t qhalf, uint32_t waves,
                           uint32_t* ctr, uint32_t* ovf_count, int num_cus, hipStream_t s, LaunchInfo* info) {
  const uint32_t lds = wave_layout(g.V, nh_words_for(MODE, g.V), qhalf, waves).total;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((uint32_t)num_cus, (a.n + waves - 1u) / waves));
  auto k = bfs_wave_kernel<MODE, 1>;
  hipError_t err =
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = "bfs_wave_kernel<lds-graph>";
  }
  note_launch("bfs_wave_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(64u * waves), lds, s, g, a, cost, qhalf, waves, ctr, ovf_count, nt_stores());
  if (prof_enabled())  // tests: which pass ran
    std::fprintf(stderr, "bfs_wave: grid=%u waves=%u n=%u qhalf=%u lds=%u\n", grid, waves, a.n, qhalf, lds);
  return hipGetLastError();
}

template <int MODE, int BLOCK, int ELLM, bool SLICED>
hipError_t launch_lvl_mode(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                           uint32_t ring_cap, int num_cus, hipStream_t s, LaunchInfo* info) {
  // Counter block of the class: [0,1] first launch, [2,3] re-run launch, [4] listed units.
  uint32_t* blk = class_counters(a);
  hipError_t err;
  if constexpr (ELLM == 2 && !SLICED && Nh<MODE>::kSingle) {
    const uint32_t need1 = std::max<uint32_t>(g.max_deg + 1u, g.est_width1 + g.est_width1 / 4u);
    // wave pass (graph in LDS) for small batches when the delta rows fit with >= 4 solve
    // slots per CU (OPENR_SPF_WAVE_QHALF, tests: a smaller half, so wide levels re-run)
    const uint32_t qforce = env_u32("OPENR_SPF_WAVE_QHALF", 0u, 0u, 65535u);
    const uint32_t qhalf = qforce ? (std::max<uint32_t>(qforce, g.max_deg + 1u) + 15u) & ~15u
                                  : (std::max<uint32_t>(64u, need1) + 15u) & ~15u;
    const uint32_t waves = (!has_ign && !a.tight) ? wave_pass_waves(g, MODE, qhalf, a.n, num_cus) : 0u;
    if (waves) {
      err = launch_lvl_wave<MODE>(g, a, cost, qhalf, waves, blk, blk + 4, num_cus, s, info);
      if (err != hipSuccess || (g.V <= qhalf && g.V <= 254u)) return err;  // nothing can overflow
      return launch_lvl_variant<MODE, 256, uint16_t, false, ELLM, SLICED>(g, a, cost, glog, has_ign, g.V, true,
                                                                          blk + 2, blk + 4, num_cus, s, info);
    }
  }
  if (!ring_cap)
    return launch_lvl_variant<MODE, BLOCK, uint16_t, false, ELLM, SLICED>(g, a, cost, glog, has_ign, g.V, false, blk,
                                                                          blk + 4, num_cus, s, info);
  if constexpr (ELLM == 2 && !SLICED && Nh<MODE>::kSingle) {
    // lean pass: its queue halves must hold the widest sampled level (else the generic ring)
    const uint32_t need1 = std::max<uint32_t>(g.max_deg + 1u, g.est_width1 + g.est_width1 / 4u);
    // (OPENR_SPF_LEAN_FORCE=1, tests: also when the halves are too small, so wide levels
    // take the overflow -> u16 re-run path)
    const bool fits = ring_cap / 2u >= need1 || env_u32("OPENR_SPF_LEAN_FORCE", 0u, 0u, 1u) != 0u;
    const bool lean = !has_ign && !a.tight && fits;
    if (lean)
      err = launch_lvl_lean<MODE, BLOCK>(g, a, cost, ring_cap, blk, blk + 4, num_cus, s, info);
    else
      err = launch_lvl_variant<MODE, BLOCK, uint8_t, true, ELLM, SLICED>(g, a, cost, glog, has_ign, ring_cap, false,
                                                                         blk, blk + 4, num_cus, s, info);
  } else {
    err = launch_lvl_variant<MODE, BLOCK, uint8_t, true, ELLM, SLICED>(g, a, cost, glog, has_ign, ring_cap, false,
                                                                       blk, blk + 4, num_cus, s, info);
  }
  if (err != hipSuccess || (g.V <= ring_cap && g.V <= 254u)) return err;  // nothing can overflow
  return launch_lvl_variant<MODE, 256, uint16_t, false, ELLM, SLICED>(g, a, cost, glog, has_ign, g.V, true, blk + 2,
                                                                      blk + 4, num_cus, s, info);
}

template <int MODE, bool SLICED>
hipError_t launch_lvl_ell(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign, int ellm,
                          int num_cus, hipStream_t s, LaunchInfo* info) {
  const bool vis = SLICED || !Nh<MODE>::kSingle;
  const LvlShape sh = lvl_shape(g, has_ign, MODE, vis, kBfsTargetWgs);
  // 128-thread workgroups when the batch fills the GPU several times over (occupancy hides
  // the level loop's latency: G100 0.863 vs 0.913 ms); 256 threads (four waves per solve,
  // a wide level in one pass) when it fills it at most twice, as a strong-scaling shard
  // does (G100 5 000 sources 0.518 vs 0.556 ms, 2 500: 0.357 vs 0.381 ms)
  const bool small_batch = (uint64_t)a.n <= 2ull * (uint64_t)num_cus * sh.per_cu;
  const bool b128 = sh.per_cu > 8u && !small_batch;
#define OPENR_LVL_MODE(BLK, E) \
  return launch_lvl_mode<MODE, BLK, E, SLICED>(g, a, cost, glog, has_ign, sh.ring_cap, num_cus, s, info)
  if (b128) {
    if (ellm == 2) OPENR_LVL_MODE(128, 2);
    if (ellm == 1) OPENR_LVL_MODE(128, 1);
    OPENR_LVL_MODE(128, 0);
  }
  if (ellm == 2) OPENR_LVL_MODE(256, 2);
  if (ellm == 1) OPENR_LVL_MODE(256, 1);
  OPENR_LVL_MODE(256, 0);
#undef OPENR_LVL_MODE
}
}  // namespace

uint32_t bfs_lvl_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int cls) {
  // the full-order u16 variant must fit (it re-runs solves the fast path flags)
  if (V > 65535u || cls < 0 || cls >= kNumLvlClasses) return 0;
  const int mode = lvl_class_mode(cls);
  const bool vis = cls == kLvlSliced || !nh_mode_single(mode);
  const uint32_t t = lvl_layout<uint16_t>(V, L, has_ignore, nh_words_for(mode, V), vis, V).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_bfs_lvl(const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes, int num_cus,
                          hipStream_t s, LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  const int cls = (int)a.cls;
  if (!bfs_lvl_lds_bytes(g.V, g.L, has_ign, cls)) return hipErrorInvalidValue;
  const bool sliced = cls == kLvlSliced;
  if (sliced && (a.nsl < 1u || a.nsl > 8u)) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  if (!a.ovf_list || !a.work) return hipErrorInvalidValue;
  uint32_t glog = 0;
  while ((1 << glog) < group_lanes && glog < 6) ++glog;
  // ELL: one lane per frontier node; ELL-only when every row fits the 4 ELL slots
  const int ellm = glog != 0 ? 0 : (g.max_deg <= 4u ? 2 : 1);
  if (sliced) return launch_lvl_ell<kNhW1, true>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
  switch (lvl_class_mode(cls)) {
    case kNhNibble: return launch_lvl_ell<kNhNibble, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
    case kNhByte: return launch_lvl_ell<kNhByte, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
    case kNhHalf: return launch_lvl_ell<kNhHalf, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
    default: return launch_lvl_ell<kNhW1, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
  }
}

}  // namespace openr_spf
