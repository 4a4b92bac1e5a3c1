// spf_ksp.hip — KSP2 path tracing on the device (LinkState::getKthPaths k = 1, 2).
//
// Reference (/root/reference/openr/decision/LinkState.cpp):
//   getKthPaths(src, dest, k)  :762-791  ignore = links of the paths of every i < k;
//                                        k = 1 uses the memoized SPF, k >= 2 a fresh
//                                        runSpf(src, true, ignore); then traceOnePath is
//                                        repeated with ONE shared visited-link set until
//                                        it fails or returns an empty path.
//   traceOnePath(src, dest, ..):398-419  DFS from dest over pathLinks(dest) in stored
//                                        order; a link is tried only if inserting it
//                                        into the visited set succeeds; the path is
//                                        returned in src -> dest order.
// pathLinks(v) = tight in-edges u->v in the order runSpf added them: by the pop order
// of u, i.e. (dist[u], name of u), then by u's linksFromNode order (= CSR position).
//
// The engine traces from dense distance rows, so tightness is recomputed here:
// u->v is tight iff the edge is up, its link is not ignored, u may expand (u == src
// or not overloaded, LinkState.cpp:831-838) and dist[u] + w(u->v) == dist[v].
//
// Shape: one wavefront per (src, dest) pair. Entering a DFS frame gathers v's live
// pathLinks with all 64 lanes and ranks them into the frame's slice of an LDS arena, so
// each later step of the frame is a few LDS reads. A frame that fails marks its node
// dead for the rest of the pair (trace_one), which bounds a pair's DFS work by the nodes
// it can kill plus the paths it finds. Visited links and dead nodes are LDS bitmaps.
//
// Output tokens per pair (ReadMe: include/openr_spf.h openr_spf_ksp2): [n_paths,
// len_0, edges_0..., len_1, edges_1..., ...], directed edge ids in src -> dest order.
#include <algorithm>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;

constexpr uint32_t kWave = 64;
constexpr uint32_t kKspProbeAfter = 64;   // DFS frame entries of one trace before the reachability probe
                                         // (OPENR_SPF_KSP_PROBE overrides: tests force 0)
constexpr uint64_t kNoKey = ~0ull;
// Optional per-launch counters (OPENR_SPF_PROF=1; tuning only), indices into KspState::stats
enum : uint32_t {
  kStPairs, kStTraces, kStPaths, kStEntries, kStCands, kStProbes, kStProbeNeg, kStCyc, kStCycLoad, kStCycProbe,
  kStProbeNodes, kStSteps, kStCycFail, kStEntFail, kStCycInit, kStCycRank, kKspStats
};

struct KspLayout {
  uint32_t vis, dead, fr_node, fr_edge, fr_beg, fr_cnt, fr_idx, ar_e, ar_l, ar_u, skd, skr, sl, su, seen, stats, d16, total;
};

constexpr uint32_t kD16Budget = 64u * 1024u;  // LDS per wavefront up to which the u16 distance copy is kept

// deg = largest row (candidate scratch of one frame); frames / arena = DFS capacity
// (KspCaps: a small tier sized from the graph's depth for occupancy, and the full tier
// that re-runs the pairs the small one could not hold).
// pack: node ids and link ids below 2^16, an arena entry's tail and link share a word
// (ar_l = link | u << 16, no ar_u): 4 B less per entry, more wavefronts per CU.
__host__ __device__ inline KspLayout ksp_layout(uint32_t V, uint32_t L, uint32_t deg, uint32_t frames, uint32_t arena,
                                                bool want_d16, bool pack, bool stats_on = false) {
  KspLayout l;
  uint32_t off = 16;  // control: [0] candidate count
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.vis = take(4u * ((L + 31u) / 32u));
  l.dead = take(4u * ((V + 31u) / 32u));
  l.fr_node = take(4u * frames);
  l.fr_edge = take(4u * frames);
  l.fr_beg = take(4u * frames);
  l.fr_cnt = take(4u * frames);
  l.fr_idx = take(4u * frames);
  l.ar_e = take(4u * arena);
  l.ar_l = take(4u * arena);
  l.ar_u = pack ? 0u : take(4u * arena);
  // candidate scratch of load_path_links_long only: rows of <= 128 in-edges rank in registers
  const uint32_t sdeg = deg > 2u * kWave ? deg : 0u;
  l.skd = take(8u * sdeg);
  l.skr = take(8u * sdeg);
  l.sl = take(4u * sdeg);
  l.su = take(4u * sdeg);
  l.seen = 0;  // the probe's visited bits live in global scratch after the queue (st.seen)
  l.stats = stats_on ? take(8u * kKspStats) : 0u;  // OPENR_SPF_PROF launches only
  l.d16 = 0;
  if (want_d16 && off + 2u * V + 16u <= kD16Budget) l.d16 = take(2u * V);
  l.total = off;
  return l;
}

// The tracer's workgroup is one wavefront, and a wavefront's LDS instructions execute in
// issue order, so a read issued after another lane's write sees it: between LDS accesses
// of the tracer only the compiler's order must hold (the hardware wait, s_waitcnt
// lgkmcnt(0), stalled every DFS step for nothing). Results in registers get their waits
// from the compiler as usual. OPENR_SPF_KSP_WAIT builds keep the wait (A/B).
#ifdef OPENR_SPF_KSP_WAIT
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#else
// ... and a convergent join (wave_barrier emits no instruction): the lane-0 stores before a
// fence reconverge there, so the compiler does not merge their join into the exits of the
// DFS and pair loops (which would make those exits divergent: per-lane exit masks)
__device__ __forceinline__ void lds_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
#endif

struct KspState {
  const DevGraph* g;
  uint32_t src;
  const uint64_t* drow;
  uint32_t* ctl;
  uint32_t* vis;   // visited links (linksToIgnore of traceOnePath; + the k = 1 links for k = 2)
  uint32_t* dead;  // nodes whose DFS subtree failed: they can never reach src again
  uint32_t *fr_node, *fr_edge, *fr_beg, *fr_cnt, *fr_idx;  // DFS frames
  uint32_t *ar_e, *ar_l, *ar_u;                            // per-frame sorted pathLinks
  bool pack;  // ar_l holds link | u << 16 (ksp_layout)
  uint64_t *skd, *skr;
  uint32_t *sl, *su;  // candidate scratch: link, tail
  uint32_t* seen;  // reachability probe: visited nodes (V bits)
  uint32_t* q;     // reachability probe queue (global, V entries per wavefront)
  uint32_t probe_after;
  uint32_t max_depth, arena_cap;  // DFS frames / arena entries of this launch's tier
  uint64_t* stats;  // LDS counters (lane 0 updates), null unless enabled
  const uint16_t* d16;  // LDS copy of drow saturated at 0xFFFF, valid when use16
  bool use16;
  const uint16_t* l16;  // non-null: the pair's row is u16 levels (0xFFFF unreached), dist = level * lcost
  uint64_t lcost;       // non-zero: every usable edge costs lcost (uniform-cost graph)
  uint32_t ltag, lshift;  // ltag != 0: l16 entries are ltag << lshift | level, other tags unreached
  // k = 1 (round 6): the source's pathLinks as lists (ksp_path_lists_kernel): node v's tight
  // in-edges in rank order are tl_ent[tl_off[v], tl_off[v + 1]) = {u->v edge, link | u << 16}
  const uint32_t* tl_off;
  const uint2* tl_ent;
  // k = 2: the source's base row. Where the pair's second SPF left v's distance as in the
  // base row, v's tight in-edges are a subset of its base list (see load_path_links)
  const uint64_t* tl_brow;
  // k = 2 over repaired rows (ksp_repair_kernel): an entry with another tag is the base
  // distance (this source's base row), level lmask reads as unreached
  const uint64_t* rbrow;
};

// dist[u] of the pair's row. With the LDS copy (dist[dest] < 0xFFFF) a saturated entry
// reads as unreached: such a u has dist[u] > dist[dest] and can never be the tail of a
// pathLink on the way to dest (tight means dist[u] + w == dist[v] <= dist[dest], w >= 1).
__device__ __forceinline__ uint64_t dist_of(const KspState& st, uint32_t u) {
  if (st.use16) {
    const uint32_t d = st.d16[u];
    return d == 0xFFFFu ? kNoKey : (uint64_t)d;
  }
  if (st.l16) {
    if (st.rbrow) {  // both loads in flight together
      const uint32_t l = st.l16[u];
      const uint64_t b = st.rbrow[u];
      if ((l >> st.lshift) != st.ltag) return b;
      const uint32_t m = (1u << st.lshift) - 1u, lev = l & m;
      return lev == m ? kNoKey : (uint64_t)lev * st.lcost;
    }
    const uint32_t l = st.l16[u];
    if (st.ltag) return (l >> st.lshift) != st.ltag ? kNoKey : (uint64_t)(l & ((1u << st.lshift) - 1u)) * st.lcost;
    return l == 0xFFFFu ? kNoKey : (uint64_t)l * st.lcost;
  }
  return st.drow[u];
}

// LDS copy of a distance row (u16, saturated), 8 row loads in flight per lane.
__device__ void copy_row16(uint16_t* d16, const uint64_t* drow, uint32_t V) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t i0 = 0; i0 < V; i0 += 8u * kWave) {
    uint64_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + j * kWave + lane;
      x[j] = i < V ? drow[i] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + j * kWave + lane;
      if (i < V) d16[i] = x[j] < 0xFFFFull ? (uint16_t)x[j] : (uint16_t)0xFFFFu;
    }
  }
}

// LDS copy of a tagged u16 level row (KSP2 second SPF): entries of another tag are
// unreached; distance = level x cost, saturated like copy_row16
__device__ void copy_row16_tagged(uint16_t* d16, const uint16_t* l16, uint32_t V, uint32_t ltag, uint32_t lshift,
                                  uint64_t lcost) {
  const uint32_t lane = threadIdx.x, mask = (1u << lshift) - 1u;
  for (uint32_t i0 = 0; i0 < V; i0 += 8u * kWave) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + j * kWave + lane;
      x[j] = i < V ? l16[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = i0 + j * kWave + lane;
      if (i < V) {
        const uint64_t d = (x[j] >> lshift) == ltag ? (uint64_t)(x[j] & mask) * lcost : 0xFFFFull;
        d16[i] = d < 0xFFFFull ? (uint16_t)d : (uint16_t)0xFFFFu;
      }
    }
  }
}

__device__ __forceinline__ void stat_add(const KspState& st, uint32_t i, uint64_t v) {
  if (st.stats) {
    if (threadIdx.x == 0) st.stats[i] += v;
    __builtin_amdgcn_wave_barrier();  // the lane-0 branch joins here, not at a caller's return or latch
  }
}

// pathLinks(v) still worth trying -> arena[beg, beg + count) as (edge u->v, link, u):
// tight in-edges (edge up, u may expand, dist[u] + w(u->v) == dist[v]) whose link is
// unvisited and whose tail is not dead, in the reference's order (dist[u], name rank of
// u, position in u's row). UINT32_MAX when the arena is full.
//
// Rows of up to 128 in-edges (every benchmark topology) are ranked from registers: each
// lane holds the keys of in-edges lane and lane + 64, and counts the smaller keys by
// walking the candidate ballot with v_readlane (no LDS round trips; keys are distinct).
// Longer rows go through an LDS append + counting rank (load_path_links_long).
struct PathCand {
  bool ok;
  uint64_t kd, kr;  // (dist[u]) and (name rank of u << 32 | u->v edge)
  uint32_t link, u;
};

__device__ __forceinline__ PathCand gather_cand(const KspState& st, uint32_t e, uint32_t end, uint64_t dv) {
  PathCand c{false, 0, 0, 0, 0};
  if (e < end) {
    const uint4 rec = st.g->erec[e];  // v->u: {u | flags, w(u->v), link, rev = u->v}
    const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
    if (!(rec.x & kEdgeDown) && !test_bit(st.vis, rec.z) && !test_bit(st.dead, u) &&
        (u == st.src || !(rec.x & kNodeSink))) {
      const uint64_t du = dist_of(st, u);
      const uint32_t rk = st.g->rank[u];
      c.ok = du != kNoKey && du + rec.y == dv;
      c.kd = du;
      c.kr = ((uint64_t)rk << 32) | rec.w;
      c.link = rec.z;
      c.u = u;
    }
  }
  return c;
}

// Uniform cost (round 3): every tight candidate of v has dist[u] = dist[v] - cost, so the
// reference's order is (name rank of u, edge) alone, which DevGraph::erecs holds each row
// in: a candidate's rank is the number of candidates before it in the row (mbcnt of the
// ballot), with no key exchange and no name-rank load.
__device__ __forceinline__ PathCand gather_cand_sorted(const KspState& st, uint32_t e, uint32_t end, uint64_t dv) {
  PathCand c{false, 0, 0, 0, 0};
  if (e < end) {
    const uint4 rec = st.g->erecs[e];
    const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
    if (!(rec.x & kEdgeDown) && !test_bit(st.vis, rec.z) && !test_bit(st.dead, u) &&
        (u == st.src || !(rec.x & kNodeSink))) {
      const uint64_t du = dist_of(st, u);
      c.ok = du != kNoKey && du + rec.y == dv;
      c.kr = rec.w;
      c.link = rec.z;
      c.u = u;
    }
  }
  return c;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t j) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)j);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t key_less(uint64_t od, uint64_t orr, const PathCand& c) {
  return (od < c.kd || (od == c.kd && orr < c.kr)) ? 1u : 0u;
}

// rank of c.kd/kr among the candidates of ballot m held by (kd, kr) registers
__device__ __forceinline__ void rank_against(uint64_t m, const PathCand& src, const PathCand& a, const PathCand& b,
                                             uint32_t& ra, uint32_t& rb, bool kr_only) {
  if (kr_only) {  // uniform cost: every candidate has dist[u] = dist[v] - cost, so kd ties
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      const uint64_t orr = readlane64(src.kr, j);
      ra += orr < a.kr ? 1u : 0u;
      rb += orr < b.kr ? 1u : 0u;
    }
    return;
  }
  while (m) {
    const uint32_t j = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    const uint64_t od = readlane64(src.kd, j), orr = readlane64(src.kr, j);
    ra += key_less(od, orr, a);
    rb += key_less(od, orr, b);
  }
}

__device__ uint32_t load_path_links_long(const KspState& st, uint32_t v, uint32_t beg);

// pathLinks(v) from the source's lists: the tight in-edges are already filtered and in
// rank order, so a frame reads its list (one offset pair, then the entries) and keeps the
// ones whose link is unvisited and whose tail is not dead, at their ballot positions
// (no record rows, no distance reads)
// CHECK (k = 2): 1, an entry also needs dist[u] + cost == dv in the pair's own row; 2 (the
// row repairs the base row, ksp_repair_kernel), u must be unaffected — no entry of this
// row's tag — since v is, and u is one of v's base pathLinks.
template <int CHECK>
__device__ uint32_t load_path_links_tl(const KspState& st, uint32_t beg, uint32_t b, uint32_t n, uint64_t dv) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = st.stats ? clock64() : 0;
  uint32_t cnt = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += kWave) {
    const uint32_t i = i0 + lane;
    bool ok = false;
    uint2 t = make_uint2(0u, 0u);
    if (i < n) {
      t = st.tl_ent[b + i];
      ok = !test_bit(st.vis, t.y & 0xFFFFu) && !test_bit(st.dead, t.y >> 16);
      if (CHECK == 1 && ok) {
        const uint64_t du = dist_of(st, t.y >> 16);
        ok = du != kNoKey && du + st.lcost == dv;
      }
      if (CHECK == 2 && ok) ok = (uint32_t)(st.l16[t.y >> 16] >> st.lshift) != st.ltag;
    }
    const uint64_t m = __ballot(ok);
    const uint32_t r = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    cnt += (uint32_t)__popcll(m);
    if (beg + cnt > st.arena_cap) return UINT32_MAX;
    if (ok) {
      st.ar_e[beg + r] = t.x;
      st.ar_l[beg + r] = t.y;
    }
  }
  lds_fence();
  if (st.stats) {
    const uint64_t t2 = clock64();
    stat_add(st, kStEntries, 1);
    stat_add(st, kStCands, cnt);
    stat_add(st, kStCycLoad, t2 - t0);
  }
  return cnt;
}

__device__ uint32_t load_path_links(const KspState& st, uint32_t v, uint32_t beg) {
  if (st.tl_off) {
    const uint32_t b = st.tl_off[v], n = st.tl_off[v + 1u] - b;
    if (!st.tl_brow) return load_path_links_tl<0>(st, beg, b, n, 0);  // k = 1: the base row's own lists
    if (st.rbrow) {
      // repaired row (ksp_repair_kernel): v keeps its base distance iff the row holds no
      // entry of its tag for v
      if ((uint32_t)(st.l16[v] >> st.lshift) != st.ltag) return load_path_links_tl<2>(st, beg, b, n, 0);
    } else {
      // k = 2 (uniform cost c): if the second SPF left dist[v] as in the base row, every
      // tight in-edge u->v of the pair's row is in v's base list: dist2[u] = dist2[v] - c =
      // dist1[v] - c, and dist1[u] <= dist2[u] (ignoring links only lengthens) while
      // dist1[u] >= dist1[v] - c (u is v's neighbour in the base graph too), so dist1[u] =
      // dist1[v] - c. The list keeps rank order; the pair's own level test filters it.
      const uint64_t dv = dist_of(st, v);
      if (dv == st.tl_brow[v]) return load_path_links_tl<1>(st, beg, b, n, dv);
    }
  }
  const uint2 r = st.g->row2[v];
  if (r.y - r.x > 2u * kWave) return load_path_links_long(st, v, beg);
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = st.stats ? clock64() : 0;
  const uint64_t dv = dist_of(st, v);
  const bool sorted = st.lcost != 0u && st.g->erecs != nullptr;  // wave-uniform
  const PathCand c0 = sorted ? gather_cand_sorted(st, r.x + lane, r.y, dv) : gather_cand(st, r.x + lane, r.y, dv);
  const PathCand c1 = sorted ? gather_cand_sorted(st, r.x + kWave + lane, r.y, dv)
                             : gather_cand(st, r.x + kWave + lane, r.y, dv);
  const uint64_t m0 = __ballot(c0.ok), m1 = __ballot(c1.ok);
  const uint64_t t1 = st.stats ? clock64() : 0;
  const uint32_t cnt = (uint32_t)(__popcll(m0) + __popcll(m1));
  if (beg + cnt > st.arena_cap) return UINT32_MAX;
  uint32_t r0 = 0, r1 = 0;
  if (sorted) {  // row order is key order: the rank is the position among the candidates
    r0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
    r1 = (uint32_t)__popcll(m0) +
         __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
  } else {
    rank_against(m0, c0, c0, c1, r0, r1, st.lcost != 0u);
    rank_against(m1, c1, c0, c1, r0, r1, st.lcost != 0u);
  }
  if (c0.ok) {
    st.ar_e[beg + r0] = (uint32_t)c0.kr;
    if (st.pack) {
      st.ar_l[beg + r0] = c0.link | (c0.u << 16);
    } else {
      st.ar_l[beg + r0] = c0.link;
      st.ar_u[beg + r0] = c0.u;
    }
  }
  if (c1.ok) {
    st.ar_e[beg + r1] = (uint32_t)c1.kr;
    if (st.pack) {
      st.ar_l[beg + r1] = c1.link | (c1.u << 16);
    } else {
      st.ar_l[beg + r1] = c1.link;
      st.ar_u[beg + r1] = c1.u;
    }
  }
  lds_fence();
  if (st.stats) {
    const uint64_t t2 = clock64();
    stat_add(st, kStEntries, 1);
    stat_add(st, kStCands, cnt);
    stat_add(st, kStCycLoad, t2 - t0);
    stat_add(st, kStCycRank, t2 - t1);
  }
  return cnt;
}

// Rows longer than 128 in-edges: wave-aggregated LDS append per 64 in-edges, ranked by
// counting over the LDS copy of the keys.
__device__ uint32_t load_path_links_long(const KspState& st, uint32_t v, uint32_t beg) {
  const DevGraph& g = *st.g;
  const uint32_t lane = threadIdx.x;
  const uint64_t dv = dist_of(st, v);
  const uint2 r = g.row2[v];
  const uint64_t t0 = st.stats ? clock64() : 0;
  if (lane == 0) st.ctl[0] = 0;
  lds_fence();
  for (uint32_t e0 = r.x; e0 < r.y; e0 += kWave) {
    const uint32_t e = e0 + lane;
    bool cand = false;
    uint64_t du = 0;
    uint32_t u = 0, rk = 0;
    uint4 rec = make_uint4(kEdgeDown, 0u, 0u, 0u);
    if (e < r.y) {
      rec = g.erec[e];  // v->u: {u | flags, w(u->v), link, rev = u->v}
      u = rec.x & ~(kEdgeDown | kNodeSink);
      if (!(rec.x & kEdgeDown) && !test_bit(st.vis, rec.z) && !test_bit(st.dead, u) &&
          (u == st.src || !(rec.x & kNodeSink))) {
        du = dist_of(st, u);
        rk = g.rank[u];
        cand = du != kNoKey && du + rec.y == dv;
      }
    }
    const uint32_t slot = wave_append(cand, &st.ctl[0]);
    if (cand) {
      st.skd[slot] = du;
      st.skr[slot] = ((uint64_t)rk << 32) | rec.w;
      st.sl[slot] = rec.z;
      st.su[slot] = u;
    }
  }
  lds_fence();
  const uint64_t t1 = st.stats ? clock64() : 0;
  const uint32_t cnt = __builtin_amdgcn_readfirstlane(st.ctl[0]);
  if (beg + cnt > st.arena_cap) return UINT32_MAX;
  for (uint32_t i = lane; i < cnt; i += kWave) {
    const uint64_t kd = st.skd[i], kr = st.skr[i];
    uint32_t rank = 0;
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint64_t od = st.skd[j], orr = st.skr[j];
      rank += (od < kd || (od == kd && orr < kr)) ? 1u : 0u;
    }
    st.ar_e[beg + rank] = (uint32_t)kr;  // re
    if (st.pack) {
      st.ar_l[beg + rank] = st.sl[i] | (st.su[i] << 16);
    } else {
      st.ar_l[beg + rank] = st.sl[i];
      st.ar_u[beg + rank] = st.su[i];
    }
  }
  lds_fence();
  if (st.stats) {
    stat_add(st, kStEntries, 1);
    stat_add(st, kStCands, cnt);
    const uint64_t t2 = clock64();
    stat_add(st, kStCycLoad, t2 - t0);
    stat_add(st, kStCycRank, t2 - t1);
  }
  return cnt;
}

// Will the running DFS still find a path? It keeps the prefix dest -> ... -> x on its
// stack and, after deeper frames fail, tries the remaining pathLinks of every stack node
// in turn, each link at most once: it succeeds iff some stack node (or `next`, the node
// it is about to enter) reaches src over live pathLinks (unvisited link, tail not dead).
// Checked by a backward BFS over the tight DAG from those seeds, one lane per frontier
// node (its in-edges in a sequential loop, 4 loads in flight), queue in global scratch
// (an edge-parallel variant — rows flattened by a wave scan — measured slower: the
// binary search per edge costs more than the idle lanes of short frontiers).
// A negative answer ends the trace (and the pair's traces) without the rest of the DFS.
// Wave-uniform result.
__device__ bool reachable(const KspState& st, uint32_t sp, uint32_t next) {
  const DevGraph& g = *st.g;
  const uint32_t lane = threadIdx.x, vw = (g.V + 31u) / 32u;
  const uint64_t t0 = st.stats ? clock64() : 0;
  for (uint32_t i = lane; i < vw; i += kWave) st.seen[i] = 0;
  __threadfence_block();  // the bits are global scratch (the probe is rare; LDS buys waves)
  if (lane == 0) {
    uint32_t t = 0;
    for (uint32_t i = 0; i <= sp; ++i) {
      const uint32_t x = i < sp ? st.fr_node[i] : next;
      const uint32_t bit = 1u << (x & 31u);
      if (!(atomicOr(&st.seen[x >> 5], bit) & bit)) st.q[t++] = x;
    }
    st.ctl[1] = t;
  }
  lds_fence();
  __threadfence_block();
  uint32_t head = 0, tail = __builtin_amdgcn_readfirstlane(st.ctl[1]);
  bool found = false;
  while (head < tail && !found) {
    const uint32_t i = head + lane;
    bool hit = false;
    if (i < tail) {
      const uint32_t v = st.q[i];
      const uint64_t dv = dist_of(st, v);
      const uint2 r = g.row2[v];
      for (uint32_t e0 = r.x; e0 < r.y && !hit; e0 += 4u) {
        uint4 rec[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) rec[j] = e0 + j < r.y ? g.erec[e0 + j] : make_uint4(kEdgeDown, 0u, 0u, 0u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t u = rec[j].x & ~(kEdgeDown | kNodeSink);
          if ((rec[j].x & kEdgeDown) || test_bit(st.vis, rec[j].z) || test_bit(st.dead, u)) continue;
          if (u != st.src && (rec[j].x & kNodeSink)) continue;
          const uint64_t du = dist_of(st, u);
          if (du == kNoKey || du + rec[j].y != dv) continue;
          if (u == st.src) {
            hit = true;
            break;
          }
          const uint32_t bit = 1u << (u & 31u);
          if (!(atomicOr(&st.seen[u >> 5], bit) & bit)) st.q[atomicAdd(&st.ctl[1], 1u)] = u;
        }
      }
    }
    found = __any(hit);
    __threadfence_block();
    lds_fence();
    head = std::min(tail, head + kWave);
    tail = __builtin_amdgcn_readfirstlane(st.ctl[1]);
  }
  if (st.stats) {
    stat_add(st, kStProbes, 1);
    stat_add(st, kStProbeNeg, found ? 0 : 1);
    stat_add(st, kStProbeNodes, tail);
    stat_add(st, kStCycProbe, clock64() - t0);
  }
  return found;
}

// Live first links of a path: src -> x tight in the pair's row (link unvisited,
// dist[src] + w(src->x) == dist[x]), x not dead and able to expand (or x == dest). Every
// traced path starts with one of them and the visited / dead sets only grow, so after
// this many more paths the next trace must fail: the pair loop stops without it.
__device__ uint32_t live_src_links(const KspState& st, uint32_t dst) {
  const DevGraph& g = *st.g;
  const uint32_t lane = threadIdx.x;
  const uint2 r = g.row2[st.src];
  const uint64_t ds = dist_of(st, st.src);
  uint32_t n = 0;
  for (uint32_t e0 = r.x; e0 < r.y; e0 += kWave) {
    const uint32_t e = e0 + lane;
    bool live = false;
    if (e < r.y) {
      const uint4 rec = g.erec[e];  // src->x: {x | flags, w(x->src), link, rev}
      const uint32_t x = rec.x & ~(kEdgeDown | kNodeSink);
      // (no edge-up test: the tracer reads x's copy of the flag; counting more is safe)
      if (!test_bit(st.vis, rec.z) && !test_bit(st.dead, x) && (x == dst || !(rec.x & kNodeSink))) {
        const uint64_t dx = dist_of(st, x);
        live = dx != kNoKey && ds + g.w[e] == dx;
      }
    }
    n += (uint32_t)__popcll(__ballot(live));
  }
  return n;
}

// One traceOnePath (LinkState.cpp:398-419): DFS from dest over pathLinks in the
// reference's order, inserting each tried link into the visited set. A frame whose
// candidates are exhausted failed: its node can no longer reach src (the visited set only
// grows), so it is marked dead and never entered again within this pair — the reference
// would re-enter it, skip or fail every candidate again and return nullopt, so the paths
// found are the same. Returns the path length (edges in fr_edge[1..len], dest side
// first), 0 for src == dest, -1 for no path, -2 when the DFS outgrows its frames/arena.
//
// `resume`: the previous trace of this pair found a path, and its dest frame (frame 0,
// arena [0, fr_cnt[0])) is still in place. The reference's next call restarts at dest and
// walks dest's pathLinks from the first: every one before fr_idx[0] was inserted into the
// visited set by the previous calls (or has a dead tail), so it skips them all and goes on
// at fr_idx[0]. The frame resumes there instead of gathering dest's row again; links
// visited and tails killed since the gather are caught by the checks at each pop.
__device__ int trace_one(const KspState& st, uint32_t dst, bool resume) {
  if (st.src == dst) return 0;
  const uint32_t lane = threadIdx.x;
  uint32_t c0, i0 = 0;
  if (resume) {
    c0 = __builtin_amdgcn_readfirstlane(st.fr_cnt[0]);
    i0 = __builtin_amdgcn_readfirstlane(st.fr_idx[0]);
  } else {
    c0 = load_path_links(st, dst, 0);
    if (c0 == UINT32_MAX) return -2;
    if (lane == 0) {
      st.fr_node[0] = dst;
      st.fr_beg[0] = 0;
      st.fr_cnt[0] = c0;
    }
    lds_fence();
  }
  // the top frame's (next index, count, arena begin) live in registers (wave-uniform);
  // fr_idx of a frame is written when a child is pushed over it and read back on the pop
  uint32_t sp = 1, top = c0, entries = 0, fi = i0, fc = c0, fb = 0;
  bool probed = false;
  while (sp > 0) {
    const uint32_t f = sp - 1;
    stat_add(st, kStSteps, 1);
    if (fi >= fc) {  // exhausted: std::nullopt back to the caller frame
      const uint32_t v = st.fr_node[f];
      if (lane == 0) st.dead[v >> 5] |= 1u << (v & 31u);
      top -= fc;
      --sp;
      if (sp) {
        fi = __builtin_amdgcn_readfirstlane(st.fr_idx[sp - 1]);
        fc = __builtin_amdgcn_readfirstlane(st.fr_cnt[sp - 1]);
        fb = __builtin_amdgcn_readfirstlane(st.fr_beg[sp - 1]);
      }
      lds_fence();
      continue;
    }
    const uint32_t idx = fi++;
    const uint32_t al = st.ar_l[fb + idx];
    const uint32_t link = st.pack ? al & 0xFFFFu : al, u = st.pack ? al >> 16 : st.ar_u[fb + idx];
    const bool fresh = !test_bit(st.vis, link);
    const bool live = !test_bit(st.dead, u);
    if (lane == 0 && fresh && live) st.vis[link >> 5] |= 1u << (link & 31u);
    lds_fence();
    if (!fresh || !live) continue;  // insert() failed, or a subtree known to fail
    if (sp >= st.max_depth) return -2;
    const uint32_t re = st.ar_e[fb + idx];
    if (u == st.src) {
      if (lane == 0) {
        st.fr_edge[sp] = re;
        st.fr_idx[f] = fi;  // frame 0's position for a resumed next trace
      }
      lds_fence();
      return (int)sp;
    }
    if (!probed && ++entries > st.probe_after) {  // a long search: is there a path at all?
      probed = true;
      if (!reachable(st, sp, u)) return -1;
    }
    const uint32_t c = load_path_links(st, u, top);
    if (c == UINT32_MAX) return -2;
    if (lane == 0) {
      st.fr_idx[f] = fi;
      st.fr_edge[sp] = re;
      st.fr_node[sp] = u;
      st.fr_beg[sp] = top;
      st.fr_cnt[sp] = c;
    }
    lds_fence();
    fi = 0;
    fc = c;
    fb = top;
    top += c;
    ++sp;
  }
  return -1;
}

// Pairs [first, first + n) of a chunk; k = pair - first. With `list` the launch covers
// only the chunk-local k of list[0 .. *list_count) (the full-tier re-run). With
// `retry_list` (small tier) a pair whose DFS outgrows the tier's frames / arena is
// appended there instead of being marked bad; the full tier re-runs it.
// KIND 1: k = 1 over the base rows (row = prow[pair]); the links of the paths found are
//         written to ign_io[k * ign_cap, ign_end[k]).
// KIND 2: k = 2 over the chunk's rows (row k); those links start out used (the second
//         SPF ignored them, so they are no pathLinks either).
template <int KIND>
__global__ __launch_bounds__(kWave) void ksp_trace_kernel(DevGraph g, const uint32_t* sources, const uint32_t* prow,
                                                          const uint32_t* pdst, uint32_t first, uint32_t n,
                                                          const uint64_t* rows, uint32_t* ign_io, uint32_t* ign_end,
                                                          uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap,
                                                          uint32_t* status, uint32_t* qbuf, uint32_t probe_after,
                                                          uint32_t use_d16, unsigned long long* gstats,
                                                          uint32_t frames, uint32_t arena, const uint32_t* list,
                                                          const uint32_t* list_count, uint32_t* retry_list,
                                                          uint32_t* retry_count, uint32_t* work_ctr,
                                                          const uint16_t* rows16, uint64_t lcost,
                                                          uint32_t ltag, const uint32_t* tl_off,
                                                          const uint2* tl_ent, const uint64_t* tl_rows,
                                                          const uint32_t* rmode) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V;
  const KspLayout lay =
      ksp_layout(V, g.L, g.max_deg, frames, arena, (use_d16 & 1u) != 0, (use_d16 & 8u) != 0, gstats != nullptr);
  const bool resume_ok = (use_d16 & 2u) != 0;  // trace_one may resume dest's frame
  char* base = reinterpret_cast<char*>(smem);
  KspState st;
  st.g = &g;
  st.ctl = smem;
  st.vis = reinterpret_cast<uint32_t*>(base + lay.vis);
  st.dead = reinterpret_cast<uint32_t*>(base + lay.dead);
  st.fr_node = reinterpret_cast<uint32_t*>(base + lay.fr_node);
  st.fr_edge = reinterpret_cast<uint32_t*>(base + lay.fr_edge);
  st.fr_beg = reinterpret_cast<uint32_t*>(base + lay.fr_beg);
  st.fr_cnt = reinterpret_cast<uint32_t*>(base + lay.fr_cnt);
  st.fr_idx = reinterpret_cast<uint32_t*>(base + lay.fr_idx);
  st.ar_e = reinterpret_cast<uint32_t*>(base + lay.ar_e);
  st.ar_l = reinterpret_cast<uint32_t*>(base + lay.ar_l);
  st.ar_u = lay.ar_u ? reinterpret_cast<uint32_t*>(base + lay.ar_u) : nullptr;
  st.pack = (use_d16 & 8u) != 0;
  st.skd = reinterpret_cast<uint64_t*>(base + lay.skd);
  st.skr = reinterpret_cast<uint64_t*>(base + lay.skr);
  st.sl = reinterpret_cast<uint32_t*>(base + lay.sl);
  st.su = reinterpret_cast<uint32_t*>(base + lay.su);
  // per-wavefront global scratch: the probe's queue (V) and its visited bits (vw words)
  st.q = qbuf + (size_t)blockIdx.x * (V + (V + 31u) / 32u);
  st.seen = st.q + V;
  st.probe_after = probe_after;
  st.max_depth = frames;
  st.arena_cap = arena;
  st.stats = gstats ? reinterpret_cast<uint64_t*>(base + lay.stats) : nullptr;
  const uint32_t lane = threadIdx.x, lw = (g.L + 31u) / 32u, vw = (V + 31u) / 32u;
  if (st.stats && lane < kKspStats) st.stats[lane] = 0;
  uint16_t* d16 = lay.d16 ? reinterpret_cast<uint16_t*>(base + lay.d16) : nullptr;
  st.d16 = d16;
  uint32_t d16_row = UINT32_MAX;  // KIND 1: the base row already in d16
  const uint32_t n_units = list ? *list_count : n;
  // dynamic scheduling: pair costs differ by an order of magnitude between destination
  // tiers, so a static stride leaves waves idle; the first gridDim.x units are static
  for (uint32_t unit = blockIdx.x; unit < n_units;
       unit = gridDim.x + __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(work_ctr, 1u) : 0u)) {
    const uint64_t tp = st.stats ? clock64() : 0;
    const uint32_t k = list ? list[unit] : unit;
    const uint32_t pair = first + k;
    const uint32_t row = prow[pair];
    const uint32_t src = sources[row], dst = pdst[pair];
    st.src = src;
    st.drow = rows + (size_t)(KIND == 1 ? row : k) * V;
    st.l16 = (KIND == 2 && rows16) ? rows16 + (size_t)k * V : nullptr;
    st.tl_off = tl_off ? tl_off + (size_t)row * (V + 1u) : nullptr;
    st.tl_ent = tl_off ? tl_ent + (size_t)row * g.E : nullptr;
    st.tl_brow = (KIND == 2 && tl_off) ? tl_rows + (size_t)row * V : nullptr;
    st.rbrow = (KIND == 2 && tl_rows && rmode && rmode[k] == 0u) ? tl_rows + (size_t)row * V : nullptr;
    st.lcost = lcost;
    st.ltag = ltag >> 8;
    st.lshift = ltag & 0xFFu;
    st.use16 = false;
    const uint64_t ddst = dst < V ? dist_of(st, dst) : kNoKey;
    if (d16 && !st.l16 && ddst < 0xFFFFull) {
      if (KIND == 2 || row != d16_row) copy_row16(d16, st.drow, V);
      d16_row = KIND == 1 ? row : UINT32_MAX;
      st.use16 = true;
    }
    uint32_t* out = tok + (size_t)pair * tok_cap;
    uint32_t* ig = ign_io + (size_t)k * ign_cap;  // chunk-local ignore slot
    for (uint32_t i = lane; i < lw; i += kWave) st.vis[i] = 0;
    for (uint32_t i = lane; i < vw; i += kWave) st.dead[i] = 0;
    lds_fence();
    if (KIND == 2) {
      const uint32_t ne = ign_end[k] - k * ign_cap;
      for (uint32_t i = lane; i < ne; i += kWave) {
        const uint32_t l = ig[i];
        atomicOr(&st.vis[l >> 5], 1u << (l & 31u));
      }
      lds_fence();
    }
    uint32_t npaths = 0, pos = 1, nign = 0;
    bool bad = src >= V || dst >= V, retry = false;
    // res.count(dest); src == dest traces an empty path, which ends the loop at once
    stat_add(st, kStPairs, 1);
    if (st.stats) stat_add(st, kStCycInit, clock64() - tp);
    if (!bad && src != dst && ddst != kNoKey) {
      uint32_t src_live = live_src_links(st, dst);
      // a tagged second-SPF row that will be traced: its LDS copy (the trace's distance
      // reads then stay in LDS)
      if (d16 && st.l16 && st.ltag && src_live && ddst < 0xFFFFull) {
        copy_row16_tagged(d16, st.l16, V, st.ltag, st.lshift, st.lcost);
        lds_fence();
        st.use16 = true;
      }
      bool resume = false;  // trace_one: dest's frame kept from the last path found
      while (src_live) {
        const uint64_t tt = st.stats ? clock64() : 0, e0 = st.stats ? st.stats[kStEntries] : 0;
        const int len = trace_one(st, dst, resume);
        if (st.stats) {
          stat_add(st, kStTraces, 1);
          if (len <= 0) {
            stat_add(st, kStCycFail, clock64() - tt);
            stat_add(st, kStEntFail, st.stats[kStEntries] - e0);
          }
        }
        if (len == -2) {  // frames / arena exhausted: the full tier re-runs the pair
          if (retry_list) retry = true;
          else bad = true;
          break;
        }
        if (len <= 0) break;  // while (path && !path->empty())
        if (pos + 1u + (uint32_t)len > tok_cap || (KIND == 1 && nign + (uint32_t)len > ign_cap)) {
          bad = true;
          break;
        }
        for (uint32_t i = lane; i < (uint32_t)len; i += kWave) {
          const uint32_t e = st.fr_edge[(uint32_t)len - i];  // dest side first -> src -> dest
          out[pos + 1u + i] = e;
          if (KIND == 1) ig[nign + i] = g.lid[e];
        }
        if (lane == 0) out[pos] = (uint32_t)len;
        pos += 1u + (uint32_t)len;
        nign += (uint32_t)len;
        ++npaths;
        --src_live;
        resume = resume_ok;
      }
    }
    if (lane == 0) {
      if (retry) {
        retry_list[atomicAdd(retry_count, 1u)] = k;
        if (KIND == 1) ign_end[k] = k * ign_cap;
      } else {
        if (KIND == 1) ign_end[k] = k * ign_cap + (bad ? 0u : nign);
        out[0] = bad ? 0xFFFFFFFFu : npaths;
        if (bad) atomicOr(status, 1u);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the lane-0 branch joins here: the pair loop's latch is uniform
    if (st.stats) {
      stat_add(st, kStPaths, npaths);
      stat_add(st, kStCyc, clock64() - tp);
    }
  }
  if (st.stats) {
    lds_fence();
    if (lane < kKspStats) atomicAdd(&gstats[lane], (unsigned long long)st.stats[lane]);
  }
}

__global__ __launch_bounds__(256) void strided_iota(uint32_t* p, uint32_t n, uint32_t stride) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) p[i] = i * stride;
}

// sources of the second SPF: the pair's source node
__global__ __launch_bounds__(256) void gather_sources(const uint32_t* sources, const uint32_t* prow, uint32_t first,
                                                      uint32_t n, uint32_t* out) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) out[i] = sources[prow[first + i]];
}

// getKthPaths(src, dest, 2) (LinkState.cpp:762-791) is empty without a second SPF when
//  * k = 1 found no path (dest unreached, or src == dest): the ignore set is empty, so
//    k = 2 re-traces the same base result and finds nothing either;
//  * the k = 1 paths use every link of src, or every link of dest: they are edge-disjoint
//    and simple (positive metrics), so each uses a distinct first and a distinct last
//    link, and n_paths == |row| means the whole row is ignored. runSpf(src, true, ignore)
//    then settles src alone, or never dest, and res.count(dest) == 0. (A row holding a
//    self-loop is longer than the links a path can use: such pairs are kept.)
// On the fabric every RSW -> RSW pair (65 % of all pairs) is of the second kind.
// Those pairs get n_paths = 0 here; the rest are appended to `list` for the second SPF
// and the k = 2 trace. A k = 1 row marked bad (0xFFFFFFFF) is kept.
__global__ __launch_bounds__(256) void ksp_select_pairs(DevGraph g, const uint32_t* sources, const uint32_t* prow,
                                                        const uint32_t* pdst, uint32_t first, uint32_t n,
                                                        const uint32_t* tok1, uint32_t* tok2, uint32_t tok_cap,
                                                        uint32_t* out_src, uint32_t* list, uint32_t* count) {
  const uint32_t lane = __lane_id();
  for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {  // block-uniform: whole waves ballot
    const uint32_t k = i0 + threadIdx.x;
    bool keep = false;
    if (k < n) {
      const uint32_t pair = first + k;
      const uint32_t src = sources[prow[pair]], dst = pdst[pair];
      out_src[k] = src;
      const uint32_t np = tok1[(size_t)pair * tok_cap];
      bool empty = np == 0u;
      if (np != 0u && np != 0xFFFFFFFFu && src < g.V && dst < g.V) {
        const uint2 rs = g.row2[src], rd = g.row2[dst];
        empty = np == rs.y - rs.x || np == rd.y - rd.x;
      }
      if (empty) tok2[(size_t)pair * tok_cap] = 0u;
      keep = !empty;
    }
    const uint64_t b = __ballot(keep);
    uint32_t at = 0;
    if (lane == 0 && b) at = atomicAdd(count, (uint32_t)__popcll(b));
    at = __shfl(at, 0);
    if (keep) list[at + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = k;
  }
}

// The k = 1 trace's pathLinks (round 6): per source of the batch, every node's tight
// in-edges over the base row in rank order (DevGraph::erecs order; uniform cost), as the
// reference's SpfResult holds them (LinkState.h:203-260, built in runSpf :867-872). Same
// test as gather_cand_sorted without the pair's visited / dead sets: edge up, tail may
// expand (the source or not overloaded), dist[u] + w(u->v) == dist[v]. One workgroup per
// source: counts into off[1 .. V], an exclusive scan over off, then the entries.
__device__ __forceinline__ bool tl_tight(const DevGraph& g, const uint64_t* drow, uint32_t src, uint4 rec,
                                         uint64_t dv) {
  const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
  if ((rec.x & kEdgeDown) || (u != src && (rec.x & kNodeSink))) return false;
  const uint64_t du = drow[u];
  return du != kNoKey && du + rec.y == dv;
}

__global__ __launch_bounds__(256) void ksp_path_lists_kernel(DevGraph g, const uint32_t* sources, uint32_t n_src,
                                                             const uint64_t* rows, uint32_t* off_all,
                                                             uint2* ent_all) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t carry;
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id(), wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (uint32_t j = blockIdx.x; j < n_src; j += gridDim.x) {
    const uint32_t src = sources[j];
    const uint64_t* drow = rows + (size_t)j * V;
    uint32_t* off = off_all + (size_t)j * (V + 1u);
    uint2* ent = ent_all + (size_t)j * g.E;
    // counts: one wavefront per node, 64 in-edges per step
    for (uint32_t v = wave; v < V; v += 4u) {
      const uint2 r = g.row2[v];
      const uint64_t dv = drow[v];
      uint32_t c = 0;
      for (uint32_t e0 = r.x; e0 < r.y; e0 += 64u) {
        const uint32_t e = e0 + lane;
        c += (uint32_t)__popcll(__ballot(e < r.y && src < V && tl_tight(g, drow, src, g.erecs[e], dv)));
      }
      if (lane == 0) off[v + 1u] = c;
    }
    if (tid == 0) {
      off[0] = 0;
      carry = 0;
    }
    __syncthreads();
    // inclusive scan of off[1 .. V] in 256-entry chunks
    for (uint32_t b = 1; b <= V; b += 256u) {
      const uint32_t i = b + tid;
      uint32_t x = i <= V ? off[i] : 0u;
      for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      if (lane == 63u) wsum[wave] = x;
      __syncthreads();
      uint32_t pre = carry;
      for (uint32_t w = 0; w < wave; ++w) pre += wsum[w];
      if (i <= V) off[i] = x + pre;
      __syncthreads();
      if (tid == 255u) carry = x + pre;
      __syncthreads();
    }
    // entries at their scanned positions, in row order
    for (uint32_t v = wave; v < V; v += 4u) {
      const uint2 r = g.row2[v];
      const uint64_t dv = drow[v];
      uint32_t at = off[v];
      for (uint32_t e0 = r.x; e0 < r.y; e0 += 64u) {
        const uint32_t e = e0 + lane;
        uint4 rec = make_uint4(kEdgeDown, 0u, 0u, 0u);
        bool t = false;
        if (e < r.y && src < V) {
          rec = g.erecs[e];
          t = tl_tight(g, drow, src, rec, dv);
        }
        const uint64_t m = __ballot(t);
        if (t) {
          const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
          ent[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              make_uint2(rec.w, rec.z | (u << 16));
        }
        at += (uint32_t)__popcll(m);
      }
    }
    __syncthreads();  // off / ent of this source done before the next one's counts
  }
}

// ---------------------------------------------------------------------------
// KSP2 second SPF as a repair of the base SPF (round 6). runSpf(src, true, ignore) differs
// from the memoized getSpfResult(src) (LinkState.cpp:776-788) only where every shortest
// path used an ignored link. With uniform cost c and base distances B:
//  * a node is *affected* (its distance grows) iff each of its base pathLinks u->v is
//    ignored or comes from an affected u. Induction on B: an unaffected node keeps a tight
//    in-edge from an unaffected node, so its distance stays; an affected node's every
//    shortest-path predecessor would have to be unaffected and tight, and none is.
//  * the affected set A is the closure of that rule from the ignored links: each node
//    counts its base pathLinks lost (ignored, or from a node found affected) against
//    its list length (the k = 1 lists, ksp_path_lists_kernel) and joins A at zero.
//  * A's new distances: a BFS over A seeded by its unaffected in-neighbours (B[u] + c),
//    in increasing level, until dest's level is settled (dest in A) or up to dest's base
//    level (dest unaffected). Only A is written: tagged level, or `lmask` (no level:
//    unreached, or not needed — at or beyond dest). The k = 2 trace reads every other
//    node's distance from the base row (dist_of with KspState::rbrow).
// On the fabric A is a few nodes to one plane (~120 nodes) where the forward solve
// expanded 11 k - 74 k edges per pair.
constexpr uint32_t kRpCtl = 16;
enum : uint32_t { kRpQTail = 0, kRpMin = 1, kRpUnit = 2, kRpOvf = 3 };
constexpr uint32_t kRpNone = 0xFFFFu;  // tent: no level yet
constexpr uint32_t kRpMaxCap = 127u;   // A's index fits the node byte's low 7 bits
constexpr uint32_t kRpHash = 512u;     // ignored-link hash slots (a pair ignoring more goes forward)

// LDS of one pair (~8 KB on the fabric, 16 pairs of 128 threads per CU): one byte per
// node — its lost-pathLink count while unaffected (a node with more than 127 base
// pathLinks hands the pair to the forward solve), 0x80 | its index in A once in A (no
// pathLink is lost after the last one); the ignored links as an open-addressing hash;
// per A entry its node, tentative level + 1 and a settled flag (A is capped).
struct RepairLayout {
  uint32_t nb, hsh, q, tent, done, total;
};
__host__ __device__ inline RepairLayout repair_layout(uint32_t V, uint32_t L) {
  RepairLayout l;
  uint32_t off = kRpCtl * 4u;
  auto take = [&](uint32_t bytes) {
    const uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.nb = take((V + 3u) & ~3u);
  l.hsh = take(4u * kRpHash);
  l.q = take(2u * kRpMaxCap);
  l.tent = take(2u * kRpMaxCap);
  l.done = take(kRpMaxCap);
  l.total = off;
  return l;
}

__device__ __forceinline__ uint32_t rp_level(uint64_t b, uint64_t cost) {
  return cost == 1u ? (uint32_t)b : (uint32_t)((double)b / (double)cost);  // exact: b is a multiple
}

template <int BLOCK, int G>
__global__ __launch_bounds__(BLOCK) void ksp_repair_kernel(DevGraph g, const uint32_t* srcs, const uint32_t* prow,
                                                          const uint32_t* tgts, const uint32_t* list,
                                                          const uint32_t* list_count, uint32_t n,
                                                          const uint32_t* ign_ptr, const uint32_t* ign_end,
                                                          const uint32_t* ign_links, const uint64_t* base_rows,
                                                          const uint32_t* tl_off_all, uint64_t cost,
                                                          uint16_t* rows16, uint32_t ltag, uint32_t lmask,
                                                          uint32_t cap, uint32_t* mode, uint32_t* retry_list,
                                                          uint32_t* retry_count, uint32_t* work_ctr) {
  static_assert(BLOCK % 64 == 0 && 64 % G == 0, "groups of G lanes inside a wavefront");
  constexpr uint32_t NG = BLOCK / G;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V, L = g.L, tid = threadIdx.x;
  const RepairLayout lay = repair_layout(V, L);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  uint32_t* nbw = reinterpret_cast<uint32_t*>(base + lay.nb);
  uint8_t* nb = reinterpret_cast<uint8_t*>(base + lay.nb);
  uint32_t* hsh = reinterpret_cast<uint32_t*>(base + lay.hsh);
  auto slot_of = [](uint32_t l) { return (l * 2654435761u) >> 23; };  // 9 bits: kRpHash
  auto is_ign = [&](uint32_t l) {
    for (uint32_t h = slot_of(l);; h = (h + 1u) & (kRpHash - 1u)) {
      const uint32_t x = hsh[h];
      if (x == l) return true;
      if (x == 0xFFFFFFFFu) return false;
    }
  };
  uint16_t* q = reinterpret_cast<uint16_t*>(base + lay.q);
  uint16_t* tent = reinterpret_cast<uint16_t*>(base + lay.tent);
  uint8_t* done = reinterpret_cast<uint8_t*>(base + lay.done);
  const uint32_t vw = (V + 3u) / 4u;
  const uint32_t grp = tid / G, lg = tid % G;
  const uint32_t units = list ? *list_count : n;
  for (uint32_t unit = blockIdx.x; unit < units;) {
    const uint32_t k = list ? list[unit] : unit;
    const uint32_t s = srcs[k], d = tgts[k];
    if (!(s < V && d < V && s != d) && tid == 0) mode[k] = 0u;
    if (s < V && d < V && s != d) {  // block-uniform (src == dest is never traced)
      const uint32_t row = prow[k];
      const uint64_t* B = base_rows + (size_t)row * V;
      const uint32_t* toff = tl_off_all + (size_t)row * (V + 1u);
      uint16_t* lrow = rows16 + (size_t)k * V;
      for (uint32_t i = tid; i < vw; i += BLOCK) nbw[i] = 0;
      for (uint32_t i = tid; i < kRpHash; i += BLOCK) hsh[i] = 0xFFFFFFFFu;
      if (tid < kRpCtl && tid != kRpUnit) ctl[tid] = 0;
      __syncthreads();
      const uint32_t ib = ign_ptr[k], ie = ign_end[k];
      if (ie - ib > kRpHash / 2u) {  // a half-full table at most (short probes)
        if (tid == 0) ctl[kRpOvf] = 1u;
      } else {
        for (uint32_t i = ib + tid; i < ie; i += BLOCK) {
          const uint32_t l = ign_links[i];
          for (uint32_t h = slot_of(l);; h = (h + 1u) & (kRpHash - 1u)) {
            const uint32_t old = atomicCAS(&hsh[h], 0xFFFFFFFFu, l);
            if (old == 0xFFFFFFFFu || old == l) break;
          }
        }
      }
      // one lost pathLink of y; the arrival that loses the last one puts y into A
      auto lose = [&](bool hit, uint32_t y) {
        bool aff = false;
        if (hit) {
          const uint32_t tin = toff[y + 1u] - toff[y];
          if (tin > 127u) {
            ctl[kRpOvf] = 1u;  // the count byte cannot hold it
          } else {
            const uint32_t sh = 8u * (y & 3u);
            aff = ((atomicAdd(&nbw[y >> 2], 1u << sh) >> sh) & 0xFFu) + 1u == tin;
          }
        }
        const uint32_t slot = wave_append(aff, &ctl[kRpQTail]);
        if (aff && slot < cap) {
          q[slot] = (uint16_t)y;
          nb[y] = (uint8_t)(0x80u | slot);  // no arrival touches y's count after its last loss
        }
      };
      // the ignored links' base pathLinks (either direction: tail may expand, edge up, tight)
      for (uint32_t i0 = ib; i0 < ie; i0 += BLOCK / 2u) {
        const uint32_t i = i0 + tid / 2u;
        bool hit = false;
        uint32_t y = 0;
        if (i < ie) {
          const uint32_t l = ign_links[i];
          const uint2 ab = l < L ? g.ledge[l] : make_uint2(UINT32_MAX, UINT32_MAX);
          if (ab.x != UINT32_MAX) {
            const uint32_t e = (tid & 1u) ? ab.y : ab.x, r = (tid & 1u) ? ab.x : ab.y;
            const uint4 re = g.erec[e], rr = g.erec[r];  // e = x->y, r = y->x (its col x, x's sink flag)
            const uint32_t x = rr.x & ~(kEdgeDown | kNodeSink);
            y = re.x & ~(kEdgeDown | kNodeSink);
            if (!(re.x & kEdgeDown) && (x == s || !(rr.x & kNodeSink))) {
              const uint64_t bx = B[x], by = B[y];
              hit = bx != kNoKey && bx + cost == by;
            }
          }
        }
        lose(hit, y);
      }
      __syncthreads();
      // closure: the base pathLinks out of every node put into A
      uint32_t head = 0, tail = __builtin_amdgcn_readfirstlane(ctl[kRpQTail]);
      const bool ovf0 = __builtin_amdgcn_readfirstlane(ctl[kRpOvf]) != 0u;
      while (!ovf0 && head < tail && tail <= cap) {
        for (uint32_t b0 = head; b0 < tail; b0 += NG) {
          const uint32_t idx = b0 + grp;
          uint32_t beg = 0, end = 0;
          uint64_t bx = 0;
          if (idx < tail) {
            const uint32_t x = q[idx];
            if (!g.ovl[x]) {  // a sink (other than src, never in A) has no pathLinks out
              const uint2 r = g.row2[x];
              beg = r.x;
              end = r.y;
              bx = B[x];
            }
          }
          for (uint32_t e = beg + lg; __any(e < end); e += G) {
            bool hit = false;
            uint32_t y = 0;
            if (e < end) {
              const uint4 rec = g.erec[e];
              y = rec.x & ~(kEdgeDown | kNodeSink);
              hit = !(rec.x & kEdgeDown) && bx + cost == B[y] && !is_ign(rec.z);
            }
            lose(hit, y);
          }
        }
        __syncthreads();
        head = tail;
        tail = __builtin_amdgcn_readfirstlane(ctl[kRpQTail]);
      }
      const uint32_t nA = tail;
      const uint32_t di = nb[d] >= 0x80u ? (nb[d] & 0x7Fu) + 1u : 0u;  // dest's index in A + 1, 0: unaffected
      const uint64_t bd = B[d];
      const bool over = nA > cap || ctl[kRpOvf] != 0u;  // block-uniform: the forward solve takes the pair
      if (tid == 0) {
        mode[k] = over ? 1u : 0u;
        if (over) retry_list[atomicAdd(retry_count, 1u)] = k;
      }
      if (!over && nA && bd != kNoKey) {  // block-uniform; dest unreached in the base: nothing is traced
        // seeds: each node of A from its unaffected in-neighbours (usable, not ignored, able
        // to expand): base level + 1, the group's minimum
        for (uint32_t b0 = 0; b0 < nA; b0 += NG) {
          const uint32_t idx = b0 + grp;
          uint32_t beg = 0, end = 0;
          if (idx < nA) {
            const uint2 r = g.row2[q[idx]];
            beg = r.x;
            end = r.y;
          }
          uint32_t best = kRpNone;
          for (uint32_t e = beg + lg; e < end; e += G) {
            const uint4 rec = g.erec[e];  // y->u, the mirror of u->y
            const uint32_t u = rec.x & ~(kEdgeDown | kNodeSink);
            if (!(rec.x & kEdgeDown) && (u == s || !(rec.x & kNodeSink)) && nb[u] < 0x80u &&
                !is_ign(rec.z)) {
              const uint64_t bu = B[u];
              if (bu != kNoKey) best = min(best, rp_level(bu, cost) + 2u);  // level + 1, stored + 1
            }
          }
#pragma unroll
          for (uint32_t m = 1; m < (uint32_t)G; m <<= 1) best = min(best, (uint32_t)__shfl_xor((int)best, (int)m));
          if (idx < nA && lg == 0u) {
            tent[idx] = (uint16_t)min(best, kRpNone);
            done[idx] = 0;
          }
        }
        __syncthreads();
        // settle A level by level: the smallest open tent, then its nodes relax their A
        // neighbours; up to dest's base level - 1 (dest unaffected) or dest's own level
        const uint32_t dlim = di ? 0xFFFFFFFFu : rp_level(bd, cost);  // levels below it are needed
        for (;;) {
          if (tid == 0) ctl[kRpMin] = kRpNone;
          __syncthreads();
          if (tid < nA && !done[tid] && tent[tid] != kRpNone) atomicMin(&ctl[kRpMin], (uint32_t)tent[tid]);
          __syncthreads();
          const uint32_t t = __builtin_amdgcn_readfirstlane(ctl[kRpMin]);  // level + 1
          if (t == kRpNone || t - 1u >= dlim) break;
          const bool d_now = di && !done[di - 1u] && tent[di - 1u] == t;
          __syncthreads();  // every thread has read done[] before the bucket is marked
          for (uint32_t b0 = 0; b0 < nA; b0 += NG) {
            const uint32_t idx = b0 + grp;
            uint32_t beg = 0, end = 0;
            if (idx < nA && !done[idx] && tent[idx] == t) {
              if (lg == 0u) done[idx] = 1;
              const uint32_t y = q[idx];
              if (!d_now && !g.ovl[y]) {  // relax out of it (a sink does not expand)
                const uint2 r = g.row2[y];
                beg = r.x;
                end = r.y;
              }
            }
            // (a bucket node of a later pass still reads open with tent == t: never lowered)
            for (uint32_t e = beg + lg; e < end; e += G) {
              const uint4 rec = g.erec[e];
              const uint32_t z = rec.x & ~(kEdgeDown | kNodeSink);
              const uint32_t zb = nb[z], zi = zb & 0x7Fu;
              if (zb >= 0x80u && !(rec.x & kEdgeDown) && !done[zi] && tent[zi] > t + 1u && !is_ign(rec.z))
                tent[zi] = (uint16_t)(t + 1u);  // every writer of this level writes the same value
            }
          }
          __syncthreads();
          if (d_now) break;
        }
        // write A: the settled levels below dest's, dest's own, lmask for the rest
        const uint32_t dl = di ? (done[di - 1u] ? (uint32_t)tent[di - 1u] - 1u : 0xFFFFFFFFu) : rp_level(bd, cost);
        if (tid < nA) {
          const uint32_t y = q[tid];
          uint32_t lev = lmask;
          if (done[tid]) {
            const uint32_t l = (uint32_t)tent[tid] - 1u;
            if (l < dl || y == d) lev = l;
          }
          lrow[y] = (uint16_t)(ltag | lev);
        }
      }
    }
    __syncthreads();  // every thread is done with this pair's LDS before the next one's zeroing
    if (tid == 0) ctl[kRpUnit] = gridDim.x + atomicAdd(work_ctr, 1u);
    __syncthreads();
    unit = __builtin_amdgcn_readfirstlane(ctl[kRpUnit]);
  }
}

}  // namespace

// A u16 copy of the pair's distance row in LDS was measured slower on the fabric (fewer
// wavefronts per CU, rounds 2-3) and is not taken; the layout keeps the slot at size 0.
bool ksp_use_d16(int) { return false; }

// Packed arena entries (ksp_layout) when node and link ids fit 16 bits. Fabric small
// tier: 11.9 -> 10.9 KB per wavefront. OPENR_SPF_KSP_PACK=0: unpacked (A/B, tests).
bool ksp_pack(uint32_t V, uint32_t L) {
  return V <= 65536u && L <= 65536u && bfs::env_u32("OPENR_SPF_KSP_PACK", 1u, 0u, 1u) != 0u;
}

// Small tier: a traced path has at most as many hops as the source's BFS depth on
// uniform-cost graphs; 2x the sampled depth + 8 covers the sample's misses and weighted
// graphs' longer hop counts, and the arena holds that many frames of typical width.
// Everything it cannot hold re-runs in the full tier (kKspMaxDepth / kKspArena).
KspCaps ksp_caps(const DevGraph& g, bool full) {
  KspCaps c{kKspMaxDepth, kKspArena};
  if (full || bfs::env_u32("OPENR_SPF_KSP_TIER", 1u, 0u, 1u) == 0) return c;
  c.frames = std::min<uint32_t>(kKspMaxDepth, std::max<uint32_t>(16u, 2u * g.est_depth + 8u));
  // half-full frames on average (measured on the fabric: arena 256 > 320 > 512 in speed,
  // the LDS it frees buys wavefronts; the rare deeper DFS re-runs in the full tier)
  const uint32_t want = (g.est_depth + 2u) * std::max<uint32_t>(g.max_deg, 1u) / 2u;
  c.arena = std::min<uint32_t>(kKspArena, std::max<uint32_t>(256u, (want + 63u) & ~63u));
  // test hooks: force tiny small-tier capacities so most pairs take the full-tier re-run
  c.frames = bfs::env_u32("OPENR_SPF_KSP_SMALL_FRAMES", c.frames, 1u, kKspMaxDepth);
  c.arena = bfs::env_u32("OPENR_SPF_KSP_SMALL_ARENA", c.arena, 1u, kKspArena);
  return c;
}

uint32_t ksp_tier_lds_bytes(const DevGraph& g, bool full, int kind, bool stats_on = false) {
  const KspCaps c = ksp_caps(g, full);
  const uint32_t t =
      ksp_layout(g.V, g.L, g.max_deg, c.frames, c.arena, ksp_use_d16(kind), ksp_pack(g.V, g.L), stats_on).total;
  return t <= kMaxLds ? t : 0;
}

uint32_t ksp_max_grid(const DevGraph& g, int num_cus) {
  uint32_t m = 0;
  for (int kind = 1; kind <= 2; ++kind)
    for (bool full : {false, true}) m = std::max(m, blocks_for(UINT32_MAX, ksp_tier_lds_bytes(g, full, kind), num_cus, kWave));
  return m;
}

uint32_t ksp_stats_count() { return kKspStats; }

uint32_t ksp_repair_lds_bytes(uint32_t V, uint32_t L) {
  const uint32_t t = repair_layout(V, L).total;
  return V < 65535u && t <= kMaxLds ? t : 0u;
}

hipError_t launch_ksp_repair(const DevGraph& g, const uint32_t* srcs, const uint32_t* prow, const uint32_t* tgts,
                             const uint32_t* list, const uint32_t* list_count, uint32_t n, const uint32_t* ign_ptr,
                             const uint32_t* ign_end, const uint32_t* ign_links, const uint64_t* base_rows,
                             const uint32_t* tl_off, uint64_t cost, uint16_t* rows16, uint32_t ltag, uint32_t lmask,
                             uint32_t* mode, uint32_t* retry_list, uint32_t* retry_count, uint32_t* work_ctr,
                             int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  if (!mode || !retry_list || !retry_count) return hipErrorInvalidValue;
  // a pair whose affected set outgrows the cap is solved forward (OPENR_SPF_KSP_REPAIR_CAP)
  const uint32_t cap = bfs::env_u32("OPENR_SPF_KSP_REPAIR_CAP", kRpMaxCap, 0u, kRpMaxCap);
  const uint32_t lds = ksp_repair_lds_bytes(g.V, g.L);
  if (!lds || !work_ctr || !cost) return hipErrorInvalidValue;
  const uint32_t gl = bfs::env_u32("OPENR_SPF_KSP_REPAIR_G", 16u, 4u, 64u);  // lanes per node (tuning)
  auto k = gl == 4 ? ksp_repair_kernel<128, 4> : gl == 8 ? ksp_repair_kernel<128, 8>
         : gl == 32 ? ksp_repair_kernel<128, 32> : gl == 64 ? ksp_repair_kernel<128, 64> : ksp_repair_kernel<128, 16>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  note_launch("ksp_repair_kernel");
  hipLaunchKernelGGL(k, dim3(blocks_for(n, lds, num_cus, 128u)), dim3(128), lds, s, g, srcs, prow, tgts, list,
                     list_count, n, ign_ptr, ign_end, ign_links, base_rows, tl_off, cost, rows16, ltag, lmask, cap,
                     mode, retry_list, retry_count, work_ctr);
  return hipGetLastError();
}

bool ksp_path_lists_ok(const DevGraph& g) {
  return g.erecs != nullptr && ksp_pack(g.V, g.L) && bfs::env_u32("OPENR_SPF_KSP_TL", 1u, 0u, 1u) != 0u;
}

hipError_t launch_ksp_path_lists(const DevGraph& g, const uint32_t* sources, uint32_t n_src, const uint64_t* rows,
                                 uint32_t* off, uint2* ent, int num_cus, hipStream_t s) {
  if (!n_src) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>(n_src, (uint32_t)num_cus * 8u);
  hipLaunchKernelGGL(ksp_path_lists_kernel, dim3(grid), dim3(256), 0, s, g, sources, n_src, rows, off, ent);
  return hipGetLastError();
}

uint32_t ksp_lds_bytes(uint32_t V, uint32_t L, uint32_t max_deg) {
  const uint32_t t =
      ksp_layout(V, L, max_deg, kKspMaxDepth, kKspArena, ksp_use_d16(1) || ksp_use_d16(2), ksp_pack(V, L)).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_ksp_trace(int kind, const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                            const uint32_t* pdst, uint32_t first, uint32_t n, const uint64_t* rows, uint32_t* ign_io,
                            uint32_t* ign_end, uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap, uint32_t* status,
                            uint32_t* qbuf, int num_cus, hipStream_t s, unsigned long long* stats,
                            const uint32_t* list, const uint32_t* list_count, uint32_t* retry_list,
                            uint32_t* retry_count, uint32_t* work_ctr, const uint16_t* rows16, uint64_t lcost,
                            uint32_t ltag, const uint32_t* tl_off, const uint2* tl_ent, const uint64_t* tl_rows,
                            const uint32_t* rmode) {
  if (!n) return hipSuccess;
  if (tl_off && (!lcost || !g.erecs || !ksp_pack(g.V, g.L) || (kind == 2 && !tl_rows))) return hipErrorInvalidValue;
  if (rmode && (kind != 2 || !tl_rows || !rows16 || !ltag)) return hipErrorInvalidValue;
  if (!work_ctr) return hipErrorInvalidValue;
  const bool full = retry_list == nullptr;  // the small tier hands overflows to a full-tier re-run
  const KspCaps caps = ksp_caps(g, full);
  const uint32_t lds = ksp_tier_lds_bytes(g, full, kind, stats != nullptr);
  if (!lds || !qbuf) return hipErrorInvalidValue;
  // a re-run launch covers the listed pairs only; its surplus wavefronts exit at once
  const uint32_t grid = blocks_for(n, lds, num_cus, kWave);  // <= ksp_max_grid: qbuf holds grid * V
  auto k = kind == 1 ? ksp_trace_kernel<1> : ksp_trace_kernel<2>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWave), lds, s, g, sources, prow, pdst, first, n, rows, ign_io, ign_end,
                     ign_cap, tok, tok_cap, status, qbuf,
                     bfs::env_u32("OPENR_SPF_KSP_PROBE", kKspProbeAfter, 0u, 1u << 30),
                     (ksp_use_d16(kind) ? 1u : 0u) | (bfs::env_u32("OPENR_SPF_KSP_RESUME", 1u, 0u, 1u) << 1) |
                         (ksp_pack(g.V, g.L) ? 8u : 0u),
                     stats, caps.frames, caps.arena, list, list_count, retry_list, retry_count, work_ctr, rows16,
                     lcost, ltag, tl_off, tl_ent, tl_rows, rmode);
  return hipGetLastError();
}

hipError_t launch_strided_iota(uint32_t* p, uint32_t n, uint32_t stride, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((n + 255u) / 256u, (uint32_t)num_cus * 8u));
  hipLaunchKernelGGL(strided_iota, dim3(grid), dim3(256), 0, s, p, n, stride);
  return hipGetLastError();
}

hipError_t launch_gather_sources(const uint32_t* sources, const uint32_t* prow, uint32_t first, uint32_t n,
                                 uint32_t* out, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((n + 255u) / 256u, (uint32_t)num_cus * 8u));
  hipLaunchKernelGGL(gather_sources, dim3(grid), dim3(256), 0, s, sources, prow, first, n, out);
  return hipGetLastError();
}

hipError_t launch_ksp_select_pairs(const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                                   const uint32_t* pdst, uint32_t first, uint32_t n, const uint32_t* tok1,
                                   uint32_t* tok2, uint32_t tok_cap, uint32_t* out_src, uint32_t* list,
                                   uint32_t* count, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((n + 255u) / 256u, (uint32_t)num_cus * 8u));
  hipLaunchKernelGGL(ksp_select_pairs, dim3(grid), dim3(256), 0, s, g, sources, prow, pdst, first, n, tok1, tok2,
                     tok_cap, out_src, list, count);
  return hipGetLastError();
}

}  // namespace openr_spf
