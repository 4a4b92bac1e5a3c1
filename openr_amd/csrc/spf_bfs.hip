// spf_bfs.hip — uniform-cost SPF kernel, "code" family (every usable edge costs the same
// c: grids and fabrics with unit metrics, and runSpf(useLinkMetric=false) hop counts).
// Chosen for shallow graphs (small diameter, wide frontiers: fabrics); deep graphs use
// the exact-level family in spf_bfs_lvl.hip (spf_capi.hip picks per graph).
//
// Semantics (LinkState::runSpf, /root/reference/openr/decision/LinkState.cpp:808-882,
// closed form for positive metrics): with uniform cost the
// reference's (metric, name) pop order settles whole BFS levels in turn, and
//   dist(v) = c * level(v)    (UINT64_MAX if v is never reached)
//   nh(v)   = OR over tight in-edges u->v of (u == src ? {v} : nh(u))
// where u->v is tight iff it is usable, u is on level L, v on level L+1, and u may be
// expanded (u == src or u not overloaded, LinkState.cpp:831-838).
//
// Per-node state in LDS is ONE packed field: [next-hop bits | 3-bit level code].
// code 0 = not reached, code (L % 3) + 1 = reached on level L, code | 4 = a sink
// (overloaded, never expanded) already settled. With unit steps every EXPANDED
// neighbour of a level-L node sits on level L-1, L or L+1, so the code alone tells a
// tight arrival (v unreached, or reached on L+1 this level) from a stale one; a sink
// can sit further back and is marked when popped so it never aliases. Levels are
// never stored, so BFS depth is unbounded. One atomicOr per tight edge ORs nh(u)
// and the code of L+1 into v's field; the arrival that saw code 0 appends v to the
// frontier ring (no visited bitmap, no level array). dist(v) = c * L is stored to HBM
// when v is expanded (scattered 8-byte stores, merged in L2); unreached nodes get
// UINT64_MAX and every node its next-hop bytes in one coalesced pass at the end.
//
// Shape: one workgroup (128 or 256 threads) owns one solve at a time, dynamically
// scheduled over the batch. Level L expands ring slots [head, tail): G lanes per
// frontier node, K=4 edges per lane loaded ahead (one 16-byte ELL load when every row
// has <= 4 edges); the K field reads and then the K atomics of a lane are issued
// together; appends are wave-aggregated (3 ballots + one ds_add per wave). One LDS
// barrier per level.
//
// Field widths by source class (distinct degree d of the source = next-hop set width):
//   8 bits (d <= 5), 16 bits (d <= 13), 32 bits (d <= 29); d > 29: the wide pass (one
//   unit per solve, a multi-word bit stream per node, bfs_wide_kernel) or, with an ignore
//   set / tight-edge output, 32-bit fields holding 29-bit slices of the set (one workgroup
//   pass per (solve, slice); the slices' chunks merged into the next-hop bytes afterwards,
//   slice_merge).
//
// No MFMA: min-plus relaxation is not a matrix contraction (DESIGN.md "Roofline").
#include <algorithm>
#include <cstdlib>

#include "spf_bfs_common.h"
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;
using namespace bfs;

// Packed node state: FB-bit fields, next-hop bits at kNhs, level code in bits [0, 3).
template <int FB>
struct State {
  static constexpr uint32_t kPer = 32u / FB;
  static constexpr uint32_t kFieldMask = FB == 32 ? 0xFFFFFFFFu : ((1u << (FB & 31)) - 1u);
  static constexpr uint32_t kNhs = 3u;           // next-hop bits start here
  static constexpr uint32_t kNhBits = FB - kNhs;  // 5 / 13 / 29
  static constexpr uint32_t kNhMask = ((1u << kNhBits) - 1u) << kNhs;
  static __host__ __device__ uint32_t words(uint32_t V) { return (V + kPer - 1u) / kPer; }
  static __device__ __forceinline__ uint32_t word(uint32_t v) { return v / kPer; }
  static __device__ __forceinline__ uint32_t shift(uint32_t v) { return (v % kPer) * FB; }
  static __device__ __forceinline__ uint32_t field(const uint32_t* st, uint32_t v) {
    return (st[word(v)] >> shift(v)) & kFieldMask;
  }
};

__device__ __forceinline__ uint32_t level_code(uint32_t L) { return L % 3u + 1u; }
constexpr uint32_t kCodeMask = 7u, kCodeSettledSink = 4u;


struct BfsLayout {
  uint32_t st, ring, ign, dummy, total;
};

// ring = frontier queue (power of two, wraps) in the fast path, or the full BFS-order
// array (capacity V, never wraps) in the fallback path.
__host__ __device__ inline BfsLayout bfs_layout(uint32_t V, uint32_t L, bool has_ign, uint32_t fb, uint32_t ring_cap) {
  BfsLayout l;
  uint32_t off = 32;  // control: append counters [0..3], overflow flag [4], target [5]
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  const uint32_t per = 32u / fb;
  l.st = take(4u * ((V + 1u + per - 1u) / per));  // + node V: a settled sentinel (lean edge loop)
  l.ring = take(2u * ring_cap);
  l.ign = has_ign ? take(4u * ((L + 31u) / 32u)) : 0u;
  l.dummy = take(4u * 64u);  // per-lane sink for the no-op atomics of non-tight edges
  l.total = off;
  return l;
}

// End of a solve: UINT64_MAX for unreached nodes (reached ones were stored when
// expanded) and the next-hop bytes of every node, coalesced. Sliced classes: slice s
// owns next-hop bytes [3s, 3s + 3); slice 0 also zero-fills the bytes past the last
// slice.
template <int FB, int BLOCK, bool SLICED, bool GENERIC>
__device__ __forceinline__ void write_out(const SolveArgs& a, uint32_t k, uint32_t sid, uint32_t slice, uint32_t V,
                                          const uint32_t* st, bool nt) {
  using S = State<FB>;
  const uint32_t tid = threadIdx.x;
  uint64_t* drow = a.dist + out_row_of(a, sid) * V;
  const uint32_t nb = a.nh_bytes;
  uint8_t* nrow = a.nh ? a.nh + out_row_of(a, sid) * V * nb : nullptr;
  if (GENERIC && a.lvl16) {  // u16 level row (dist-only, never sliced)
    if (a.lvl_tag) return;  // tagged rows: unreached nodes stay unwritten
    uint16_t* lrow = a.lvl16 + out_row_of(a, sid) * V;
    for (uint32_t v = tid; v < V; v += BLOCK)
      if ((S::field(st, v) & kCodeMask) == 0u) lrow[v] = 0xFFFFu;
    return;
  }
  if (!SLICED || slice == 0)
    for (uint32_t v = tid; v < V; v += BLOCK)
      if ((S::field(st, v) & kCodeMask) == 0u) drow[v] = ~0ull;
  if (!nrow) return;
  if (SLICED) {  // the slice's 29-bit chunks, coalesced; slice_merge packs the bytes
    uint32_t* trow = a.slice_tmp + ((size_t)(k - a.k0) * a.nsl + slice) * V;  // chunk-local row
    for (uint32_t v = tid; v < V; v += BLOCK) store_row<uint32_t>(&trow[v], S::field(st, v) >> S::kNhs, nt);
    return;
  }
  if (FB == 8 && nb == 1 && ((reinterpret_cast<uintptr_t>(nrow) | V) & 3u) == 0) {
    // four nodes (one state dword) per lane -> one u32 of four next-hop bytes
    uint32_t* n32 = reinterpret_cast<uint32_t*>(nrow);
    for (uint32_t i = tid; i < V / 4u; i += BLOCK) store_row<uint32_t>(&n32[i], (st[i] >> 3) & 0x1F1F1F1Fu, nt);
    return;
  }
  for (uint32_t i = tid; i < V * nb; i += BLOCK) {
    const uint32_t v = i / nb, j = i - v * nb;
    const uint32_t x = S::field(st, v) >> S::kNhs;
    nrow[i] = j < 4u ? (uint8_t)(x >> (8u * j)) : (uint8_t)0;
  }
}

// ELLM: 0 = CSR rows only; 1 = the first 4 edges of a row from one 16-byte ELL load,
// the rest from CSR (G == 1); 2 = ELL only (every row has <= 4 edges, no ignore set,
// no tight-edge output).
// RING = true : queue = power-of-two ring; a (solve, slice) unit whose two adjacent
//               levels exceed the ring is appended to a.ovf_list (count *ovf_count).
// RING = false: full BFS order (capacity V, never overflows). from_list != 0: the
//               units of a.ovf_list only (the re-run of what the ring variant flagged).
// SLICED: one unit = (solve, 29-bit slice of the next-hop set).
// GENERIC = false: no ignore set and no tight-edge output (compile time), the
// all-sources / prefetch case; GENERIC = true handles both at run time.
template <int FB, int BLOCK, bool RING, int ELLM, bool GENERIC, bool SLICED>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(BLOCK >= 1024 ? 4 : 8))) void bfs_code_kernel(
    DevGraph g, SolveArgs a, uint64_t cost, uint32_t glog, uint32_t has_ign_rt, uint32_t ring_cap, uint32_t from_list,
    uint32_t* ctr, uint32_t* ovf_count, uint32_t nt) {
  using S = State<FB>;
  constexpr int K = (int)kBfsEdgesPerLane;
  const bool has_ign = GENERIC && has_ign_rt != 0;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t s_next;
  const uint32_t V = g.V, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = __lane_id();
  const BfsLayout lay = bfs_layout(V, g.L, has_ign, FB, ring_cap);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  uint32_t* st = reinterpret_cast<uint32_t*>(base + lay.st);
  uint16_t* ring = reinterpret_cast<uint16_t*>(base + lay.ring);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  uint32_t* dummy = reinterpret_cast<uint32_t*>(base + lay.dummy);
  const uint32_t st_words = S::words(V + 1u);
  // lean edge loop (no ignore set, no tight-edge output, CSR rows): padding and down slots
  // read the sentinel node V, whose code is "settled" (never tight, never empty), and a
  // lane's no-op atomic goes to its own all-ones dummy word, so the returned field alone
  // elects the appending arrival
  constexpr bool kLeanT = !GENERIC && ELLM == 0;
  const bool kLean = kLeanT;
  if (kLean && tid < 64) dummy[tid] = 0xFFFFFFFFu;
  const uint32_t ign_words = (g.L + 31u) / 32u;
  const uint32_t G = 1u << glog, ngroups = BLOCK >> glog, groups_per_wave = 64u >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  const uint32_t tight_words = (g.E + 63u) / 64u;
  const uint32_t rmask = ring_cap - 1u;  // RING: ring_cap is a power of two
  const uint32_t nsl = SLICED ? a.nsl : 1u;
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  // sliced class in chunks: class-local solves [k0, k0 + krows) (a re-run lists global uids)
  const uint32_t k0 = SLICED ? a.k0 : 0u;
  const uint32_t in_chunk = !SLICED || !a.krows ? count : count > k0 ? min(a.krows, count - k0) : 0u;
  // a re-run launch with nothing flagged does no work
  const uint32_t units = from_list ? *ovf_count : in_chunk * nsl;
  // nothing flagged: every workgroup leaves at once (no unit is taken, so the scheduling
  // counters stay at rest and no workgroup needs to retire; saves the 256 retire atomics)
  if (from_list && units == 0u) return;
#ifdef OPENR_SPF_PROFILE
  // [0] load (ring + ELL/row), [1] field reads, [2] atomics, [3] append, [4] barrier,
  // [5] init + level 0, [6] write out, [7] passes, [8] levels, [9] solves
  uint64_t pc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
#endif

  for (uint32_t unit = blockIdx.x; unit < units;) {
    const uint32_t uid = from_list ? a.ovf_list[unit] : k0 * nsl + unit;  // class-local (solve, slice) index
    const uint32_t k = SLICED ? uid / nsl : uid, slice = SLICED ? uid - k * nsl : 0u;
    const uint32_t sid = a.perm ? a.perm[first + k] : k;
    const uint32_t src = a.sources[sid];
    if (src < V) {  // block-uniform
      OPENR_PROF_STAMP(t0);
      const bool own_dist = !SLICED || slice == 0;
      uint64_t* drow = a.dist + out_row_of(a, sid) * V;
      uint16_t* lrow = (GENERIC && a.lvl16) ? a.lvl16 + out_row_of(a, sid) * V : nullptr;
      // settle node u on level l (distance l * cost): u64 distance or u16 level row
      const uint32_t ltag = (GENERIC && lrow) ? a.lvl_tag << a.lvl_shift : 0u;
      auto put = [&](uint32_t u, uint32_t l) {
        if (GENERIC && lrow) lrow[u] = (uint16_t)(ltag | l);
        else drow[u] = (uint64_t)l * cost;
      };
      for (uint32_t i = tid; i < st_words; i += BLOCK) st[i] = 0;
      if (has_ign)
        for (uint32_t i = tid; i < ign_words; i += BLOCK) ign[i] = 0;
      if (tid < 8) ctl[tid] = 0;
      __syncthreads();
      if (has_ign) load_ignore(ign, ign_words, a, sid, g.L);
      if (tid == 0) {
        atomicOr(&st[S::word(V)], kCodeSettledSink << S::shift(V));  // the sentinel
        atomicOr(&st[S::word(src)], level_code(0) << S::shift(src));
        if (own_dist) put(src, 0u);
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
              const uint32_t b = g.nbr[e];
              uint32_t nhb = 0;
              if (!SLICED) nhb = a.dist_only ? 0u : 1u << b;
              else if (b / S::kNhBits == slice) nhb = 1u << (b - slice * S::kNhBits);
              const uint32_t x = (nhb << S::kNhs) | level_code(1);
              fresh = ((atomicOr(&st[S::word(v)], x << S::shift(v)) >> S::shift(v)) & kCodeMask) == 0u;
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

      uint32_t head = 1, tail = 1u + ctl[0], L = 1, cnext = level_code(2);
      bool overflow = false;  // block-uniform
      // pull test (2): the target's usable in-neighbours w, one per lane (w = V: none), and
      // their rows, loaded at the first test of the solve and kept for the later levels
      uint32_t pw_w = V, pw_beg = 0, pw_end = 0;
      bool pw_ready = false;  // block-uniform
      while (head < tail) {
        uint32_t* cnt = &ctl[L & 3u];
        if (tid == 0) ctl[(L + 1u) & 3u] = 0;  // last read three barriers ago
        const uint64_t dL = (uint64_t)L * cost;
        if (!SLICED && a.target && a.dist_only) {
          // pull tests for the target (KSP2 second SPF). A trace to the target walks tight
          // in-edges (LinkState.cpp:398-419), so it reads only nodes on shortest paths to
          // it; every other node may read UINT64_MAX. With the target unreached:
          //  (1) a usable edge to a level-L node (not a sink) puts it on level L+1;
          //  (2) else each unreached neighbour w (not a sink) with a usable edge to a
          //      level-L node (not a sink) lies on level L+1, and then the target on L+2.
          // Either way level L is settled without expanding it and the solve ends.
          const uint32_t t = a.target[sid];  // block-uniform
          if (t < V) {
            bool hit1 = false, hit2 = false;  // wave-uniform
            if ((S::field(st, t) & kCodeMask) == 0u) {
              const uint2 rt = g.row2[t];
              const uint32_t cL = level_code(L);
              if (rt.y - rt.x <= (uint32_t)BLOCK && !(a.dist_only & 2u)) {  // bit 1: per-wave form (A/B)
                // t's row spread over the block (entry wave + lane * waves): test (1) is one
                // ballot, and the unreached w's rows are scanned four at a time with every
                // load in flight at once, instead of one w per wave with three dependent
                // loads each (t's record, w's row bounds, w's row) at every level
                if (!pw_ready) {
                  pw_ready = true;
                  const uint32_t i = rt.x + wave + (BLOCK / 64u) * lane;
                  if (i < rt.y) {
                    const uint4 rw = g.erec[i];  // t->w: {w | flags, ., link, .}
                    if (!((rw.x & (kEdgeDown | kNodeSink)) || (has_ign && test_bit(ign, rw.z)))) {
                      pw_w = rw.x & ~(kEdgeDown | kNodeSink);
                      const uint2 rr = g.row2[pw_w];
                      pw_beg = rr.x;
                      pw_end = rr.y;
                    }
                  }
                }
                const uint32_t cw = pw_w < V ? (S::field(st, pw_w) & kCodeMask) : 0xFFu;
                hit1 = __any(cw == cL);
                uint64_t m = __ballot(cw == 0u);
                const uint32_t* er = reinterpret_cast<const uint32_t*>(g.erec);
                while (m) {
                  uint32_t bw[4], bb[4], be[4];
#pragma unroll
                  for (int b = 0; b < 4; ++b) {
                    const uint32_t j = m ? (uint32_t)__builtin_ctzll(m) : 0u;
                    const bool has = m != 0u;
                    m &= m - 1u;
                    bw[b] = has ? (uint32_t)__builtin_amdgcn_readlane((int)pw_w, (int)j) : V;
                    bb[b] = has ? (uint32_t)__builtin_amdgcn_readlane((int)pw_beg, (int)j) : 0u;
                    be[b] = has ? (uint32_t)__builtin_amdgcn_readlane((int)pw_end, (int)j) : 0u;
                  }
                  uint32_t rx[8], rz[8];
#pragma unroll
                  for (int c = 0; c < 8; ++c) {  // w->x records: w b = c / 2, chunk c % 2
                    const uint32_t e = bb[c >> 1] + (uint32_t)(c & 1) * 64u + lane;
                    const bool in = e < be[c >> 1];
                    rx[c] = in ? er[4u * e] : kEdgeDown;
                    rz[c] = in ? er[4u * e + 2u] : 0u;
                  }
#pragma unroll
                  for (int b = 0; b < 4; ++b) {
                    if (bw[b] >= V) continue;  // wave-uniform
                    bool q = false;
#pragma unroll
                    for (int c = 2 * b; c < 2 * b + 2; ++c) {
                      const uint32_t x = rx[c] & ~(kEdgeDown | kNodeSink);
                      q |= !(rx[c] & (kEdgeDown | kNodeSink)) && !(has_ign && test_bit(ign, rz[c])) &&
                           (S::field(st, x) & kCodeMask) == cL;
                    }
                    for (uint32_t e = bb[b] + 128u + lane; e < be[b]; e += 64u) {  // rows past 128 edges
                      const uint32_t xr = er[4u * e];
                      q |= !(xr & (kEdgeDown | kNodeSink)) && !(has_ign && test_bit(ign, er[4u * e + 2u])) &&
                           (S::field(st, xr & ~(kEdgeDown | kNodeSink)) & kCodeMask) == cL;
                    }
                    if (__any(q)) {  // w lies on level L+1 (its code was 0, so no level-L test reads it)
                      hit2 = true;
                      if (lane == 0) {
                        atomicOr(&st[S::word(bw[b])], cnext << S::shift(bw[b]));
                        put(bw[b], L + 1u);
                      }
                    }
                  }
                }
              } else
              for (uint32_t i = rt.x + wave; i < rt.y; i += BLOCK / 64u) {
                const uint4 rw = g.erec[i];  // t->w: {w | flags, ., link, .} (same for all lanes)
                if ((rw.x & (kEdgeDown | kNodeSink)) || (has_ign && test_bit(ign, rw.z))) continue;
                const uint32_t w = rw.x & ~(kEdgeDown | kNodeSink);
                const uint32_t cw = S::field(st, w) & kCodeMask;
                if (cw == cL) hit1 = true;
                if (cw != 0u) continue;
                const uint2 rr = g.row2[w];
                bool q = false;
                for (uint32_t e = rr.x + lane; e < rr.y; e += 64u) {
                  const uint4 rx = g.erec[e];  // w->x
                  const uint32_t x = rx.x & ~(kEdgeDown | kNodeSink);
                  q |= !(rx.x & (kEdgeDown | kNodeSink)) && !(has_ign && test_bit(ign, rx.z)) &&
                       (S::field(st, x) & kCodeMask) == cL;
                }
                if (__any(q)) {  // w lies on level L+1 (its code was 0, so no level-L test reads it)
                  hit2 = true;
                  if (lane == 0) {
                    atomicOr(&st[S::word(w)], cnext << S::shift(w));
                    put(w, L + 1u);
                  }
                }
              }
            }
            if (lane == 0 && (hit1 || hit2)) atomicOr(&ctl[5], hit1 ? 1u : 2u);  // zero until a hit
            lds_barrier();
            const uint32_t f = ctl[5];
            if (f) {
              for (uint32_t i = head + tid; i < tail; i += BLOCK) put(ring[RING ? (i & rmask) : i], L);
              if (tid == t % BLOCK) {  // the thread write_out reads t's field with
                const bool near = (f & 1u) != 0u;
                put(t, near ? L + 1u : L + 2u);
                atomicOr(&st[S::word(t)], (near ? cnext : level_code(L + 2u)) << S::shift(t));
              }
              // the one-thread branch joins here, not at the level loop's exit (a divergent
              // exit: per-lane exit masks around the whole level loop)
              __builtin_amdgcn_wave_barrier();
              break;
            }
          }
        }
        for (uint32_t fb = head; fb < tail; fb += ngroups) {
          if (fb + wave * groups_per_wave >= tail) continue;  // this wave has no slice (uniform)
          OPENR_PROF_STAMP(t0);
          const uint32_t idx = fb + group;
          const bool live = idx < tail;
          uint32_t u = 0, beg = 0, end = 0;
          uint4 ell = make_uint4(kEdgeDown, kEdgeDown, kEdgeDown, kEdgeDown);
          if (live) {
            u = ring[RING ? (idx & rmask) : idx];
            bool sink;
            if (ELLM == 2) {
              ell = g.ellt[u];
              sink = (ell.x & kNodeSink) != 0u;
            } else {
              const uint2 r = g.row2t[u];  // empty (beg flagged kNodeSink) for overloaded nodes
              beg = r.x;
              end = r.y;
              sink = (beg & kNodeSink) != 0u;
              if (ELLM == 1) ell = g.ellt[u];
            }
            if (lane_g == 0) {
              if (own_dist) {  // u settled on level L
                if (GENERIC && lrow) lrow[u] = (uint16_t)(ltag | L);
                else drow[u] = dL;
              }
              if (sink) atomicOr(&st[S::word(u)], kCodeSettledSink << S::shift(u));
            }
          }
          if (ELLM == 2 && live) end = 4;  // kEdgeDown-padded ELL slots stand for the row end
          // nh(u) (final: u was reached a level ago) + the code of level L+1
          const uint32_t xu = (S::field(st, u) & S::kNhMask) | cnext;
#ifdef OPENR_SPF_PROFILE
          OPENR_PROF_STAMP(t1);
          OPENR_PROF_ADD(0, t0, t1);
          pc[7] += 1;
#endif
          if (kLeanT && kLean) {
            for (uint32_t e0 = beg + lane_g; __any(e0 < end); e0 += G * K) {
              uint32_t vv[K], cw[K], old[K];
#pragma unroll
              for (int j = 0; j < K; ++j) {
                const uint32_t e = e0 + j * G;
                const uint32_t raw = e < end ? g.adj[e] : kEdgeDown;  // masked: padding lanes issue no load
                vv[j] = (raw & kEdgeDown) ? V : raw;                  // padding / down edge: the sentinel
              }
#pragma unroll
              for (int j = 0; j < K; ++j) cw[j] = st[S::word(vv[j])];
#pragma unroll
              for (int j = 0; j < K; ++j) {
                const uint32_t c = (cw[j] >> S::shift(vv[j])) & kCodeMask;
                const bool tight = c == 0u || c == cnext;  // first or equal-cost arrival (LinkState.cpp:857-873)
                old[j] = atomicOr(tight ? &st[S::word(vv[j])] : &dummy[lane], xu << S::shift(vv[j]));
              }
              __builtin_amdgcn_sched_barrier(0);  // the K atomics in flight together
              bool fresh[K];
              unsigned long long bj[K];
              uint32_t off[K + 1];
              off[0] = 0;
#pragma unroll
              for (int j = 0; j < K; ++j) {
                fresh[j] = ((old[j] >> S::shift(vv[j])) & kCodeMask) == 0u;  // a dummy field never is
                bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
                off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
              }
              const uint32_t total = off[K];
              if (total) {  // wave-uniform
                const int leader = __ffsll((long long)__ballot(1)) - 1;
                uint32_t wbase = 0;
                if ((int)lane == leader) wbase = atomicAdd(cnt, total);
                const uint32_t base = tail + __builtin_amdgcn_readfirstlane(wbase);
                if (!RING || base + total - head <= ring_cap) {
#pragma unroll
                  for (int j = 0; j < K; ++j) {
                    if (fresh[j]) {
                      const uint32_t slot = base + off[j] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                      ring[RING ? (slot & rmask) : slot] = (uint16_t)vv[j];
                    }
                  }
                } else if ((int)lane == leader) {
                  ctl[4] = 1;  // two adjacent levels exceed the ring
                }
              }
            }
            continue;
          }
          for (uint32_t e0 = (ELLM == 2 ? 0u : beg) + lane_g; __any(e0 < end); e0 += G * K) {
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
            // (1) tight test: the K field reads are issued together (every vv[j] is a
            //     valid node id, padding included, so no address select is needed)
            bool tight[K];
            uint32_t vv[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j * G;
              vv[j] = av[j] & ~(kEdgeDown | kNodeSink);  // always a valid node id
              const bool ok = !(av[j] & kEdgeDown) && (ELLM == 2 || e < end) && !(has_ign && test_bit(ign, lv[j]));
              const uint32_t c = S::field(st, vv[j]) & kCodeMask;
              tight[j] = ok && (c == 0u || c == cnext);  // first or equal-cost arrival (LinkState.cpp:857-873)
            }
#ifdef OPENR_SPF_PROFILE
            OPENR_PROF_STAMP(t2);
            OPENR_PROF_ADD(1, t1, t2);
#endif
            // (2) addNextHops(nh(u)) + level code + election of the appending arrival:
            //     K atomics in flight together; non-tight edges OR 0 into the lane's
            //     own dummy word
            uint32_t old[K];
#pragma unroll
            for (int j = 0; j < K; ++j)
              old[j] = atomicOr(tight[j] ? &st[S::word(vv[j])] : &dummy[lane], tight[j] ? xu << S::shift(vv[j]) : 0u);
            bool fresh[K];  // this arrival appends v (kept as lane masks: ballots read them directly)
#pragma unroll
            for (int j = 0; j < K; ++j) {
              fresh[j] = tight[j] && ((old[j] >> S::shift(vv[j])) & kCodeMask) == 0u;
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
        cnext = cnext == 3u ? 1u : cnext + 1u;
        if (RING && ctl[4]) {  // ring overflow; ctl[4] is uniform after the barrier
          overflow = true;
          break;
        }
        if (tail == V) {
          // every node is reached: no edge out of level [head, tail) can be tight (its
          // heads are settled at levels <= L), so the level is only settled here
          if (own_dist)
            for (uint32_t i = head + tid; i < tail; i += BLOCK) put(ring[RING ? (i & rmask) : i], L);
          __builtin_amdgcn_wave_barrier();  // the per-thread loop joins before the break (uniform exit)
          break;
        }
        if (!SLICED && a.target && a.dist_only) {
          // the target is settled: every node nearer than it has its distance; the
          // target's level [head, tail) gets its distances here instead of on expansion
          const uint32_t t = a.target[sid];
          if (t < V && (S::field(st, t) & kCodeMask) != 0u) {
            for (uint32_t i = head + tid; i < tail; i += BLOCK) put(ring[RING ? (i & rmask) : i], L);
            __builtin_amdgcn_wave_barrier();
            break;
          }
        }
      }
      if (RING && overflow) {  // re-run by the full-order variant (from the list)
        if (tid == 0) a.ovf_list[atomicAdd(ovf_count, 1u)] = uid;
      } else {
#ifdef OPENR_SPF_PROFILE
        OPENR_PROF_STAMP(t0);
#endif
        write_out<FB, BLOCK, SLICED, GENERIC>(a, k, sid, slice, V, st, nt != 0);
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

struct BfsShape {
  uint32_t block = 256, ring_cap = 0, per_cu = 1;  // ring_cap == 0: full BFS order
};

// As many solves per CU as LDS allows (<= 32 waves; 128-thread workgroups when more than
// 8 fit). At each occupancy the full-order queue (never overflows) is preferred when it
// fits, else a ring wide enough for the graph's estimated two-level frontier
// (g.est_width2, sampled on the host) — a ring that overflows re-runs its solves, which
// costs more than the occupancy it buys (fabric: levels of thousands of nodes).
BfsShape bfs_shape(const DevGraph& g, bool has_ign, uint32_t fb) {
  BfsShape sh;
  const uint32_t fixed = bfs_layout(g.V, g.L, has_ign, fb, 0).total;
  const uint32_t full = bfs_layout(g.V, g.L, has_ign, fb, g.V).total;
  const uint32_t need = std::max<uint32_t>(std::max<uint32_t>(256u, g.max_deg + 2u), g.est_width2 + g.est_width2 / 4u);
  const bool force_full = env_u32("OPENR_SPF_BFS_FULL", 0u, 0u, 1u) != 0u;
  for (uint32_t want = 16u; want >= 1; --want) {
    const uint32_t budget = kMaxLds / want;
    sh.per_cu = want;
    if (full <= budget) {
      sh.ring_cap = 0;
      break;
    }
    if (force_full || budget <= fixed) continue;
    uint32_t cap = 1;
    while (cap * 2u <= (budget - fixed) / 2u && cap < 4096u) cap *= 2u;
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
  sh.block = sh.per_cu > 8u ? 128u : 256u;
  return sh;
}

template <int FB, int BLOCK, bool RING, int ELLM, bool SLICED>
hipError_t launch_bfs_variant(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                              uint32_t ring_cap, bool from_list, uint32_t* ctr, uint32_t* ovf_count, int num_cus,
                              hipStream_t s, LaunchInfo* info) {
  const uint32_t lds = bfs_layout(g.V, g.L, has_ign, FB, ring_cap).total;
  // a re-run covers only the listed units (usually none): one workgroup per CU is plenty
  const uint32_t grid = from_list ? std::min<uint32_t>(blocks_for(a.n * (SLICED ? a.nsl : 1u), lds, num_cus, BLOCK),
                                                       (uint32_t)num_cus)
                                  : blocks_for(a.n * (SLICED ? a.nsl : 1u), lds, num_cus, BLOCK);
  const bool generic = has_ign || a.tight != nullptr;
  auto k = generic ? bfs_code_kernel<FB, BLOCK, RING, ELLM == 2 ? 1 : ELLM, true, SLICED>
                   : bfs_code_kernel<FB, BLOCK, RING, ELLM, false, SLICED>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  if (info && !from_list) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = RING ? "bfs_code_kernel<ring>" : "bfs_code_kernel<full>";
  }
  note_launch(RING ? "bfs_code_kernel<ring>" : from_list ? "bfs_code_kernel<full>:rerun" : "bfs_code_kernel<full>");
  hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), lds, s, g, a, cost, glog, (uint32_t)has_ign, ring_cap,
                     (uint32_t)from_list, ctr, ovf_count, nt_stores());
  return hipGetLastError();
}

template <int FB, int BLOCK, int ELLM, bool SLICED>
hipError_t launch_bfs_shape(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign,
                            uint32_t ring_cap, int num_cus, hipStream_t s, LaunchInfo* info) {
  // Counter block of the class: [0,1] first launch, [2,3] re-run launch, [4] listed units.
  uint32_t* blk = class_counters(a);
  if (!ring_cap)
    return launch_bfs_variant<FB, BLOCK, false, ELLM, SLICED>(g, a, cost, glog, has_ign, g.V, false, blk, blk + 4,
                                                              num_cus, s, info);
  hipError_t err = launch_bfs_variant<FB, BLOCK, true, ELLM, SLICED>(g, a, cost, glog, has_ign, ring_cap, false, blk,
                                                                     blk + 4, num_cus, s, info);
  if (err != hipSuccess || g.V <= ring_cap) return err;  // a ring of >= V slots never overflows
  return launch_bfs_variant<FB, 256, false, ELLM, SLICED>(g, a, cost, glog, has_ign, g.V, true, blk + 2, blk + 4,
                                                          num_cus, s, info);
}

template <int FB, bool SLICED>
hipError_t launch_bfs_fb(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, bool has_ign, int ellm,
                         int num_cus, hipStream_t s, LaunchInfo* info) {
  const BfsShape sh = bfs_shape(g, has_ign, FB);
#define OPENR_BFS_SHAPE(BLK, E) \
  return launch_bfs_shape<FB, BLK, E, SLICED>(g, a, cost, glog, has_ign, sh.ring_cap, num_cus, s, info)
  // A batch of at most half as many (solve, slice) units as CUs (a refresh's few affected
  // rows, LFA / KSP prefetches of one node): a launch is one solve's latency, so each solve
  // takes a whole CU — 1 024 threads, full-order queue — instead of 256 threads beside
  // idle CUs
  const uint64_t units = (uint64_t)a.n * (SLICED ? std::max(a.nsl, 1u) : 1u);
  if (units * 2u <= (uint64_t)num_cus && bfs_layout(g.V, g.L, has_ign, FB, g.V).total <= kMaxLds) {
    if (ellm == 2) return launch_bfs_shape<FB, 1024, 2, SLICED>(g, a, cost, glog, has_ign, 0u, num_cus, s, info);
    if (ellm == 1) return launch_bfs_shape<FB, 1024, 1, SLICED>(g, a, cost, glog, has_ign, 0u, num_cus, s, info);
    return launch_bfs_shape<FB, 1024, 0, SLICED>(g, a, cost, glog, has_ign, 0u, num_cus, s, info);
  }
  // High-degree graphs (G > 1 lanes per frontier node, CSR rows) with at most 8 solves per
  // CU by LDS, full solves (no ignore set, no target): 512-thread workgroups, four per CU —
  // fewer solves in flight, each with twice the lanes (fabric 16-bit class: all-sources
  // launch 0.628 -> 0.601 ms). The KSP2 second SPFs (ignore set + target) keep 256 threads
  // (fabric all pairs 2 453 vs 2 504 ms with 512). OPENR_SPF_BFS_BLOCK=256 (tests, A/B): the
  // 256-thread shape everywhere.
  if (ellm == 0 && sh.block == 256 && !has_ign && !a.target &&
      env_u32("OPENR_SPF_BFS_BLOCK", 512u, 256u, 512u) == 512u)
    OPENR_BFS_SHAPE(512, 0);
  if (sh.block == 128) {
    if (ellm == 2) OPENR_BFS_SHAPE(128, 2);
    if (ellm == 1) OPENR_BFS_SHAPE(128, 1);
    OPENR_BFS_SHAPE(128, 0);
  }
  if (ellm == 2) OPENR_BFS_SHAPE(256, 2);
  if (ellm == 1) OPENR_BFS_SHAPE(256, 1);
  OPENR_BFS_SHAPE(256, 0);
#undef OPENR_BFS_SHAPE
}

// Sliced class, next-hop output: byte jj of node v's set is bits [8jj, 8jj + 8) of the
// concatenated 29-bit slice chunks. A workgroup takes 256 nodes of one solve: each thread
// reads its node's chunks (coalesced) and assembles its nb bytes in LDS, then the
// workgroup stores the 256 * nb bytes of the row segment as coalesced dwords.
__global__ __launch_bounds__(256) void slice_merge(SolveArgs a, uint32_t V) {
  constexpr uint32_t kMaxNb = 40u;  // 11 slices x 29 bits; wider caller strides store directly
  __shared__ uint32_t seg[256u * kMaxNb / 4u];
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  const uint32_t nsl = a.nsl, nb = a.nh_bytes, tiles = (V + 255u) / 256u;
  // this chunk's solves [k0, k0 + in_chunk) of the class
  const uint32_t in_chunk = !a.krows ? count : count > a.k0 ? min(a.krows, count - a.k0) : 0u;
  uint8_t* segb = reinterpret_cast<uint8_t*>(seg);
  for (uint64_t blk = blockIdx.x; blk < (uint64_t)in_chunk * tiles; blk += gridDim.x) {
    const uint32_t kc = (uint32_t)(blk / tiles), v0 = (uint32_t)(blk - (uint64_t)kc * tiles) * 256u;
    const uint32_t k = a.k0 + kc;
    const uint32_t sid = a.perm ? a.perm[first + k] : k;
    const uint32_t* t = a.slice_tmp + (size_t)kc * nsl * V;
    const uint32_t nv = std::min<uint32_t>(256u, V - v0), v = v0 + threadIdx.x;
    uint8_t* dst = a.nh + out_row_of(a, sid) * (size_t)V * nb + (size_t)v0 * nb;
    const bool staged = nb <= kMaxNb;
    if (threadIdx.x < nv) {
      uint8_t* out = staged ? segb + threadIdx.x * nb : dst + (size_t)threadIdx.x * nb;
      uint64_t acc = 0;
      uint32_t have = 0, sl = 0;
      for (uint32_t j = 0; j < nb; ++j) {
        while (have < 8u && sl < nsl) {
          acc |= (uint64_t)t[(size_t)sl * V + v] << have;
          have += 29u;
          ++sl;
        }
        out[j] = (uint8_t)acc;
        acc >>= 8;
        have = have >= 8u ? have - 8u : 0u;
      }
    }
    if (!staged) continue;  // block-uniform
    __syncthreads();
    const uint32_t bytes = nv * nb;
    if ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0) {
      for (uint32_t i = threadIdx.x; i < bytes / 4u; i += 256u) reinterpret_cast<uint32_t*>(dst)[i] = seg[i];
      for (uint32_t i = (bytes & ~3u) + threadIdx.x; i < bytes; i += 256u) dst[i] = segb[i];
    } else {
      for (uint32_t i = threadIdx.x; i < bytes; i += 256u) dst[i] = segb[i];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Wide pass: the sliced class (next-hop sets wider than 29 bits) in ONE unit per solve.
// The sliced pass runs a source's BFS once per 29-bit slice (a degree-84 fabric switch:
// three full traversals) and merges the slices' scratch rows afterwards (slice_merge).
// Here the node state is a multi-word bit stream per node: word 0 = [29 next-hop bits |
// 3-bit level code] exactly as the 32-bit class, words 1..nw-1 = the next 32 bits each
// (next-hop bit b sits at stream position b + 3). The tight test, the first-arrival
// election and the append read word 0 only, so the BFS order is computed once; a tight
// edge then ORs nh(u)'s upper words into v's (plain ds_or, no return, only where u's word
// is non-zero — on a fabric most sets span one or two words). The row is written straight
// from LDS: byte j of v's set is stream bits [8j + 3, 8j + 11), assembled a dword of the
// output row per lane — no slice scratch, no merge launch. Lean edge loop only (no ignore
// set, no tight-edge output; CSR rows, G lanes per frontier node as the lean pass); full
// BFS order (never wraps).
// ---------------------------------------------------------------------------
struct WideLayout {
  uint32_t st, ext, ring, dummy, total;
};
__host__ __device__ inline WideLayout wide_layout(uint32_t V, uint32_t nw) {
  WideLayout l;
  uint32_t off = 32;  // control: append counters [0..3]
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.st = take(4u * (V + 1u));  // + node V: the settled sentinel
  l.ext = take(4u * V * (nw - 1u));
  l.ring = take(2u * V);
  l.dummy = take(4u * 64u);
  l.total = off;
  return l;
}

template <int BLOCK, uint32_t NW>
__global__ __launch_bounds__(BLOCK) void bfs_wide_kernel(DevGraph g, SolveArgs a, uint64_t cost, uint32_t glog,
                                                         uint32_t nw, uint32_t* ctr, uint32_t nt) {
  using S = State<32>;
  constexpr int K = (int)kBfsEdgesPerLane;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t s_next;
  const uint32_t V = g.V, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = __lane_id();
  const WideLayout lay = wide_layout(V, nw);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* ctl = smem;
  uint32_t* st = reinterpret_cast<uint32_t*>(base + lay.st);
  uint32_t* ext = reinterpret_cast<uint32_t*>(base + lay.ext);  // [nw - 1][V]
  uint16_t* ring = reinterpret_cast<uint16_t*>(base + lay.ring);
  uint32_t* dummy = reinterpret_cast<uint32_t*>(base + lay.dummy);
  if (tid < 64) dummy[tid] = 0xFFFFFFFFu;
  const uint32_t G = 1u << glog, ngroups = BLOCK >> glog, groups_per_wave = 64u >> glog;
  const uint32_t group = tid >> glog, lane_g = tid & (G - 1u);
  const uint32_t ne = nw - 1u;  // upper words (nw <= NW, the compiled bound)
  const uint32_t count = a.perm ? a.part[a.cls] : a.n, first = a.perm ? a.part[kMaxClasses + a.cls] : 0u;
  for (uint32_t unit = blockIdx.x; unit < count;) {
    const uint32_t sid = a.perm ? a.perm[first + unit] : unit;
    const uint32_t src = a.sources[sid];
    if (src < V) {  // block-uniform
      uint64_t* drow = a.dist + out_row_of(a, sid) * V;
      for (uint32_t i = tid; i < V + 1u; i += BLOCK) st[i] = 0;
      for (uint32_t i = tid; i < ne * V; i += BLOCK) ext[i] = 0;
      if (tid < 8) ctl[tid] = 0;
      __syncthreads();
      if (tid == 0) {
        st[V] = kCodeSettledSink;  // the sentinel
        st[src] = level_code(0);
        drow[src] = 0;
      }
      __syncthreads();
      // level 0: the source's own row (even when overloaded); a directly connected node's
      // next hop is the node itself (LinkState.cpp:867-872)
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
              const uint32_t pos = g.nbr[e] + S::kNhs, w = pos >> 5;
              fresh = (atomicOr(&st[v], (w == 0u ? 1u << pos : 0u) | level_code(1)) & kCodeMask) == 0u;
              if (w != 0u) atomicOr(&ext[(w - 1u) * V + v], 1u << (pos & 31u));
            }
          }
          const uint32_t slot = 1u + wave_append(fresh, &ctl[0]);
          if (fresh) ring[slot] = (uint16_t)v;  // slot < 1 + deg(src) <= V
        }
      }
      __syncthreads();
      uint32_t head = 1, tail = 1u + ctl[0], L = 1, cnext = level_code(2);
      while (head < tail) {
        uint32_t* cnt = &ctl[L & 3u];
        if (tid == 0) ctl[(L + 1u) & 3u] = 0;  // last read three barriers ago
        const uint64_t dL = (uint64_t)L * cost;
        for (uint32_t fb = head; fb < tail; fb += ngroups) {
          if (fb + wave * groups_per_wave >= tail) continue;  // this wave has no frontier node (uniform)
          const uint32_t idx = fb + group;
          const bool live = idx < tail;
          uint32_t u = V, beg = 0, end = 0;
          if (live) {
            u = ring[idx];
            const uint2 r = g.row2t[u];  // empty (beg flagged kNodeSink) for overloaded nodes
            beg = r.x;
            end = r.y;
            if (lane_g == 0) {
              drow[u] = dL;  // u settled on level L
              if (beg & kNodeSink) atomicOr(&st[u], kCodeSettledSink);
            }
          }
          // nh(u) (final: u was reached a level ago): word 0 + the code of level L+1, and
          // the upper words (the sentinel's, for a lane past the level, are never used)
          const uint32_t xu = (st[u] & S::kNhMask) | cnext;
          uint32_t xe[NW - 1u];
#pragma unroll
          for (uint32_t s = 0; s < NW - 1u; ++s) xe[s] = (s < ne && live) ? ext[s * V + u] : 0u;
          for (uint32_t e0 = beg + lane_g; __any(e0 < end); e0 += G * K) {
            uint32_t vv[K], cw[K], old[K];
            bool tight[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t e = e0 + j * G;
              const uint32_t raw = e < end ? g.adj[e] : kEdgeDown;
              vv[j] = (raw & kEdgeDown) ? V : raw;  // padding / down edge: the sentinel
            }
#pragma unroll
            for (int j = 0; j < K; ++j) cw[j] = st[vv[j]];
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const uint32_t c = cw[j] & kCodeMask;
              tight[j] = c == 0u || c == cnext;  // first or equal-cost arrival (LinkState.cpp:857-873)
              old[j] = atomicOr(tight[j] ? &st[vv[j]] : &dummy[lane], xu);
            }
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
              for (uint32_t s = 0; s < NW - 1u; ++s)
                if (tight[j] && xe[s]) atomicOr(&ext[s * V + vv[j]], xe[s]);
            bool fresh[K];
            unsigned long long bj[K];
            uint32_t off[K + 1];
            off[0] = 0;
#pragma unroll
            for (int j = 0; j < K; ++j) {
              fresh[j] = (old[j] & kCodeMask) == 0u;  // a dummy word never is
              bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
              off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
            }
            const uint32_t total = off[K];
            if (total) {  // wave-uniform
              const int leader = __ffsll((long long)__ballot(1)) - 1;
              uint32_t wbase = 0;
              if ((int)lane == leader) wbase = atomicAdd(cnt, total);
              const uint32_t slot0 = tail + __builtin_amdgcn_readfirstlane(wbase);
#pragma unroll
              for (int j = 0; j < K; ++j) {
                if (fresh[j]) {
                  const uint32_t slot = slot0 + off[j] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                  ring[slot] = (uint16_t)vv[j];
                }
              }
            }
          }
        }
        lds_barrier();
        head = tail;
        tail += *cnt;
        ++L;
        cnext = cnext == 3u ? 1u : cnext + 1u;
        if (tail == V) {
          // every node is reached: no edge out of level [head, tail) can be tight
          for (uint32_t i = head + tid; i < tail; i += BLOCK) drow[ring[i]] = (uint64_t)L * cost;
          break;
        }
      }
      // rows out: UINT64_MAX for unreached nodes, then the next-hop bytes, a dword of the
      // row per lane (byte q of the dword: node (4i + q) / nb, byte (4i + q) % nb)
      for (uint32_t v = tid; v < V; v += BLOCK)
        if ((st[v] & kCodeMask) == 0u) drow[v] = ~0ull;
      const uint32_t nb = a.nh_bytes;
      uint8_t* nrow = a.nh + out_row_of(a, sid) * V * nb;
      // 32 bits of v's stream from bit p (p >= 3: never the code)
      auto bits32 = [&](uint32_t v, uint32_t p) -> uint32_t {
        const uint32_t w = p >> 5, sh = p & 31u;
        const uint32_t lo = w == 0u ? st[v] : w < nw ? ext[(w - 1u) * V + v] : 0u;
        const uint32_t hi = w + 1u < nw ? ext[w * V + v] : 0u;
        return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
      };
      const uint32_t row_bytes = V * nb;
      if (((reinterpret_cast<uintptr_t>(nrow) | row_bytes) & 3u) == 0) {
        uint32_t* n32 = reinterpret_cast<uint32_t*>(nrow);
        for (uint32_t i = tid; i < row_bytes / 4u; i += BLOCK) {
          const uint32_t p = 4u * i, v = p / nb, j = p - v * nb, n0 = min(4u, nb - j);
          uint32_t x = bits32(v, 8u * j + S::kNhs);
          if (n0 < 4u) x = (x & ((1u << (8u * n0)) - 1u)) | (bits32(v + 1u, S::kNhs) << (8u * n0));
          store_row<uint32_t>(&n32[i], x, nt != 0);
        }
      } else {
        for (uint32_t i = tid; i < row_bytes; i += BLOCK) {
          const uint32_t v = i / nb, j = i - v * nb;
          nrow[i] = (uint8_t)bits32(v, 8u * j + S::kNhs);
        }
      }
    }
    __syncthreads();  // every lane is done with this unit's LDS and s_next
    if (tid == 0) s_next = gridDim.x + atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unit = s_next;
  }
  retire_workgroup(ctr, nullptr);
}

// Upper words of the wide pass for a class of nsl 29-bit slices (bits <= 29 * nsl).
uint32_t wide_words(uint32_t nsl) { return 1u + (29u * (nsl - 1u) + 31u) / 32u; }

template <int BLOCK, uint32_t NW>
hipError_t launch_wide_nw(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, uint32_t nw,
                          int num_cus, hipStream_t s, LaunchInfo* info) {
  const uint32_t lds = wide_layout(g.V, nw).total;
  const uint32_t grid = blocks_for(a.n, lds, num_cus, BLOCK);
  auto k = bfs_wide_kernel<BLOCK, NW>;
  hipError_t err =
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = "bfs_wide_kernel";
  }
  note_launch("bfs_wide_kernel");
  hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), lds, s, g, a, cost, glog, nw, class_counters(a), nt_stores());
  return hipGetLastError();
}

template <int BLOCK>
hipError_t launch_wide(const DevGraph& g, const SolveArgs& a, uint64_t cost, uint32_t glog, uint32_t nw, int num_cus,
                       hipStream_t s, LaunchInfo* info) {
  if (nw <= 2u) return launch_wide_nw<BLOCK, 2>(g, a, cost, glog, nw, num_cus, s, info);
  if (nw <= 3u) return launch_wide_nw<BLOCK, 3>(g, a, cost, glog, nw, num_cus, s, info);
  if (nw <= 4u) return launch_wide_nw<BLOCK, 4>(g, a, cost, glog, nw, num_cus, s, info);
  return launch_wide_nw<BLOCK, 8>(g, a, cost, glog, nw, num_cus, s, info);
}

uint32_t field_bits(int cls) { return cls == kCls8 ? 8u : cls == kCls16 ? 16u : 32u; }
}  // namespace

uint32_t bfs_code_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int cls) {
  // the full-order variant must fit (it re-runs solves the fast path flags)
  if (V > 65535u || cls < 0 || cls >= kNumClasses) return 0;
  const uint32_t t = bfs_layout(V, L, has_ignore, field_bits(cls), V).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_bfs_code(const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes, int num_cus,
                           hipStream_t s, LaunchInfo* info) {
  const bool has_ign = a.ign_ptr != nullptr;
  const int cls = (int)a.cls;
  if (!bfs_code_lds_bytes(g.V, g.L, has_ign, cls)) return hipErrorInvalidValue;
  const bool sliced = cls == kClsSliced;
  if (sliced && (a.nsl < 1u || a.nsl > 11u)) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  if (!a.ovf_list || !a.work) return hipErrorInvalidValue;
  uint32_t glog = 0;
  while ((1 << glog) < group_lanes && glog < 6) ++glog;
  // ELL: one lane per frontier node; ELL-only when every row fits the 4 ELL slots
  const int ellm = glog != 0 ? 0 : (g.max_deg <= 4u ? 2 : 1);
  switch (field_bits(cls)) {
    case 8: return launch_bfs_fb<8, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
    case 16: return launch_bfs_fb<16, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
    default:
      if (sliced) {
        // the wide pass (one unit per solve) where it applies: next-hop output, lean edge
        // loop (no ignore set / tight-edge output), sets of <= 8 words, the full-order state
        // in LDS. 512-thread workgroups (fabric 5 000: 0.632 ms per all-sources launch vs
        // 0.706 with 256 and 0.651 with 1 024; sliced pass 0.790). OPENR_SPF_WIDE (tests,
        // A/B): 0 = the sliced pass, 2 = 256-thread workgroups.
        const uint32_t nw = wide_words(a.nsl);
        const uint32_t wide = env_u32("OPENR_SPF_WIDE", 1u, 0u, 2u);
        if (a.nh && !has_ign && !a.tight && nw <= 8u && wide_layout(g.V, nw).total <= kMaxLds && wide != 0u) {
          if (wide == 2u) return launch_wide<256>(g, a, cost, glog, nw, num_cus, s, info);
          return launch_wide<512>(g, a, cost, glog, nw, num_cus, s, info);
        }
        if (!a.nh) {  // no next-hop output: no slice scratch, one launch
          SolveArgs c = a;
          c.k0 = c.krows = 0;
          return launch_bfs_fb<32, true>(g, c, cost, glog, has_ign, ellm, num_cus, s, info);
        }
        if (!a.slice_tmp) return hipErrorInvalidValue;
        // the class in chunks of krows solves (slice_tmp holds one chunk; the launcher sized
        // krows from its scratch budget); chunks past the class's device-side count exit at once
        const uint32_t rows = a.krows ? a.krows : std::max(a.n, 1u);
        for (uint32_t k0 = 0; k0 < a.n; k0 += rows) {
          SolveArgs c = a;
          c.k0 = k0;
          c.krows = rows;
          hipError_t err = launch_bfs_fb<32, true>(g, c, cost, glog, has_ign, ellm, num_cus, s, info);
          if (err != hipSuccess) return err;
          const uint64_t items = (uint64_t)std::min(rows, a.n - k0) * ((g.V + 255u) / 256u);  // (solve, 256-node tile) pairs
          const uint32_t grid = (uint32_t)std::min<uint64_t>(items, 8192u);
          hipLaunchKernelGGL(slice_merge, dim3(std::max(grid, 1u)), dim3(256), 0, s, c, g.V);
          err = hipGetLastError();
          if (err != hipSuccess) return err;
        }
        return hipSuccess;
      }
      return launch_bfs_fb<32, false>(g, a, cost, glog, has_ign, ellm, num_cus, s, info);
  }
}

}  // namespace openr_spf
