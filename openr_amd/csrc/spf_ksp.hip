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
// Shape: one wavefront per (src, dest) pair. Instead of the reference's backtracking
// DFS, the kernel keeps the exact set of nodes that can still be reached from src over
// unused tight edges ("dead" = not), so each traceOnePath is a straight descent from
// dest (see descend()); after a path is found its links are used and the nodes that
// lose their last live pathLink are killed by a decremental sweep down the tight DAG
// (kill_unreachable). Visited links and dead nodes are LDS bitmaps.
//
// Output tokens per pair (ReadMe: include/openr_spf.h openr_spf_ksp2): [n_paths,
// len_0, edges_0..., len_1, edges_1..., ...], directed edge ids in src -> dest order.
#include <algorithm>

#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {
using namespace dev;

constexpr uint32_t kWave = 64;
constexpr uint64_t kNoKey = ~0ull;

struct KspLayout {
  uint32_t vis, dead, path, work, total;
};

__host__ __device__ inline KspLayout ksp_layout(uint32_t V, uint32_t L) {
  KspLayout l;
  uint32_t off = 16;  // control: [0] worklist tail
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  l.vis = take(4u * ((L + 31u) / 32u));
  l.dead = take(4u * ((V + 31u) / 32u));
  l.path = take(4u * kKspMaxDepth);
  l.work = take(2u * V);
  l.total = off;
  return l;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}

struct KspState {
  const DevGraph* g;
  uint32_t src;
  const uint64_t* drow;
  uint32_t* ctl;
  uint32_t* vis;   // used links: visited by found paths (+ the k = 1 links for k = 2)
  uint32_t* dead;  // nodes that can no longer be reached from src over unused tight edges
  uint32_t* path;
  uint16_t* work;
};

// Tight in-edge u->v (e = v's row entry for v->u, re = rev[e] = u->v) usable as a
// pathLink now: edge up, link unused, u may expand, dist[u] + w(u->v) == dist[v], u alive.
__device__ __forceinline__ bool live_pred(const KspState& st, uint32_t e, uint64_t dv, uint32_t* u_out,
                                          uint64_t* du_out) {
  const DevGraph& g = *st.g;
  const uint32_t av = g.adj[e];
  const uint32_t u = av & ~kEdgeDown;
  *u_out = u;
  if ((av & kEdgeDown) || test_bit(st.vis, g.lid[e]) || (u != st.src && g.ovl[u]) || test_bit(st.dead, u))
    return false;
  const uint64_t du = st.drow[u];
  *du_out = du;
  return du != kNoKey && du + g.win[e] == dv;
}

// Does v keep a live pathLink? (lanes over v's in-edges; wave-uniform result)
__device__ bool has_live_pred(const KspState& st, uint32_t v) {
  const DevGraph& g = *st.g;
  const uint64_t dv = st.drow[v];
  const uint2 r = g.row2[v];
  for (uint32_t e = r.x + threadIdx.x; __any(e < r.y); e += kWave) {
    uint32_t u;
    uint64_t du;
    const bool ok = e < r.y && live_pred(st, e, dv, &u, &du);
    if (__any(ok)) return true;
  }
  return false;
}

// The links of a found path are now used: nodes left without a live pathLink die, and
// their death is pushed down their tight out-edges (decremental reachability from src
// over the tight DAG). Keeps `dead` exact, so the next descent never backtracks.
__device__ void kill_unreachable(const KspState& st, uint32_t len) {
  const DevGraph& g = *st.g;
  const uint32_t lane = threadIdx.x;
  uint32_t head = 0, tail = 0;
  // heads of the path's edges lost an in-edge (path[i] = edge u->v, src side first)
  for (uint32_t i = 0; i < len; ++i) {
    const uint32_t v = g.adj[st.path[i]] & ~kEdgeDown;  // head of u->v
    if (v == st.src || test_bit(st.dead, v) || has_live_pred(st, v)) continue;
    if (lane == 0) {
      st.dead[v >> 5] |= 1u << (v & 31u);
      st.work[tail] = (uint16_t)v;
    }
    lds_fence();
    ++tail;
  }
  while (head < tail) {
    const uint32_t b = st.work[head++];
    if (b != st.src && g.ovl[b]) continue;  // a sink never expanded: no tight out-edges
    const uint64_t db = st.drow[b];
    const uint2 r = g.row2[b];
    for (uint32_t e0 = r.x; e0 < r.y; e0 += kWave) {
      const uint32_t e = e0 + lane;
      uint32_t c = 0;
      bool cand = false;
      if (e < r.y) {
        const uint32_t av = g.adj[e];
        c = av & ~kEdgeDown;
        cand = !(av & kEdgeDown) && !test_bit(st.vis, g.lid[e]) && c != st.src && !test_bit(st.dead, c) &&
               st.drow[c] != kNoKey && db + g.w[e] == st.drow[c];
      }
      unsigned long long m = __ballot(cand);
      while (m) {  // re-check each tight successor, one at a time (all lanes help)
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const uint32_t cc = __shfl(c, l);
        if (test_bit(st.dead, cc) || has_live_pred(st, cc)) continue;
        if (lane == 0) {
          st.dead[cc >> 5] |= 1u << (cc & 31u);
          st.work[tail] = (uint16_t)cc;
        }
        lds_fence();
        ++tail;
      }
    }
  }
}

// One traceOnePath (LinkState.cpp:398-419) given exact liveness: from dest, take the
// first pathLink in the reference's order whose link is unused and whose tail is live,
// down to src. The reference's DFS would also try (and mark) links into dead tails and
// backtrack out of them; such links lead to nodes that can never reach src again, so
// skipping them finds the same path and leaves every later trace unchanged.
// Returns the path length (edges in path[0..len), src side first), 0 for no path,
// -1 when the path is longer than kKspMaxDepth (or liveness was inconsistent).
__device__ int descend(const KspState& st, uint32_t dst) {
  const DevGraph& g = *st.g;
  const uint32_t lane = threadIdx.x;
  uint32_t v = dst, len = 0;
  while (v != st.src) {
    const uint64_t dv = st.drow[v];
    const uint2 r = g.row2[v];
    uint64_t best_d = kNoKey, best_r = kNoKey;
    for (uint32_t e = r.x + lane; __any(e < r.y); e += kWave) {
      uint64_t kd = kNoKey, kr = kNoKey;
      uint32_t u;
      uint64_t du;
      if (e < r.y && live_pred(st, e, dv, &u, &du)) {
        kd = du;  // pathLinks order: pop order of u = (dist, name), then u's row order
        kr = ((uint64_t)g.rank[u] << 32) | g.rev[e];
      }
      const uint64_t md = wave_min_u64(kd);
      const uint64_t mr = wave_min_u64(kd == md ? kr : kNoKey);
      if (md < best_d || (md == best_d && mr < best_r)) {
        best_d = md;
        best_r = mr;
      }
    }
    if (best_d == kNoKey) return v == dst ? 0 : -1;  // a live node always has a live pathLink
    if (len >= kKspMaxDepth) return -1;
    const uint32_t re = (uint32_t)best_r;
    const uint32_t link = g.lid[re];
    if (lane == 0) {
      st.vis[link >> 5] |= 1u << (link & 31u);
      st.path[kKspMaxDepth - 1u - len] = re;  // filled dest side first
    }
    lds_fence();
    ++len;
    v = g.adj[g.rev[re]] & ~kEdgeDown;  // pathLink.prevNode = tail of re
  }
  // move to path[0..len), src side first
  for (uint32_t i = lane; i < len; i += kWave) {
    const uint32_t x = st.path[kKspMaxDepth - len + i];
    st.path[i] = x;  // i < kKspMaxDepth - len + i: reads stay ahead of writes within a chunk
  }
  lds_fence();
  return (int)len;
}

// Pairs [first, first + n) of a chunk; k = pair - first.
// KIND 1: k = 1 over the base rows (row = prow[pair]); the links of the paths found are
//         written to ign_io[k * ign_cap, ign_end[k]).
// KIND 2: k = 2 over the chunk's rows (row k); those links start out used (the second
//         SPF ignored them, so they are no pathLinks either).
template <int KIND>
__global__ __launch_bounds__(kWave) void ksp_trace_kernel(DevGraph g, const uint32_t* sources, const uint32_t* prow,
                                                          const uint32_t* pdst, uint32_t first, uint32_t n,
                                                          const uint64_t* rows, uint32_t* ign_io, uint32_t* ign_end,
                                                          uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap,
                                                          uint32_t* status) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V;
  const KspLayout lay = ksp_layout(V, g.L);
  char* base = reinterpret_cast<char*>(smem);
  KspState st;
  st.g = &g;
  st.ctl = smem;
  st.vis = reinterpret_cast<uint32_t*>(base + lay.vis);
  st.dead = reinterpret_cast<uint32_t*>(base + lay.dead);
  st.path = reinterpret_cast<uint32_t*>(base + lay.path);
  st.work = reinterpret_cast<uint16_t*>(base + lay.work);
  const uint32_t lane = threadIdx.x, lw = (g.L + 31u) / 32u, vw = (V + 31u) / 32u;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t pair = first + k;
    const uint32_t row = prow[pair];
    const uint32_t src = sources[row], dst = pdst[pair];
    st.src = src;
    st.drow = rows + (size_t)(KIND == 1 ? row : k) * V;
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
    bool bad = src >= V || dst >= V;
    // res.count(dest); src == dest traces an empty path, which ends the loop at once
    if (!bad && src != dst && st.drow[dst] != kNoKey) {
      for (;;) {
        const int len = descend(st, dst);
        if (len < 0) {
          bad = true;
          break;
        }
        if (len == 0) break;
        if (pos + 1u + (uint32_t)len > tok_cap || (KIND == 1 && nign + (uint32_t)len > ign_cap)) {
          bad = true;
          break;
        }
        for (uint32_t i = lane; i < (uint32_t)len; i += kWave) {
          const uint32_t e = st.path[i];
          out[pos + 1u + i] = e;
          if (KIND == 1) ig[nign + i] = g.lid[e];
        }
        if (lane == 0) out[pos] = (uint32_t)len;
        pos += 1u + (uint32_t)len;
        nign += (uint32_t)len;
        ++npaths;
        kill_unreachable(st, (uint32_t)len);
      }
    }
    if (lane == 0) {
      if (KIND == 1) ign_end[k] = k * ign_cap + (bad ? 0u : nign);
      out[0] = bad ? 0xFFFFFFFFu : npaths;
      if (bad) atomicOr(status, 1u);
    }
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

}  // namespace

uint32_t ksp_lds_bytes(uint32_t V, uint32_t L) {
  if (V > 65535u) return 0;
  const uint32_t t = ksp_layout(V, L).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_ksp_trace(int kind, const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                            const uint32_t* pdst, uint32_t first, uint32_t n, const uint64_t* rows, uint32_t* ign_io,
                            uint32_t* ign_end, uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap, uint32_t* status,
                            int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t lds = ksp_lds_bytes(g.V, g.L);
  if (!lds) return hipErrorInvalidValue;
  const uint32_t grid = blocks_for(n, lds, num_cus, kWave);
  auto k = kind == 1 ? ksp_trace_kernel<1> : ksp_trace_kernel<2>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWave), lds, s, g, sources, prow, pdst, first, n, rows, ign_io, ign_end,
                     ign_cap, tok, tok_cap, status);
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

}  // namespace openr_spf
