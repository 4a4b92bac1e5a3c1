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
// Shape: one wavefront per (src, dest) pair. A DFS frame keeps the key of the last
// pathLink it tried; the next one is the minimum key above it among v's in-edges, found
// with all 64 lanes (one in-edge each) and two wave min-reductions — so a frame costs
// O(1) LDS, and the DFS depth (hops of a shortest path) is bounded by kKspMaxDepth.
// The visited-link and ignore sets are LDS bitmaps over link ids.
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
  uint32_t vis, ign, st_node, st_edge, st_kd, st_kr, total;
};

__host__ __device__ inline KspLayout ksp_layout(uint32_t L, bool ign) {
  KspLayout l;
  uint32_t off = 16;
  auto take = [&](uint32_t bytes) {
    uint32_t o = off;
    off += (bytes + 15u) & ~15u;
    return o;
  };
  const uint32_t lw = (L + 31u) / 32u;
  l.vis = take(4u * lw);
  l.ign = ign ? take(4u * lw) : 0u;
  l.st_node = take(4u * kKspMaxDepth);
  l.st_edge = take(4u * kKspMaxDepth);
  l.st_kd = take(8u * kKspMaxDepth);
  l.st_kr = take(8u * kKspMaxDepth);
  l.total = off;
  return l;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// One DFS (traceOnePath). Returns the path length (>= 1) with the edges left in
// st_edge[1..len] (dest side first), 0 for src == dest, -1 for "no path", -2 for a DFS
// deeper than kKspMaxDepth. All values wave-uniform.
template <bool IGN>
__device__ int trace_one(const DevGraph& g, uint32_t src, uint32_t dst, const uint64_t* drow, uint32_t* vis,
                         const uint32_t* ign, uint32_t* st_node, uint32_t* st_edge, uint64_t* st_kd,
                         uint64_t* st_kr) {
  if (src == dst) return 0;
  const uint32_t lane = threadIdx.x;
  uint32_t sp = 1;
  if (lane == 0) st_node[0] = dst;
  lds_fence();
  bool first = true;  // the top frame has tried no pathLink yet (every key qualifies)
  while (sp > 0) {
    const uint32_t v = st_node[sp - 1];
    const uint64_t lkd = first ? 0ull : st_kd[sp - 1];
    const uint64_t lkr = first ? 0ull : st_kr[sp - 1];
    const bool any = first;  // first visit of this frame: every key qualifies
    const uint64_t dv = drow[v];
    const uint2 r = g.row2[v];
    // next pathLink of v after (lkd, lkr): min key over tight in-edges above it
    uint64_t best_d = kNoKey, best_r = kNoKey;
    for (uint32_t e = r.x + lane; __any(e < r.y); e += kWave) {
      uint64_t kd = kNoKey, kr = kNoKey;
      if (e < r.y) {
        const uint32_t av = g.adj[e];
        const uint32_t u = av & ~kEdgeDown;
        if (!(av & kEdgeDown) && !(IGN && test_bit(ign, g.lid[e])) && (u == src || !g.ovl[u])) {
          const uint64_t du = drow[u];
          if (du != kNoKey && du + g.win[e] == dv) {
            const uint32_t re = g.rev[e];
            const uint64_t rk = ((uint64_t)g.rank[u] << 32) | re;
            if (any || du > lkd || (du == lkd && rk > lkr)) {
              kd = du;
              kr = rk;
            }
          }
        }
      }
      const uint64_t md = wave_min_u64(kd);
      const uint64_t mr = wave_min_u64(kd == md ? kr : kNoKey);
      if (md < best_d || (md == best_d && mr < best_r)) {
        best_d = md;
        best_r = mr;
      }
    }
    if (best_d == kNoKey) {  // exhausted: std::nullopt back to the caller frame
      --sp;
      first = false;
      continue;
    }
    const uint32_t re = (uint32_t)best_r;
    const uint32_t link = g.lid[re];
    const bool fresh = !test_bit(vis, link);  // linksToIgnore.insert(link).second
    if (lane == 0) {
      st_kd[sp - 1] = best_d;
      st_kr[sp - 1] = best_r;
      if (fresh) vis[link >> 5] |= 1u << (link & 31u);
    }
    if (!fresh) {
      first = false;
      lds_fence();
      continue;
    }
    if (sp >= kKspMaxDepth) return -2;
    const uint32_t u = g.adj[g.rev[re]] & ~kEdgeDown;  // prevNode = tail of re
    if (lane == 0) {
      st_edge[sp] = re;
      st_node[sp] = u;
    }
    lds_fence();
    ++sp;
    first = true;
    if (u == src) return (int)(sp - 1);
  }
  return -1;
}

// Pairs [first, first + n) of a chunk; k = pair - first.
// KIND 1: k = 1 over the base rows (row = prow[pair]); the links of the paths found are
//         written to ign_io[k * ign_cap ..] (rest padded with 0xFFFFFFFF).
// KIND 2: k = 2 over the chunk's rows (row k), ignoring the links in ign_io[k].
template <int KIND>
__global__ __launch_bounds__(kWave) void ksp_trace_kernel(DevGraph g, const uint32_t* sources, const uint32_t* prow,
                                                          const uint32_t* pdst, uint32_t first, uint32_t n,
                                                          const uint64_t* rows, uint32_t* ign_io, uint32_t ign_cap,
                                                          uint32_t* tok, uint32_t tok_cap, uint32_t* status) {
  constexpr bool IGN = KIND == 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const KspLayout lay = ksp_layout(g.L, IGN);
  char* base = reinterpret_cast<char*>(smem);
  uint32_t* vis = reinterpret_cast<uint32_t*>(base + lay.vis);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  uint32_t* st_node = reinterpret_cast<uint32_t*>(base + lay.st_node);
  uint32_t* st_edge = reinterpret_cast<uint32_t*>(base + lay.st_edge);
  uint64_t* st_kd = reinterpret_cast<uint64_t*>(base + lay.st_kd);
  uint64_t* st_kr = reinterpret_cast<uint64_t*>(base + lay.st_kr);
  const uint32_t lane = threadIdx.x, lw = (g.L + 31u) / 32u, V = g.V;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t pair = first + k;
    const uint32_t row = prow[pair];
    const uint32_t src = sources[row], dst = pdst[pair];
    const uint64_t* drow = rows + (size_t)(KIND == 1 ? row : k) * V;
    uint32_t* out = tok + (size_t)pair * tok_cap;
    uint32_t* ig = ign_io + (size_t)k * ign_cap;  // chunk-local ignore slot
    for (uint32_t i = lane; i < lw; i += kWave) vis[i] = 0;
    if (IGN) {
      for (uint32_t i = lane; i < lw; i += kWave) ign[i] = 0;
      lds_fence();
      for (uint32_t i = lane; i < ign_cap; i += kWave) {
        const uint32_t l = ig[i];
        if (l < g.L) atomicOr(&ign[l >> 5], 1u << (l & 31u));
      }
    }
    lds_fence();
    uint32_t npaths = 0, pos = 1, nign = 0;
    bool bad = src >= V || dst >= V;
    if (!bad && drow[dst] != kNoKey) {  // res.count(dest)
      for (;;) {
        const int len = trace_one<IGN>(g, src, dst, drow, vis, ign, st_node, st_edge, st_kd, st_kr);
        if (len == -2) {
          bad = true;
          break;
        }
        if (len <= 0) break;  // while (path && !path->empty())
        if (pos + 1u + (uint32_t)len > tok_cap || (KIND == 1 && nign + (uint32_t)len > ign_cap)) {
          bad = true;
          break;
        }
        // st_edge[1..len] holds dest-side first: emit src -> dest
        for (uint32_t i = lane; i < (uint32_t)len; i += kWave) {
          const uint32_t e = st_edge[(uint32_t)len - i];
          out[pos + 1u + i] = e;
          if (KIND == 1) ig[nign + i] = g.lid[e];
        }
        if (lane == 0) out[pos] = (uint32_t)len;
        pos += 1u + (uint32_t)len;
        nign += (uint32_t)len;
        ++npaths;
      }
    }
    if (KIND == 1)
      for (uint32_t i = nign + lane; i < ign_cap; i += kWave) ig[i] = 0xFFFFFFFFu;
    if (lane == 0) {
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

uint32_t ksp_lds_bytes(uint32_t L, bool ign) {
  const uint32_t t = ksp_layout(L, ign).total;
  return t <= kMaxLds ? t : 0;
}

hipError_t launch_ksp_trace(int kind, const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                            const uint32_t* pdst, uint32_t first, uint32_t n, const uint64_t* rows, uint32_t* ign_io,
                            uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap, uint32_t* status, int num_cus,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t lds = ksp_lds_bytes(g.L, kind == 2);
  if (!lds) return hipErrorInvalidValue;
  const uint32_t grid = blocks_for(n, lds, num_cus, kWave);
  auto k = kind == 1 ? ksp_trace_kernel<1> : ksp_trace_kernel<2>;
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWave), lds, s, g, sources, prow, pdst, first, n, rows, ign_io, ign_cap, tok,
                     tok_cap, status);
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
