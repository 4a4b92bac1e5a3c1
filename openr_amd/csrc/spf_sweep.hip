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
        const uint64_t* trow = base_tight + (size_t)j * tight_words;
        hit = ((trow[ee.x >> 6] >> (ee.x & 63u)) & 1ull) || ((trow[ee.y >> 6] >> (ee.y & 63u)) & 1ull);
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
                                                    uint32_t* changed) {
  __shared__ uint32_t part[4];
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t unit = wunit[k], j = unit % n_src;
    const uint64_t* d = dist + (size_t)k * V;
    const uint64_t* bd = base_dist + (size_t)j * V;
    const uint8_t* h = nh ? nh + (size_t)k * V * nb : nullptr;
    const uint8_t* bh = nh ? base_nh + (size_t)j * V * nb : nullptr;
    uint32_t c = 0;
    for (uint32_t v = threadIdx.x; v < V; v += 256u) {
      bool diff = d[v] != bd[v];
      if (h)
        for (uint32_t b = 0; b < nb && !diff; ++b) diff = h[(size_t)v * nb + b] != bh[(size_t)v * nb + b];
      c += diff ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (__lane_id() == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) changed[unit] = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
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
                               uint32_t n_src, uint32_t* changed, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(rows_compare, dim3(grid_for(n, 1u, num_cus)), dim3(256), 0, s, n, V, nb, dist, nh, base_dist,
                     base_nh, wunit, n_src, changed);
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* p, uint32_t n, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(iota_u32, dim3(grid_for(n, 256u, num_cus)), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

}  // namespace openr_spf
