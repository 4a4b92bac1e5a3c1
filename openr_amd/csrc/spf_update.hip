// spf_update.hip — incremental mirror updates: in-place attribute patches of the device
// CSR mirror and the affected-row filter of openr_spf_refresh.
//
// The reference clears its whole SPF memo whenever updateAdjacencyDatabase /
// decrementHolds report a topology change (/root/reference/openr/decision/LinkState.cpp:
// 509-512, 714-717) and re-runs Dijkstra per source on demand. Most such changes are
// attribute changes — a metric (setMetricFromNode), an adjacency overload or hold
// (Link::isUp, :233-236), a node overload bit (updateNodeOverloaded) — on a fixed set of
// links. Here they patch the resident mirror element by element (no rebuild / upload),
// and resident all-sources rows are refreshed by re-solving only the rows the change can
// touch:
//
//   row of source s is affected  <=>  for some changed directed edge e = u->v,
//     old:  e usable, u expands for s (u == s or u not overloaded), d[u] + w_old == d[v]
//     new:  e usable, u expands for s,                              d[u] + w_new <= d[v]
//   with d = the row's distances before the change (d[u] finite).
//
// If no changed edge is tight before or may be tight/shorter after, the old distances
// still satisfy every edge's triangle inequality with the same tight set, so dist, the
// next-hop sets (LinkState.cpp:867-872: unions over tight in-edges) and pathLinks are
// unchanged. Integer work, one wavefront per row, HBM-light (two 8-byte reads per delta
// edge and row).
#include "spf_device.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {

__global__ __launch_bounds__(256) void patch_apply(DevGraph g, const PatchRec* recs, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const PatchRec r = recs[i];
  switch (r.arr) {
    case kPatchAdj: g.adj[r.idx] = r.val.x; break;
    case kPatchW: g.w[r.idx] = r.val.x; break;
    case kPatchWin: g.win[r.idx] = r.val.x; break;
    case kPatchErec: g.erec[r.idx] = r.val; break;
    case kPatchEllt: g.ellt[r.idx] = r.val; break;
    case kPatchEllv: g.ellv[r.idx] = r.val; break;
    case kPatchElld:
      if (g.elld) g.elld[r.idx] = r.val.x;
      break;
    case kPatchRow2t: g.row2t[r.idx] = make_uint2(r.val.x, r.val.y); break;
    case kPatchOvl: g.ovl[r.idx] = (uint8_t)r.val.x; break;
    case kPatchOvlBits: g.ovl_bits[r.idx] = r.val.x; break;
    case kPatchW64: g.w64[r.idx] = ((uint64_t)r.val.y << 32) | r.val.x; break;
    default: break;
  }
}

// One wavefront per row; lanes stride over the delta edges.
__global__ __launch_bounds__(256) void refresh_filter(const DeltaEdge* delta, uint32_t n_delta,
                                                      const uint32_t* sources, uint32_t n, uint32_t V,
                                                      const uint64_t* dist, uint32_t unit_cost, uint32_t* alist,
                                                      uint32_t* asrc, uint32_t* count) {
  const uint32_t lane = __lane_id();
  const uint32_t waves = gridDim.x * 4u;
  for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < n; i += waves) {
    const uint32_t src = sources[i];
    const uint64_t* d = dist + (size_t)i * V;
    bool hit = false;
    for (uint32_t j = lane; j < n_delta && !hit; j += 64u) {
      const DeltaEdge x = delta[j];
      const uint64_t du = d[x.u];
      if (du == ~0ull) continue;  // u unreached: none of its edges is or can be relaxed
      const uint64_t dv = d[x.v];
      const bool exp0 = x.u == src || !(x.flags & kDeltaOvl0);
      const bool exp1 = x.u == src || !(x.flags & kDeltaOvl1);
      const bool a0 = (x.flags & kDeltaUp0) && exp0;
      const bool a1 = (x.flags & kDeltaUp1) && exp1;
      const uint64_t w0 = unit_cost ? 1u : x.w0, w1 = unit_cost ? 1u : x.w1;
      if (a0 == a1 && w0 == w1) continue;  // no change as seen from this source
      hit = (a0 && du + w0 == dv) || (a1 && du + w1 <= dv);
    }
    if (__ballot(hit) != 0ull && lane == 0) {
      const uint32_t k = atomicAdd(count, 1u);
      alist[k] = i;
      asrc[k] = src;
    }
  }
}

__global__ __launch_bounds__(256) void zero_rows(uint64_t* rows, uint32_t words, const uint32_t* alist, uint32_t n) {
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    uint64_t* r = rows + (size_t)alist[k] * words;
    for (uint32_t w = threadIdx.x; w < words; w += 256u) r[w] = 0ull;
  }
}

}  // namespace

hipError_t launch_patch_apply(const DevGraph& g, const PatchRec* recs, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(patch_apply, dim3((n + 255u) / 256u), dim3(256), 0, s, g, recs, n);
  return hipGetLastError();
}

hipError_t launch_refresh_filter(const DeltaEdge* delta, uint32_t n_delta, const uint32_t* sources, uint32_t n,
                                 uint32_t V, const uint64_t* dist, bool unit_cost, uint32_t* alist, uint32_t* asrc,
                                 uint32_t* count, int num_cus, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>((n + 3u) / 4u, (uint32_t)num_cus * 8u);
  hipLaunchKernelGGL(refresh_filter, dim3(grid), dim3(256), 0, s, delta, n_delta, sources, n, V, dist,
                     unit_cost ? 1u : 0u, alist, asrc, count);
  return hipGetLastError();
}

hipError_t launch_zero_rows(uint64_t* rows, uint32_t words, const uint32_t* alist, uint32_t n, int num_cus,
                            hipStream_t s) {
  if (!n || !words) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>(n, (uint32_t)num_cus * 8u);
  hipLaunchKernelGGL(zero_rows, dim3(grid), dim3(256), 0, s, rows, words, alist, n);
  return hipGetLastError();
}

}  // namespace openr_spf
