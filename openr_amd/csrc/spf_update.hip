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
    case kPatchErecS:
      if (g.erecs) g.erecs[r.idx] = r.val;
      break;
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

// Second, exact stage (round 3) for rows the first stage listed, when the
// caller keeps next-hop rows and no tight-edge rows (LinkState's dense memo, the update
// loop): a listed row is re-solved only if the change really moves its dist or next hops.
// With R = the row before the change (d, nh), R is still the solution on the patched graph
// iff every changed edge u->v keeps R a fixed point of runSpf's closed form
// (LinkState.cpp:846-873: d(v) = min over usable in-edges out of expanding nodes of
// d(u) + w, nh(v) = union over the tight ones of contrib(u) = nh(u), or {v} for u == src):
//   * new state usable with d(u) + w < d(v)                        -> changed;
//   * becomes tight (d(u) + w == d(v))  and contrib(u) not in nh(v) -> changed;
//   * stops being tight: v's tight in-edges under the new graph are none, or the union of
//     their contributions differs from nh(v)                        -> changed.
// Otherwise every node's equations hold with R's values, and the positive-weight solution
// is unique, so dist and next hops (not pathLinks, which is why tight rows opt out) are
// unchanged. One wavefront per listed row; lanes stride a node's in-edges.
constexpr uint32_t kExactMaxNb = 32;  // next-hop bytes the exact stage handles (256 bits)
__device__ __forceinline__ uint32_t nh_word(const uint8_t* p, uint32_t nb, uint32_t w) {
  uint32_t x = 0;
  for (uint32_t b = 0; b < 4u && 4u * w + b < nb; ++b) x |= (uint32_t)p[4u * w + b] << (8u * b);
  return x;
}
__global__ __launch_bounds__(256) void refresh_exact(DevGraph g, const DeltaEdge* delta, uint32_t n_delta,
                                                     uint32_t V, const uint64_t* dist, const uint8_t* nh, uint32_t nb,
                                                     uint32_t unit_cost, const uint32_t* alist_in,
                                                     const uint32_t* asrc_in, const uint32_t* count_in,
                                                     uint32_t* alist, uint32_t* asrc, uint32_t* count) {
  const uint32_t lane = __lane_id();
  const uint32_t waves = gridDim.x * 4u, n = *count_in, nw = (nb + 3u) / 4u;
  for (uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6); k < n; k += waves) {
    const uint32_t row = alist_in[k], src = asrc_in[k];
    const uint64_t* d = dist + (size_t)row * V;
    const uint8_t* h = nh + (size_t)row * V * nb;
    bool changed = false;  // wave-uniform
    for (uint32_t j = 0; j < n_delta && !changed; ++j) {
      const DeltaEdge x = delta[j];
      const uint64_t du = d[x.u];
      if (du == ~0ull) continue;
      const uint64_t dv = d[x.v];
      const bool a0 = (x.flags & kDeltaUp0) && (x.u == src || !(x.flags & kDeltaOvl0));
      const bool a1 = (x.flags & kDeltaUp1) && (x.u == src || !(x.flags & kDeltaOvl1));
      const uint64_t w0 = unit_cost ? 1u : x.w0, w1 = unit_cost ? 1u : x.w1;
      if (a0 == a1 && w0 == w1) continue;
      if (a1 && du + w1 < dv) {
        changed = true;
        break;
      }
      const bool t0 = a0 && du + w0 == dv, t1 = a1 && du + w1 == dv;
      if (t0 == t1) continue;
      const uint8_t* hv = h + (size_t)x.v * nb;
      if (t1) {  // v gains u's contribution: changed unless it is already in nh(v)
        bool extra = false;
        if (lane < nw) {
          uint32_t c;
          if (x.u == src) {
            const uint32_t bit = g.nbr[x.pad0];
            c = (bit / 32u == lane) ? 1u << (bit & 31u) : 0u;
          } else {
            c = nh_word(h + (size_t)x.u * nb, nb, lane);
          }
          extra = (c & ~nh_word(hv, nb, lane)) != 0u;
        }
        changed = __builtin_amdgcn_ballot_w64(extra) != 0ull;
        continue;
      }
      // v loses u->v: the union over v's tight in-edges in the patched graph must equal nh(v)
      uint32_t acc[kExactMaxNb / 4u];
#pragma unroll
      for (uint32_t w = 0; w < kExactMaxNb / 4u; ++w) acc[w] = 0u;
      bool any = false;
      const uint2 rv = g.row2[x.v];
      for (uint32_t e = rv.x + lane; e < rv.y; e += 64u) {
        const uint32_t r = g.rev[e];  // u' -> v
        const uint32_t ar = g.adj[r];
        const uint32_t up = g.adj[e] & ~kEdgeDown;  // u'
        if ((ar & kEdgeDown) || (up != src && g.ovl[up])) continue;
        const uint64_t dp = d[up];
        if (dp == ~0ull || dp + (unit_cost ? 1u : g.w[r]) != dv) continue;
        any = true;
        if (up == src) {
          const uint32_t bit = g.nbr[r];
#pragma unroll
          for (uint32_t w = 0; w < kExactMaxNb / 4u; ++w)
            if (w == bit / 32u) acc[w] |= 1u << (bit & 31u);
        } else {
          const uint8_t* hu = h + (size_t)up * nb;
#pragma unroll
          for (uint32_t w = 0; w < kExactMaxNb / 4u; ++w)
            if (w < nw) acc[w] |= nh_word(hu, nb, w);
        }
      }
      if (__builtin_amdgcn_ballot_w64(any) == 0ull) {
        changed = true;  // no tight in-edge left: d(v) grows
        break;
      }
      bool diff = false;
#pragma unroll
      for (uint32_t w = 0; w < kExactMaxNb / 4u; ++w) {
        if (w >= nw) break;
        const uint32_t u = __reduce_or_sync(~0ull, acc[w]);
        diff |= u != nh_word(hv, nb, w);
      }
      changed = diff;  // uniform: every lane holds the reduced words
    }
    if (changed && lane == 0) {
      const uint32_t q = atomicAdd(count, 1u);
      alist[q] = row;
      asrc[q] = src;
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

hipError_t launch_refresh_exact(const DevGraph& g, const DeltaEdge* delta, uint32_t n_delta, uint32_t V,
                                const uint64_t* dist, const uint8_t* nh, uint32_t nb, bool unit_cost,
                                const uint32_t* alist_in, const uint32_t* asrc_in, const uint32_t* count_in,
                                uint32_t n_max, uint32_t* alist, uint32_t* asrc, uint32_t* count, int num_cus,
                                hipStream_t s) {
  if (!n_max) return hipSuccess;
  if (nb > kExactMaxNb) return hipErrorInvalidValue;
  const uint32_t grid = std::min<uint32_t>((n_max + 3u) / 4u, (uint32_t)num_cus * 8u);
  hipLaunchKernelGGL(refresh_exact, dim3(grid), dim3(256), 0, s, g, delta, n_delta, V, dist, nh, nb,
                     unit_cost ? 1u : 0u, alist_in, asrc_in, count_in, alist, asrc, count);
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
