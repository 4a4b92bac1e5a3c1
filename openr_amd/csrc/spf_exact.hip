// spf_exact.hip — the exact-order SPF kernel: LinkState::runSpf's heap process itself.
//
// The fast kernels (spf_bfs*.hip, spf_fringe.hip, spf_rounds.hip) rely on two facts that
// hold for usable metrics in [1, 2^31-1] on graphs that fit their LDS layouts: the
// reference's (metric, name) pop order is the sorted (dist, name) order, and pathLinks(v)
// are all tight in-edges. Outside that domain the engine used to refuse the graph
// (ENOTSUP / E2BIG). This kernel covers it instead, on the GPU:
//   * zero metrics and i32-negative metrics (which wrap to huge u64 values on Link
//     construction, LinkState.cpp:151-152), where the pop order is history-dependent
//     (SURVEY.md Appendix A.2);
//   * graphs too large for the LDS-resident kernels, and next-hop sets wider than 256.
// It replays /root/reference/openr/decision/LinkState.cpp:808-882 step by step: pop the
// minimum (metric, name) of the queue (DijkstraQ, LinkState.h:475-535: a wave-wide argmin
// over the queued nodes), record it, skip expansion of overloaded non-source nodes
// (:831-838), relax u's links in linksFromNode order with u64 wrapping sums: insert an
// untouched node, reset on a strictly better metric, then addPath + addNextHops, and the
// direct-neighbour next hop when the set is still empty (:846-873). The relaxation of one
// row runs in link order on one lane because later links of a row see the effect of
// earlier ones (parallel links). Cost: a wave argmin over the queue per pop, O(V * queue
// / 64) per solve — the correctness path for graphs outside the fast kernels' domain,
// not a fast path. Outputs: dist / nh like every solve; tight = the edges left in pathLinks at
// the end (u popped before v: for zero metrics a subset of the tight in-edges); and,
// optionally, the pop index of every node (the settle order pathLinks follow).
//
// State per solve: in LDS when it fits (graphs of a few thousand nodes), else in a
// global-memory scratch slot. One wavefront per solve, persistent over the batch.
#include <algorithm>

#include "spf_bfs_common.h"
#include "spf_kernels.h"

namespace openr_spf {

namespace {

struct ExLayout {
  uint32_t key, state, order, queue, nh, plep, recep, ign, total;
  uint64_t total64;  // the slot's bytes; the u32 offsets above hold only when it is <= UINT32_MAX
};

// per-solve state, offsets from the slot base; nbw = next-hop words per node
__host__ __device__ inline ExLayout ex_layout(uint32_t V, uint32_t E, uint32_t L, uint32_t nbw) {
  ExLayout l;
  uint64_t off = 16;  // [0] queue length, [1] pops, [2] group end
  auto take = [&](uint64_t bytes) {
    const uint64_t o = off;
    off += (bytes + 15u) & ~15ull;
    return (uint32_t)o;
  };
  l.key = take(8ull * V);
  l.state = take(V);  // 0 untouched, 1 queued, 2 recorded
  l.order = take(4ull * V);
  l.queue = take(4ull * V);
  l.nh = take(4ull * V * nbw);
  l.plep = take(4ull * V);  // pathLinks epoch of v (a reset starts a new one)
  l.recep = take(4ull * E);  // epoch + 1 at which edge e was appended to pathLinks(col)
  l.ign = take(4ull * ((L + 31u) / 32u));
  l.total = (uint32_t)std::min<uint64_t>(off, 0xFFFFFFFFull);
  l.total64 = off;
  return l;
}

__device__ __forceinline__ bool ex_less(uint64_t ka, uint32_t ra, uint64_t kb, uint32_t rb) {
  return ka < kb || (ka == kb && ra < rb);
}

__global__ __launch_bounds__(64) void spf_exact_kernel(DevGraph g, SolveArgs a, const uint64_t* w64,
                                                       uint32_t use_metric, uint32_t nbw,
                                                       uint32_t in_lds, uint8_t* scratch, uint64_t slot_bytes,
                                                       uint32_t* order_out, uint32_t* ctr) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t V = g.V, E = g.E, lane = __lane_id();
  const ExLayout lay = ex_layout(V, E, g.L, nbw);
  char* base = in_lds ? reinterpret_cast<char*>(smem) : reinterpret_cast<char*>(scratch + slot_bytes * blockIdx.x);
  uint32_t* ctl = reinterpret_cast<uint32_t*>(base);
  uint64_t* key = reinterpret_cast<uint64_t*>(base + lay.key);
  uint8_t* st = reinterpret_cast<uint8_t*>(base + lay.state);
  uint32_t* order = reinterpret_cast<uint32_t*>(base + lay.order);
  uint32_t* queue = reinterpret_cast<uint32_t*>(base + lay.queue);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + lay.nh);
  uint32_t* plep = reinterpret_cast<uint32_t*>(base + lay.plep);
  uint32_t* recep = reinterpret_cast<uint32_t*>(base + lay.recep);
  uint32_t* ign = reinterpret_cast<uint32_t*>(base + lay.ign);
  const uint32_t iw = (g.L + 31u) / 32u, tw = (E + 63u) / 64u;
  auto fence = [&] {
    if (in_lds) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else __threadfence_block();
  };
  for (uint32_t k = blockIdx.x; k < a.n;) {
    const uint32_t src = a.sources[k];
    const size_t orow = out_row_of(a, k);
    // reset the slot
    for (uint32_t v = lane; v < V; v += 64u) {
      st[v] = 0;
      plep[v] = 0;
      key[v] = ~0ull;
    }
    for (uint32_t i = lane; i < V * nbw; i += 64u) nh[i] = 0;
    for (uint32_t e = lane; e < E; e += 64u) recep[e] = 0;
    for (uint32_t i = lane; i < iw; i += 64u) ign[i] = 0;
    fence();
    if (a.ign_ptr) {
      const uint32_t b = a.ign_ptr[k], e = a.ign_end ? a.ign_end[k] : a.ign_ptr[k + 1];
      for (uint32_t i = b + lane; i < e; i += 64u) {
        const uint32_t l = a.ign_links[i];
        if (l < g.L) atomicOr(&ign[l >> 5], 1u << (l & 31u));
      }
    }
    if (lane == 0) {
      key[src] = 0;
      st[src] = 1;
      queue[0] = src;
      ctl[0] = 1;
      ctl[1] = 0;
    }
    fence();
    uint32_t qn = 1, pops = 0;
    while (qn) {
      // argmin (metric, name rank) over the queue
      uint64_t bk = ~0ull;
      uint32_t br = UINT32_MAX, bi = UINT32_MAX;
      for (uint32_t i = lane; i < qn; i += 64u) {
        const uint32_t v = queue[i];
        const uint64_t kv = key[v];
        const uint32_t rv = g.rank[v];
        if (ex_less(kv, rv, bk, br)) {
          bk = kv;
          br = rv;
          bi = i;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t k2 = __shfl_xor(bk, o);
        const uint32_t r2 = __shfl_xor(br, o), i2 = __shfl_xor(bi, o);
        if (ex_less(k2, r2, bk, br)) {
          bk = k2;
          br = r2;
          bi = i2;
        }
      }
      // lane 0 pops the minimum and relaxes its row in link order
      if (lane == 0) {
        const uint32_t u = queue[bi];
        queue[bi] = queue[--qn];
        st[u] = 2;
        order[u] = pops++;
        if (u == src || !g.ovl[u]) {
          const uint64_t du = key[u];
          for (uint32_t e = g.row[u]; e < g.row[u + 1]; ++e) {
            const uint32_t av = g.adj[e];
            const uint32_t v = av & ~kEdgeDown;
            if ((av & kEdgeDown) || st[v] == 2 || ((ign[g.lid[e] >> 5] >> (g.lid[e] & 31u)) & 1u)) continue;
            const uint64_t c = du + (use_metric ? w64[e] : 1ull);  // u64 wrap, as the reference
            uint32_t* nv = nh + (size_t)v * nbw;
            if (st[v] == 0) {  // q.insertNode
              st[v] = 1;
              key[v] = c;
              queue[qn++] = v;
            }
            if (key[v] >= c) {
              if (key[v] > c) {  // reset + reMake
                key[v] = c;
                ++plep[v];
                for (uint32_t b = 0; b < nbw; ++b) nv[b] = 0;
              }
              recep[e] = plep[v] + 1u;  // addPath(link, u)
              const uint32_t* nu = nh + (size_t)u * nbw;
              uint32_t any = 0;
              for (uint32_t b = 0; b < nbw; ++b) any |= (nv[b] |= nu[b]);  // addNextHops
              if (!any && u == src) {  // directly connected: addNextHop(v)
                const uint32_t bit = g.nbr[e];
                nv[bit >> 5] |= 1u << (bit & 31u);
              }
            }
          }
        }
        ctl[0] = qn;
        ctl[1] = pops;
      }
      fence();
      qn = __shfl(qn, 0);
      pops = __shfl(pops, 0);
    }
    // outputs
    uint64_t* drow = a.dist + orow * V;
    for (uint32_t v = lane; v < V; v += 64u) drow[v] = st[v] == 2 ? key[v] : ~0ull;
    if (a.nh) {
      uint8_t* nrow = a.nh + orow * V * a.nh_bytes;
      for (uint32_t i = lane; i < V * a.nh_bytes; i += 64u) {
        const uint32_t v = i / a.nh_bytes, b = i - v * a.nh_bytes;
        nrow[i] = (st[v] == 2 && b / 4u < nbw) ? (uint8_t)(nh[(size_t)v * nbw + b / 4u] >> (8u * (b & 3u))) : 0u;
      }
    }
    if (a.tight) {  // the edges left in pathLinks: appended in v's final epoch, v recorded
      uint64_t* trow = a.tight + orow * tw;
      for (uint32_t wd = lane; wd < tw; wd += 64u) {
        uint64_t m = 0;
        for (uint32_t b = 0; b < 64u; ++b) {
          const uint32_t e = wd * 64u + b;
          if (e >= E) break;
          const uint32_t v = g.adj[e] & ~kEdgeDown;
          if (recep[e] && st[v] == 2 && recep[e] == plep[v] + 1u) m |= 1ull << b;
        }
        trow[wd] = m;
      }
    }
    if (order_out) {
      uint32_t* orow_p = order_out + orow * V;
      for (uint32_t v = lane; v < V; v += 64u) orow_p[v] = st[v] == 2 ? order[v] : UINT32_MAX;
    }
    fence();
    uint32_t nxt = 0;
    if (lane == 0) nxt = gridDim.x + atomicAdd(&ctr[0], 1u);
    k = __builtin_amdgcn_readfirstlane(__shfl(nxt, 0));
  }
  if (lane == 0) {
    __threadfence();
    if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1u) {
      ctr[0] = 0;
      ctr[1] = 0;
      __threadfence();
    }
  }
}

}  // namespace

uint64_t exact_slot_bytes(uint32_t V, uint32_t E, uint32_t L, uint32_t nh_bits) {
  const uint32_t nbw = std::max<uint32_t>(1u, (nh_bits + 31u) / 32u);
  return ex_layout(V, E, L, nbw).total64;  // > UINT32_MAX: the layout does not fit (make_plan refuses)
}

hipError_t launch_exact(const DevGraph& g, const SolveArgs& a, const uint64_t* w64, bool use_metric, uint32_t nh_bits, uint8_t* scratch, uint64_t scratch_bytes, uint32_t* order_out,
                        uint32_t* ctr, int num_cus, hipStream_t s) {
  if (!a.n) return hipSuccess;
  const uint32_t nbw = std::max<uint32_t>(1u, (nh_bits + 31u) / 32u);
  const uint64_t slot = exact_slot_bytes(g.V, g.E, g.L, nh_bits);
  if (slot > 0xFFFFFFFFull) return hipErrorInvalidValue;  // u32 slot offsets (make_plan refuses such graphs)
  const bool in_lds = slot <= kMaxLds && !bfs::env_u32("OPENR_SPF_EXACT_GLOBAL", 0u, 0u, 1u);
  uint32_t grid;
  if (in_lds) {
    grid = blocks_for(a.n, (uint32_t)slot, num_cus, 64u);
  } else {
    if (!scratch || scratch_bytes < slot) return hipErrorInvalidValue;
    grid = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(a.n, scratch_bytes / slot), (uint64_t)num_cus * 8u);
  }
  if (in_lds) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(spf_exact_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)slot);
    if (err != hipSuccess) return err;
  }
  note_launch("spf_exact_kernel");
  hipLaunchKernelGGL(spf_exact_kernel, dim3(grid), dim3(64), in_lds ? (uint32_t)slot : 0u, s, g, a, w64,
                     (uint32_t)use_metric, nbw, (uint32_t)in_lds, scratch, slot, order_out, ctr);
  return hipGetLastError();
}

}  // namespace openr_spf
