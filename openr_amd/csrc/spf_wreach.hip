// spf_wreach.hip — wave-reach pass (round 3): all-sources level rows on ELL-delta graphs
// (row-major grids: BASELINE config 3), one wavefront per source, the graph staged in LDS,
// levels stored straight to the HBM level rows.
//
// The closed form of LinkState::runSpf for uniform cost (LinkState.cpp:808-882) splits into
// levels and next hops, and when a batch holds every source's usable neighbours the next
// hops follow from the neighbours' level rows (spf_allsrc.hip, nh_from_levels_kernel). The
// level pass then needs no per-node state but "visited": a wavefront solves one source over
// a visited bitmap (V bits) and a two-half frontier queue — about 2.3 KB of LDS on G100
// against 16.3 KB for the lean pass (u8 levels + next-hop nibbles + queue), so a CU holds
// 32 solves in flight instead of 10 — and a node's level is written to its level row in
// HBM by the arrival that appends it (one byte store per node and solve, the row's only
// write). The transit rows come from LDS as four signed byte deltas (DevGraph::elld, the
// wave pass's form: 4 B per node), so a level's dependent chain is queue entry -> delta row
// -> visited ds_or_rtn -> append, with no global load and no barrier (a wavefront's LDS
// operations complete in issue order). Unreached nodes (disconnected graphs) get 0xFF when
// the solve ends; a solve deeper than 253 levels or a level wider than a queue half is
// flagged (rowok = 0) for the u16 full-order re-run.
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

constexpr uint32_t kWrWaves = 16;  // wavefronts (solve slots) per workgroup; two workgroups per CU

struct WrLayout {
  uint32_t slot0, vis, q, per_slot, total;
};
// [0, 4V) delta rows, then kWrWaves slots [visited words | two queue halves]
__host__ __device__ inline WrLayout wr_layout(uint32_t V, uint32_t qhalf) {
  WrLayout l;
  l.slot0 = (4u * V + 15u) & ~15u;
  l.vis = 0;
  l.q = (4u * ((V + 31u) / 32u) + 15u) & ~15u;
  l.per_slot = l.q + ((4u * qhalf + 15u) & ~15u);
  l.total = l.slot0 + kWrWaves * l.per_slot;
  return l;
}

__global__ __launch_bounds__(64 * kWrWaves) __attribute__((amdgpu_waves_per_eu(8))) void bfs_wreach_kernel(DevGraph g, SolveArgs a, uint32_t qhalf,
                                                                  uint32_t ntot, uint32_t* ctr, uint32_t* ovf_count,
                                                                  uint32_t ablate) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // no static LDS: smem is LDS address 0
  const uint32_t V = g.V, tid = threadIdx.x, lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const WrLayout lay = wr_layout(V, qhalf);
  const uint32_t slot = lay.slot0 + wave * lay.per_slot;
  lds_u32* const rows = (lds_u32*)(size_t)0u;
  lds_u32* const vis = (lds_u32*)(size_t)(slot + lay.vis);
  lds_u16* const q = (lds_u16*)(size_t)(slot + lay.q);
  for (uint32_t i = tid; i < V; i += blockDim.x) rows[i] = g.elld[i];
  __syncthreads();
  const uint32_t vwords = (V + 31u) / 32u, vfull = V / 32u;
  const uint32_t rb = reach_row_bytes(V);
  // rows: the call's, then (extended batch) the halo rows
  const uint32_t n_rows = a.xcount ? ntot + a.xcount[0] : ntot;
  // the first grid x W units are static, dealt wave-major (unit i to workgroup i % grid) so a
  // small batch spreads over every CU, then dynamic
  uint32_t unit = wave * gridDim.x + blockIdx.x;
  while (unit < n_rows) {
    const uint32_t src = a.sources[unit];
    bool ok = false;
    if (src < V) {  // wave-uniform
      uint8_t* lrow = a.lvl8 + (size_t)unit * rb;
      for (uint32_t i = lane; i < vwords; i += 64u)  // ids >= V count as visited
        vis[i] = i < vfull ? 0u : ~((1u << (V & 31u)) - 1u);
      if (lane == 0) {
        vis[src >> 5] |= 1u << (src & 31u);
        lrow[src] = 0;
      }
      // level 0: the source expands even when overloaded (its full CSR row)
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
              const uint32_t bit = 1u << (v & 31u);
              fresh = (lds_or(&vis[v >> 5], bit) & bit) == 0u;
            }
          }
          const unsigned long long b = __builtin_amdgcn_ballot_w64(fresh);
          if (fresh) {  // slot < deg(src) < qhalf (host-checked)
            q[qhalf + cur + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] =
                (uint16_t)v;
            lrow[v] = 1;
          }
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
        for (uint32_t fb = 0; fb < cur; fb += 64u) {
          const uint32_t idx = fb + lane;
          const bool live = idx < cur;
          const uint32_t qe = q[rd + (live ? idx : 0u)];
          const uint32_t u = live ? qe : src;  // past the level: the source (visited)
          const uint32_t r4 = rows[u];
          const uint32_t d4 = live ? r4 : 0u;  // no slots: every slot resolves to u (visited)
          uint32_t vv[4], old[4];
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) vv[j] = u + (uint32_t)__builtin_amdgcn_sbfe((int32_t)d4, 8u * j, 8u);
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) old[j] = lds_or(&vis[vv[j] >> 5], 1u << (vv[j] & 31u));
          __builtin_amdgcn_sched_barrier(0);  // all atomics in flight before their results are used
          unsigned long long bj[4];
          bool fresh[4];
          uint32_t off[5];
          off[0] = 0;
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) {
            fresh[j] = __builtin_amdgcn_ubfe(old[j], vv[j] & 31u, 1u) == 0u;  // first arrival
            bj[j] = __builtin_amdgcn_ballot_w64(fresh[j]);
            off[j + 1] = off[j] + (uint32_t)__popcll(bj[j]);
          }
          const uint32_t total = off[4];
          if (total) {  // wave-uniform
            if (nxt + total <= qhalf) {
#pragma unroll
              for (uint32_t j = 0; j < 4u; ++j) {
                if (fresh[j]) {
                  const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(bj[j] >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], 0u));
                  q[wr + nxt + off[j] + k] = (uint16_t)vv[j];
                  if (!ablate) lrow[vv[j]] = lnext;  // the appending arrival stores v's level (its row's only write)
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
      }
      if (!overflow) {
        ok = true;
        if (reached < V)  // nodes the solve never reached: 0xFF
          for (uint32_t i = lane; i < vwords; i += 64u) {
            uint32_t m = ~vis[i];
            while (m) {
              const uint32_t b = (uint32_t)__builtin_ctz(m);
              m &= m - 1u;
              lrow[32u * i + b] = 0xFFu;
            }
          }
      }
    }
    if (lane == 0) {
      a.rowok[unit] = ok ? 1u : 0u;
      // a halo row is no call row: the sources that need it are listed by the next-hop pass
      if (!ok && src < V && unit < ntot) a.ovf_list[atomicAdd(ovf_count, 1u)] = unit;
    }
    uint32_t nx = 0;
    if (lane == 0) nx = gridDim.x * kWrWaves + atomicAdd(&ctr[0], 1u);
    unit = __builtin_amdgcn_readfirstlane(nx);
  }
  __syncthreads();  // no wave of this workgroup takes units any more
  retire_workgroup(ctr, nullptr);
}

}  // namespace

// LDS of the wave-reach pass for graph g and queue half qhalf; 0 when it does not apply
// (no delta rows, or two workgroups do not fit a CU)
uint32_t wreach_lds_bytes(const DevGraph& g, uint32_t qhalf) {
  if (!g.elld || qhalf <= g.max_deg) return 0;
  const uint32_t t = wr_layout(g.V, qhalf).total;
  return 2u * t <= kMaxLds ? t : 0u;
}

hipError_t launch_wreach(const DevGraph& g, const SolveArgs& a, uint32_t qhalf, uint32_t* blk, int num_cus,
                         hipStream_t s, LaunchInfo* info) {
  const uint32_t lds = wreach_lds_bytes(g, qhalf);
  if (!lds) return hipErrorInvalidValue;
  const uint32_t rows_max = a.xcount ? ms_ext_rows(g, a.n) : a.n;
  const uint32_t grid = std::max<uint32_t>(
      1u, std::min<uint32_t>(2u * (uint32_t)num_cus, (rows_max + kWrWaves - 1u) / kWrWaves));
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(bfs_wreach_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  if (info) {
    info->lds_bytes = lds;
    info->grid = grid;
    info->kernel = "bfs_wreach_kernel";
  }
  note_launch("bfs_wreach_kernel");
  // OPENR_SPF_WREACH_ABLATE=1: measurement only — the level stores of levels >= 2 are
  // skipped (wrong rows) to price them
  const uint32_t ablate = env_u32("OPENR_SPF_WREACH_ABLATE", 0u, 0u, 1u);
  hipLaunchKernelGGL(bfs_wreach_kernel, dim3(grid), dim3(64u * kWrWaves), lds, s, g, a, qhalf, a.n, blk, blk + 4,
                     ablate);
  return hipGetLastError();
}

}  // namespace openr_spf
