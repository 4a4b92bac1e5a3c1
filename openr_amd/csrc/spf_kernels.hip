// spf_kernels.hip — shared launch helpers of the OpenR SPF engine.
//
// Semantics restated from LinkState::runSpf (/root/reference/openr/decision/
// LinkState.cpp:808-882) in closed form for strictly positive metrics
// (SURVEY.md Appendix A.3):
//   dist  = shortest distance over usable edges, no transit through overloaded
//           nodes other than the source;
//   nh(v) = OR over tight in-edges u->v of (u == src ? {v} : nh(u)).
// The reference's heap order (metric, name) only matters for pathLinks order,
// which the host rebuilds from the tight-edge mask (include/openr_spf.h).
//
// Kernels: spf_bfs.hip / spf_bfs_lvl.hip (uniform edge cost, level-synchronous BFS,
// two families), spf_fringe.hip (general positive metrics, one wavefront per solve),
// spf_sweep.hip (what-if filter / row comparison). This file: launch helpers shared
// by them and the device-side source-class partition.
// No MFMA: min-plus relaxation is not a matrix contraction; the bound is the CSR
// stream and the result write (DESIGN.md "Roofline").
#include "spf_kernels.h"

#include <algorithm>
#include <cstdlib>

#include "spf_device.h"

namespace openr_spf {

namespace {
using namespace dev;


}  // namespace

template <int MODE>
uint32_t nh_words_host(uint32_t V) {
  return Nh<MODE>::words(V);
}

uint32_t nh_words_for(int mode, uint32_t V) {
  switch (mode) {
    case kNhNibble: return nh_words_host<kNhNibble>(V);
    case kNhByte: return nh_words_host<kNhByte>(V);
    case kNhHalf: return nh_words_host<kNhHalf>(V);
    case kNhW1: return nh_words_host<kNhW1>(V);
    case kNhW2: return nh_words_host<kNhW2>(V);
    case kNhW4: return nh_words_host<kNhW4>(V);
    case kNhW8: return nh_words_host<kNhW8>(V);
  }
  return 0;
}

uint32_t blocks_for(uint32_t n, uint32_t lds, int num_cus, uint32_t block) {
  const uint32_t max_wg = 2048u / block;  // 2048 threads (32 waves) per CU
  uint32_t per_cu = lds ? kMaxLds / lds : max_wg;
  if (per_cu > max_wg) per_cu = max_wg;
  if (per_cu < 1) per_cu = 1;
  uint64_t g = (uint64_t)num_cus * per_cu;
  if (g > n) g = n;
  return (uint32_t)(g ? g : 1);
}

bool nh_mode_single(int mode) {
  return mode == kNhNibble || mode == kNhByte || mode == kNhHalf || mode == kNhW1;
}

int src_class_for_degree(int family, uint32_t d) {
  if (d > 256) return -1;
  if (family == kFamLvl) {
    if (d <= 4) return kLvl4;
    if (d <= 8) return kLvl8;
    if (d <= 16) return kLvl16;
    if (d <= 32) return kLvl32;
    return kLvlSliced;
  }
  if (d <= 5) return kCls8;
  if (d <= 13) return kCls16;
  if (d <= 29) return kCls32;
  return kClsSliced;
}

int num_classes(int family) { return family == kFamLvl ? kNumLvlClasses : kNumClasses; }
int sliced_class(int family) { return family == kFamLvl ? kLvlSliced : kClsSliced; }
uint32_t slice_bits(int family) { return family == kFamLvl ? 32u : 29u; }

uint32_t bfs_lds_bytes(int family, uint32_t V, uint32_t L, bool has_ignore, int cls) {
  return family == kFamLvl ? bfs_lvl_lds_bytes(V, L, has_ignore, cls) : bfs_code_lds_bytes(V, L, has_ignore, cls);
}

hipError_t launch_bfs(int family, const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes,
                      int num_cus, hipStream_t s, LaunchInfo* info) {
  return family == kFamLvl ? launch_bfs_lvl(g, a, cost, group_lanes, num_cus, s, info)
                           : launch_bfs_code(g, a, cost, group_lanes, num_cus, s, info);
}

namespace {
// Wave-aggregated class histogram / scatter of a source batch (one atomic per class
// per wave). part = [counts | offsets | cursors], each kMaxClasses u32, zeroed by the
// launcher.
__global__ __launch_bounds__(256) void partition_count(const uint32_t* src, uint32_t n, const uint8_t* cls,
                                                       uint32_t V, uint32_t* part) {
  for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t u = i < n ? src[i] : V;
    const uint32_t c = u < V ? cls[u] : 0u;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      const unsigned long long m = __ballot(i < n && c == k);
      if (m && __lane_id() == (uint32_t)(__ffsll((long long)m) - 1)) atomicAdd(&part[k], (uint32_t)__popcll(m));
    }
  }
}

__global__ __launch_bounds__(256) void partition_scatter(const uint32_t* src, uint32_t n, const uint8_t* cls,
                                                         uint32_t V, uint32_t* part, uint32_t* perm) {
  __shared__ uint32_t off[kMaxClasses];
  if (threadIdx.x == 0) {
    uint32_t o = 0;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      off[k] = o;
      o += part[k];
      if (blockIdx.x == 0) part[kMaxClasses + k] = off[k];
    }
  }
  __syncthreads();
  const uint32_t lane = __lane_id();
  for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t u = i < n ? src[i] : V;
    const uint32_t c = u < V ? cls[u] : 0u;
    for (uint32_t k = 0; k < kMaxClasses; ++k) {
      const unsigned long long m = __ballot(i < n && c == k);
      if (!m) continue;
      const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&part[2u * kMaxClasses + k], (uint32_t)__popcll(m));
      base = __shfl(base, (int)leader);
      if (i < n && c == k) perm[off[k] + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
    }
  }
}
}  // namespace

hipError_t launch_partition(const uint32_t* d_sources, uint32_t n, const uint8_t* d_node_cls, uint32_t V,
                            uint32_t* d_part, uint32_t* d_perm, hipStream_t s) {
  hipError_t err = hipMemsetAsync(d_part, 0, 3u * kMaxClasses * sizeof(uint32_t), s);
  if (err != hipSuccess || n == 0) return err;
  const uint32_t grid = std::min<uint32_t>((n + 255u) / 256u, 1024u);
  hipLaunchKernelGGL(partition_count, dim3(grid), dim3(256), 0, s, d_sources, n, d_node_cls, V, d_part);
  err = hipGetLastError();
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(partition_scatter, dim3(grid), dim3(256), 0, s, d_sources, n, d_node_cls, V, d_part, d_perm);
  return hipGetLastError();
}

int nh_mode_for_bits(uint32_t bits) {
  if (bits <= 4) return kNhNibble;
  if (bits <= 8) return kNhByte;
  if (bits <= 16) return kNhHalf;
  if (bits <= 32) return kNhW1;
  if (bits <= 64) return kNhW2;
  if (bits <= 128) return kNhW4;
  if (bits <= 256) return kNhW8;
  return -1;
}

uint32_t nh_mode_lds_bytes(int mode, uint32_t V) { return 4u * nh_words_for(mode, V); }

}  // namespace openr_spf
