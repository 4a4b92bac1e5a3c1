// spf_bfs_common.h — helpers shared by the two uniform-cost BFS kernel families
// (spf_bfs.hip: packed level-code state; spf_bfs_lvl.hip: exact level bytes).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "spf_kernels.h"

// Profiling build (make prof): per-phase cycle counters of the level loop. Every stamp
// drains outstanding memory ops first, so a phase is charged for what it waited on.
#ifdef OPENR_SPF_PROFILE
#define OPENR_PROF_STAMP(var)                                   \
  do {                                                          \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    var = clock64();                                            \
  } while (0)
#define OPENR_PROF_ADD(i, a, b) pc[i] += (uint64_t)((b) - (a))
#else
#define OPENR_PROF_STAMP(var) \
  do {                        \
  } while (0)
#define OPENR_PROF_ADD(i, a, b) \
  do {                          \
  } while (0)
#endif

namespace openr_spf {
namespace bfs {

// LDS through address-space-3 pointers: constant offsets fold into the ds instruction
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u128;
__device__ __forceinline__ void lds_store4(uint32_t byte_addr, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
  u32x4 v = {x, y, z, w};
  *(lds_u128*)(size_t)byte_addr = v;
}

__device__ __forceinline__ uint32_t lds_or(lds_u32* p, uint32_t v) {
  return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add(lds_u32* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <typename T>
__device__ __forceinline__ void store_row(T* p, const T& x, bool nt) {
  if (nt)
    __builtin_nontemporal_store(x, p);  // streamed result rows: keep the CSR resident in L2
  else
    *p = x;
}

// Workgroup barrier for LDS only: global stores issued during a level stay in flight
// across it (__syncthreads()' release fence would drain them every level).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-launch device counters: [0] next unit (dynamic scheduling), [1] finished
// workgroups. The last workgroup to finish zeroes both (and `also_zero`), so every
// launch finds its counters zero without a memset.
__device__ __forceinline__ void retire_workgroup(uint32_t* ctr, uint32_t* also_zero) {
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1u) {
      ctr[0] = 0;
      ctr[1] = 0;
      if (also_zero) *also_zero = 0;
      __threadfence();
    }
  }
}

inline uint32_t env_u32(const char* name, uint32_t dflt, uint32_t lo, uint32_t hi) {
  if (const char* e = std::getenv(name)) {  // tuning knobs (benchmarks only)
    const long v = std::atol(e);
    if (v >= (long)lo && v <= (long)hi) return (uint32_t)v;
  }
  return dflt;
}

// Result rows are written once and read by the host / the next consumer, never by the
// kernel: non-temporal stores keep them from evicting the CSR mirror out of L2.
inline uint32_t nt_stores() { return 1u; }

// Counter block of a source class: [0,1] fast launch, [2,3] re-run launch, [4] solves
// the fast launch flagged for the re-run (cleared by the re-run's last workgroup).
inline uint32_t* class_counters(const SolveArgs& a) { return a.work + kCtrPerClass * a.cls; }

}  // namespace bfs
}  // namespace openr_spf
