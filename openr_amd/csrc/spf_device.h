// spf_device.h — device helpers shared by the SPF kernels (LDS next-hop bitsets,
// wave-level compaction, ignore masks). Header-only; included by the .hip files.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace openr_spf {
namespace dev {

// ---------------------------------------------------------------------------
// Next-hop bitset storage in LDS
// ---------------------------------------------------------------------------
template <int MODE>
struct Nh;

// Packed modes (one node's set inside one dword): the first arrival at v is the one
// whose atomicOr sees v's field empty (every reached node's set is non-empty), so
// these modes elect the appending arrival without a separate visited bitmap.
template <uint32_t BITS>
struct NhPacked {
  static constexpr bool kSingle = true;
  static constexpr uint32_t kPer = 32u / BITS;
  static constexpr uint32_t kMask = BITS == 32 ? 0xFFFFFFFFu : ((1u << (BITS & 31u)) - 1u);
  static __host__ __device__ uint32_t words(uint32_t V) { return (V + kPer - 1u) / kPer; }
  static __device__ uint32_t word(uint32_t v) { return v / kPer; }
  static __device__ uint32_t shift(uint32_t v) { return (v % kPer) * BITS; }
  static __device__ void or_bit(uint32_t* nh, uint32_t v, uint32_t b) { atomicOr(&nh[word(v)], (1u << b) << shift(v)); }
  // OR bit b into v's set; returns the set's previous bits (0 <=> first arrival)
  static __device__ uint32_t fetch_or_bit(uint32_t* nh, uint32_t v, uint32_t b) {
    return (atomicOr(&nh[word(v)], (1u << b) << shift(v)) >> shift(v)) & kMask;
  }
  static __device__ void or_from(uint32_t* nh, uint32_t v, uint32_t u) {
    const uint32_t x = (nh[word(u)] >> shift(u)) & kMask;
    if (x) atomicOr(&nh[word(v)], x << shift(v));
  }
  static __device__ uint32_t byte(const uint32_t* nh, uint32_t v, uint32_t j) {
    return j * 8u < BITS ? (nh[word(v)] >> (shift(v) + 8u * j)) & (BITS < 8 ? kMask : 0xFFu) : 0u;
  }
  struct Val { uint32_t x; };
  static __device__ Val load(const uint32_t* nh, uint32_t u) { return {(nh[word(u)] >> shift(u)) & kMask}; }
  static __device__ void or_val(uint32_t* nh, uint32_t v, const Val& s) {
    if (s.x) atomicOr(&nh[word(v)], s.x << shift(v));
  }
};
template <> struct Nh<kNhNibble> : NhPacked<4> {};  // <= 4 bits (grids): eight nodes per dword
template <> struct Nh<kNhByte> : NhPacked<8> {};    // <= 8 bits: four nodes per dword
template <> struct Nh<kNhHalf> : NhPacked<16> {};   // <= 16 bits: two nodes per dword
template <> struct Nh<kNhW1> : NhPacked<32> {};     // <= 32 bits: one dword per node

template <int W>
struct NhWords {  // W dwords per node (W >= 2)
  static constexpr bool kSingle = false;  // arrivals are elected by a visited bitmap
  static __host__ __device__ uint32_t words(uint32_t V) { return V * W; }
  static __device__ void or_bit(uint32_t* nh, uint32_t v, uint32_t b) {
    atomicOr(&nh[v * W + (b >> 5)], 1u << (b & 31u));
  }
  static __device__ void or_from(uint32_t* nh, uint32_t v, uint32_t u) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      uint32_t x = nh[u * W + k];
      if (x) atomicOr(&nh[v * W + k], x);
    }
  }
  static __device__ uint32_t byte(const uint32_t* nh, uint32_t v, uint32_t j) {
    return j < 4u * W ? (nh[v * W + (j >> 2)] >> (8u * (j & 3u))) & 0xFFu : 0u;
  }
  struct Val { uint32_t x[W]; };
  static __device__ Val load(const uint32_t* nh, uint32_t u) {
    Val r;
#pragma unroll
    for (int k = 0; k < W; ++k) r.x[k] = nh[u * W + k];
    return r;
  }
  static __device__ void or_val(uint32_t* nh, uint32_t v, const Val& s) {
#pragma unroll
    for (int k = 0; k < W; ++k)
      if (s.x[k]) atomicOr(&nh[v * W + k], s.x[k]);
  }
};
template <> struct Nh<kNhW2> : NhWords<2> {};
template <> struct Nh<kNhW4> : NhWords<4> {};
template <> struct Nh<kNhW8> : NhWords<8> {};

__device__ __forceinline__ bool test_bit(const uint32_t* bits, uint32_t i) {
  return (bits[i >> 5] >> (i & 31u)) & 1u;
}

// Append `item` for every lane with `fresh` set; one LDS atomic per wave.
// Returns the slot index for fresh lanes. Must be reached by the whole wave.
__device__ __forceinline__ uint32_t wave_append(bool fresh, uint32_t* counter) {
  const unsigned long long m = __ballot(fresh);
  uint32_t base = 0;
  if (m) {
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    base += (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  }
  return base;
}

// Build the per-solve ignore mask (linksToIgnore) in LDS.
__device__ __forceinline__ void load_ignore(uint32_t* ign, uint32_t words, const SolveArgs& a,
                                            uint32_t sid, uint32_t L) {
  const uint32_t b = a.ign_ptr[sid], e = a.ign_end ? a.ign_end[sid] : a.ign_ptr[sid + 1];
  for (uint32_t k = b + threadIdx.x; k < e; k += blockDim.x) {  // any workgroup size
    const uint32_t l = a.ign_links[k];
    if (l < L) atomicOr(&ign[l >> 5], 1u << (l & 31u));
  }
  (void)words;
}

// Exclusive prefix of a small per-lane count (< 8) across the wave, via 3 ballots.
__device__ __forceinline__ uint32_t wave_prefix_small(uint32_t c, uint32_t* total) {
  const unsigned long long b0 = __ballot(c & 1u), b1 = __ballot(c & 2u), b2 = __ballot(c & 4u);
  const unsigned long long lt = (1ull << __lane_id()) - 1ull;
  *total = (uint32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
  return (uint32_t)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt));
}

}  // namespace dev
}  // namespace openr_spf
