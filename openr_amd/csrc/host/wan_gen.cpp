// wan_gen.cpp — the WAN topology generator of BASELINE config 4 (include/openr_topogen.h).
//
// 1000 nodes, ring + uniform chords to 3000 links,
// per-direction metric 1 + rng() % 64, std::mt19937_64(seed = 1), optional parallel links.
#include <cstdint>
#include <random>
#include <unordered_set>

#include "../../../include/openr_topogen.h"

extern "C" int openr_topogen_wan(uint32_t num_nodes, uint32_t num_links, uint32_t max_metric, uint64_t seed,
                                 uint32_t parallel_links, uint32_t* ends, uint32_t* metric_uv,
                                 uint32_t* metric_vu) {
  if (num_nodes < 3 || num_links < num_nodes || max_metric < 1 || !ends || !metric_uv || !metric_vu) return -22;
  if ((uint64_t)num_links > (uint64_t)num_nodes * (num_nodes - 1) / 2) return -22;
  std::mt19937_64 rng(seed);
  std::unordered_set<uint64_t> seen;
  seen.reserve(num_links * 2u);
  auto key = [](uint32_t a, uint32_t b) { return a < b ? ((uint64_t)a << 32) | b : ((uint64_t)b << 32) | a; };
  uint32_t L = 0;
  for (uint32_t i = 0; i < num_nodes; ++i) {
    const uint32_t j = (i + 1) % num_nodes;
    ends[2 * L] = i;
    ends[2 * L + 1] = j;
    seen.insert(key(i, j));
    ++L;
  }
  while (L < num_links) {
    const uint32_t a = (uint32_t)(rng() % num_nodes);
    const uint32_t b = (uint32_t)(rng() % num_nodes);
    if (a == b || !seen.insert(key(a, b)).second) continue;
    ends[2 * L] = a;
    ends[2 * L + 1] = b;
    ++L;
  }
  for (uint32_t i = 0; i < parallel_links; ++i) {
    const uint32_t k = (uint32_t)(rng() % num_links);
    ends[2 * L] = ends[2 * k];
    ends[2 * L + 1] = ends[2 * k + 1];
    ++L;
  }
  for (uint32_t l = 0; l < L; ++l) metric_uv[l] = 1u + (uint32_t)(rng() % max_metric);
  for (uint32_t l = 0; l < L; ++l) metric_vu[l] = 1u + (uint32_t)(rng() % max_metric);
  return 0;
}
