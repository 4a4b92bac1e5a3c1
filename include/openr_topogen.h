/* openr_topogen.h — seeded synthetic topology generators (libopenr_decision.so).
 *
 * Benchmark/test inputs only; no reference API is replaced. The reference's own
 * generators (grid, fabric: openr/decision/tests/RoutingBenchmarkUtils.cpp:82-400) are
 * deterministic and restated in openr_amd/topology.py. The WAN topology of BASELINE
 * config 4 is new and is drawn here from the C++
 * standard library's std::mt19937_64 so that every consumer (Python bench, C++ tests,
 * a reference-side harness) gets the identical graph from the identical generator.
 *
 * Conventions as in openr_spf.h: extern "C", caller-owned buffers, 0 / negative errno.
 */
#ifndef OPENR_TOPOGEN_H
#define OPENR_TOPOGEN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* WAN: num_nodes nodes "wan{i}", a ring (i, i+1 mod n) plus uniform random chords
 * (a = rng() % n, b = rng() % n, rejected if a == b or already linked) up to num_links
 * links; then parallel_links extra copies of links[rng() % num_links]; then per-link
 * directional metrics metric_uv[l] = 1 + rng() % max_metric for every link, followed by
 * metric_vu[l] likewise. rng = std::mt19937_64(seed).
 * Outputs: ends [2 * (num_links + parallel_links)] (u, v per link), metric_uv / metric_vu
 * [num_links + parallel_links]. Fails with -22 on num_nodes < 3, num_links < num_nodes,
 * num_links > n(n-1)/2, max_metric < 1 or a null pointer. */
int openr_topogen_wan(uint32_t num_nodes, uint32_t num_links, uint32_t max_metric, uint64_t seed,
                      uint32_t parallel_links, uint32_t* ends, uint32_t* metric_uv, uint32_t* metric_vu);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_TOPOGEN_H */
