/*
 * spf_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference SPF path of OpenR's Decision module:
 *   - LinkState::runSpf            /root/reference/openr/decision/LinkState.cpp:808-882
 *   - DijkstraQ / DijkstraQNode     /root/reference/openr/decision/LinkState.h:475-535
 *   - LinkState::getKthPaths        /root/reference/openr/decision/LinkState.cpp:762-791
 *   - LinkState::traceOnePath       /root/reference/openr/decision/LinkState.cpp:398-419
 * plus multi-threaded batch drivers over them (all-sources, KSP2 pairs, what-if units).
 *
 * It is the CHECKER for the HIP engine (openr_amd/csrc) and the CPU baseline
 * ("port") timed by bench.py. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product path never calls it.
 *
 * The reference itself is unbuildable in this image (it needs fbthrift-generated
 * Lsdb/Network types, folly, fb303 and glog); parity of this restatement is pinned
 * against the reference's own test expectations transcribed under tests/golden/
 * (LinkStateTest.cpp, DecisionTest.cpp), see DESIGN.md "Oracle".
 *
 * Graph input is the same CSR mirror the engine's C-ABI consumes
 * (include/openr_spf.h): row u lists the directed edges u->v in
 * LinkState::linksFromNode(u) iteration order.
 */
#ifndef OPENR_SPF_ORACLE_H
#define OPENR_SPF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t num_nodes;
  uint32_t num_dir_edges;
  uint32_t num_links;
  const uint32_t* row_ptr;         /* [V+1] */
  const uint32_t* col;             /* [E]   */
  const uint64_t* metric;          /* [E]   Link::getMetricFromNode(u), u64 */
  const uint32_t* link_id;         /* [E]   undirected link id < num_links   */
  const uint8_t* edge_up;          /* [E]   Link::isUp()                      */
  const uint8_t* node_overloaded;  /* [V]   LinkState::isNodeOverloaded()     */
  const uint32_t* name_rank;       /* [V]   rank under std::string operator<  */
} oracle_graph;

/* Number of distinct neighbours in row `src` (next-hop bit width for src). */
uint32_t oracle_num_distinct_neighbors(const oracle_graph* g, uint32_t src);

/*
 * One reference-faithful SPF run (Dijkstra with the (metric, name) heap order).
 *   ignore_links : NULL or bitmask over link ids (ceil(L/64) u64) = linksToIgnore
 *   out_dist     : [V] u64; UINT64_MAX for nodes absent from the SpfResult
 *   out_nh       : NULL or [V * nh_bytes]; bit i of node v = the src's i-th
 *                  distinct neighbour (row order) is in nextHops(v)
 *   out_order    : NULL or [V]; nodes in settle (extractMin) order
 *   out_pl_ptr   : NULL or [V+1]; pathLinks offsets per node
 *   out_pl_edge  : NULL or [E]; pathLinks as directed edge ids (prev = row owner)
 * Returns the number of settled nodes (SpfResult size), or -1 on error.
 */
int64_t oracle_run_spf(const oracle_graph* g, uint32_t src, int use_link_metric,
                       const uint64_t* ignore_links, uint64_t* out_dist,
                       uint8_t* out_nh, uint32_t nh_bytes, uint32_t* out_order,
                       uint32_t* out_pl_ptr, uint32_t* out_pl_edge);

/*
 * getKthPaths(src, dest, k): edge-disjoint paths as directed edge ids in
 * src->dest order. Paths are written back-to-back into out_edges with
 * out_path_ptr[i]..out_path_ptr[i+1] delimiting path i.
 * Returns the number of paths, or -1 on error / insufficient capacity.
 */
int64_t oracle_kth_paths(const oracle_graph* g, uint32_t src, uint32_t dest,
                         uint32_t k, uint32_t* out_path_ptr, uint32_t max_paths,
                         uint32_t* out_edges, uint32_t max_edges);

/*
 * All-sources driver used for the CPU baseline: runs oracle_run_spf for
 * sources[0..n) on `nthreads` pthreads (strided), writing dist[n][V] and
 * nh[n][V][nh_bytes] (either may be NULL). Returns 0 on success.
 */
int oracle_all_sources(const oracle_graph* g, const uint32_t* sources, uint32_t n,
                       int use_link_metric, uint64_t* dist, uint8_t* nh,
                       uint32_t nh_bytes, int nthreads);

/*
 * getKthPaths(src[i], dst[i], 1) and (.., 2) for n pairs on `nthreads` pthreads, as
 * token rows tok1 / tok2 [n][tok_cap] in the openr_spf_ksp2 layout
 * [n_paths, len_0, e.., len_1, e.., ...]; a pair that does not fit gets
 * n_paths = 0xFFFFFFFF. Returns 0 on success.
 */
int oracle_ksp2_batch(const oracle_graph* g, const uint32_t* src, const uint32_t* dst, uint32_t n,
                      uint32_t tok_cap, uint32_t* tok1, uint32_t* tok2, int nthreads);

/*
 * Per-link-failure what-if counts: changed[i][j] = nodes whose distance or next-hop
 * set differ between runSpf(sources[j], use, {links[i]}) and runSpf(sources[j], use)
 * (a node leaving the SpfResult counts). Sources are split across `nthreads`.
 */
int oracle_whatif(const oracle_graph* g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                  uint32_t n_sources, int use_link_metric, uint32_t* changed, int nthreads);

/*
 * The same sweep with a digest of each unit's delta (test infrastructure for
 * openr_spf_whatif_delta): digest[i][j] = sum mod 2^64 over the changed nodes v of
 * mix(v, new distance, new next-hop bytes [nh_bytes]) (delta_entry_hash, splitmix64
 * steps), so a delta is checked without shipping rows. Order-independent by construction.
 */
int oracle_whatif_delta_digest(const oracle_graph* g, const uint32_t* links, uint32_t n_links,
                               const uint32_t* sources, uint32_t n_sources, int use_link_metric,
                               uint32_t* changed, uint64_t* digest, uint32_t nh_bytes, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
