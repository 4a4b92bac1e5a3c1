/*
 * openr_spf.h — C-ABI of the MI355X-native SPF engine for OpenR's Decision module.
 *
 * This is the drop-in boundary under openr::LinkState. Each entry point names
 * the reference interface it replaces:
 *
 *   openr_spf_set_graph        LinkState topology mirror; call wherever the reference
 *                              clears its SPF memo: updateAdjacencyDatabase
 *                              (LinkState.cpp:714-717), deleteAdjacencyDatabase
 *                              (:730-731), decrementHolds (:509-512)
 *   openr_spf_solve            LinkState::runSpf(src, useLinkMetric)  (LinkState.cpp:808-882,
 *                              LinkState.h:436-443), batched over sources; the memoized
 *                              LinkState::getSpfResult (LinkState.cpp:793-803) and the
 *                              per-neighbour LFA solves of SpfSolver::getNextHopsWithMetric
 *                              (Decision.cpp:1170-1204) are batches of this call
 *   openr_spf_solve_ignore     LinkState::runSpf(src, true, linksToIgnore) as used by
 *                              getKthPaths k>=2 (LinkState.cpp:769-779) and per-link-failure
 *                              what-if sweeps; one (source, ignore-set) pair per solve
 *   openr_spf_solve_device     the same on device-resident buffers and a caller stream
 *                              (batched prefetch / benchmarks / multi-GPU shards)
 *   openr_spf_whatif           per-link-failure what-if sweep: runSpf(src, useLinkMetric, {link})
 *                              for every (link, source), reduced to changed-node counts
 *   openr_spf_whatif_delta     the same sweep plus each unit's changed nodes with their
 *                              new distance and next-hop bits
 *   openr_spf_ksp2             LinkState::getKthPaths(src, dst, 1 and 2) (LinkState.cpp:762-791)
 *                              for a batch of pairs, paths traced on the device
 *   openr_spf_patch_graph      attribute-only mirror updates (metric, Link::isUp, node
 *                              overload) at the same memo-clearing points, without a rebuild
 *   openr_spf_refresh          incremental re-SPF of resident rows after a patch: only the
 *                              rows the change can touch are re-solved
 *   openr_spf_last_error       glog CHECK / exception text of the reference
 *
 * Conventions
 *   - All functions return 0 (OPENR_SPF_OK) or a negative errno-style code; no C++
 *     exception crosses the ABI. openr_spf_last_error() returns a thread-local message.
 *   - Host output buffers are caller-owned. Device memory is library-owned except in
 *     openr_spf_solve_device, where every pointer is device memory owned by the caller.
 *   - A context is single-threaded (one per LinkState, matching the reference's
 *     threading: everything in Decision runs on one event-base thread). Host-buffer calls
 *     are synchronous on return.
 *   - There is no CPU fallback: if the HIP runtime or a device is unavailable,
 *     openr_spf_create fails with OPENR_SPF_ENODEV.
 *
 * Semantics (bit-exact with LinkState::runSpf, any metric values)
 *   dist[s][v]   u64 shortest distance (NodeSpfResult::metric), UINT64_MAX if v is not
 *                in the SpfResult (unreachable). dist[s][src] = 0. (With wrapped metrics a
 *                reached node's sum can itself be UINT64_MAX: openr_spf_solve_order's
 *                order[] tells the two apart.)
 *   nh[s][v][b]  next-hop set of v as a bitset over the source's DISTINCT neighbours in
 *                CSR row order: bit i (byte i/8, bit i%8) <-> the i-th distinct `col`
 *                value of row src (openr_spf_neighbor_map). nh bits of src itself are 0.
 *   tight[s][w]  (OPENR_SPF_EMIT_TIGHT) bit e of the E-bit mask is set iff directed edge e
 *                u->v is in NodeSpfResult::pathLinks(v). For metrics in [1, 2^31-1] these
 *                are the tight in-edges: usable, dist[u]+w(e)==dist[v], u may expand
 *                (u==src or !node_overloaded[u]); pathLinks(v) orders them by
 *                (dist[u], name_rank[u]) then by position of e in row u. In general
 *                pathLinks(v) orders them by the pop index of u (openr_spf_solve_order)
 *                then by row position.
 *   A directed edge is usable iff edge_up[e] and link_id[e] is not in the solve's
 *   ignore set. Overloaded nodes other than the source are reached but never expanded.
 *   Usable metrics in [1, 2^31-1] (the positive i32 Adjacency.metric range) run on the
 *   fast kernels. Zero or wrapped-negative metrics (an i32 < 0 stored as u64, sums wrap
 *   mod 2^64 as in the reference) make the pop order history-dependent; those graphs,
 *   next-hop sets wider than 256 and graphs beyond the LDS-resident layouts run on the
 *   exact-order kernel, which replays the reference's heap process (slower, same
 *   results). openr_spf_ksp2 needs metrics in [1, 2^31-1] (OPENR_SPF_ENOTSUP otherwise).
 */
#ifndef OPENR_SPF_H
#define OPENR_SPF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OPENR_SPF_ABI_VERSION 1

enum {
  OPENR_SPF_OK = 0,
  OPENR_SPF_EIO = -5,       /* HIP runtime error */
  OPENR_SPF_ENOMEM = -12,   /* host or device allocation failed */
  OPENR_SPF_ENODEV = -19,   /* no usable GPU / HIP runtime */
  OPENR_SPF_EINVAL = -22,   /* bad argument (null, out of range, no graph set) */
  OPENR_SPF_E2BIG = -7,     /* graph too large for the engine (see openr_spf_limits) */
  OPENR_SPF_ENOTSUP = -95,  /* KSP2 on a graph with a metric outside [1, 2^31-1] */
};

enum {
  OPENR_SPF_USE_LINK_METRIC = 1u << 0, /* runSpf useLinkMetric; else every hop costs 1 */
  OPENR_SPF_EMIT_TIGHT = 1u << 1,      /* fill tight[] (pathLinks reconstruction)      */
  OPENR_SPF_EMIT_ORDER = 1u << 2,      /* exact-order kernel (openr_spf_solve_order)  */
  OPENR_SPF_EMIT_LEVELS8 = 1u << 3,    /* solve_device: u8 level rows in d_dist (below) */
  OPENR_SPF_EMIT_LEVELS16 = 1u << 4,   /* solve_device: u16 level rows in d_dist        */
};

/* Sticky device-side conditions (openr_spf_take_status) */
enum {
  OPENR_SPF_STATUS_LEVEL_OVERFLOW = 1u, /* an EMIT_LEVELS8 row held a finite level > 254 (written 0xFE) */
};

typedef struct openr_spf_ctx openr_spf_ctx;

/* CSR mirror of LinkState::linkMap_ (LinkState.h:456-467). Row u lists u's
   directed edges in LinkState::linksFromNode(u) iteration order. Every link id
   appears exactly twice (u->v and v->u). Arrays are copied by set_graph. */
typedef struct {
  uint32_t num_nodes;               /* V */
  uint32_t num_dir_edges;           /* E */
  uint32_t num_links;               /* L: link ids are in [0, L) */
  const uint32_t* row_ptr;          /* [V+1] */
  const uint32_t* col;              /* [E] neighbour node id */
  const uint64_t* metric;           /* [E] Link::getMetricFromNode(u) (hold-aware value()) */
  const uint32_t* link_id;          /* [E] undirected link id */
  const uint8_t* edge_up;           /* [E] Link::isUp() */
  const uint8_t* node_overloaded;   /* [V] LinkState::isNodeOverloaded() */
  const uint32_t* name_rank;        /* [V] rank of the node name under std::string < */
} openr_spf_graph;

typedef struct {
  uint32_t max_nodes;       /* largest V the engine accepts */
  uint32_t max_nh_bits;     /* largest distinct degree (next-hop bitset width) */
} openr_spf_limits_t;

typedef struct {
  uint64_t spf_runs;        /* logical SPFs solved (fb303 decision.spf_runs) */
  uint64_t batches;         /* solve calls */
  double last_batch_ms;     /* wall time of the last host-buffer solve (decision.spf_ms) */
  double last_kernel_ms;    /* device time of the last solve's kernels (what-if sweep: its
                               repair kernel alone, HIP events around that launch) */
} openr_spf_stats_t;

int openr_spf_abi_version(void);
/* "<sha256/16 of the engine sources> <source files>" (Makefile build_id): lets the host
   verify the library was built from the sources it ships with. */
const char* openr_spf_build_id(void);
const char* openr_spf_last_error(void);
/* Diagnostics: "name;name;..." of the kernels the calling thread's last solve call
   (openr_spf_solve*, _solve_device) enqueued, re-run launches included (tests assert
   which kernel a configuration runs). */
const char* openr_spf_last_kernels(void);
void openr_spf_limits(openr_spf_limits_t* out);

/* device_ids: n_devices HIP ordinals (NULL -> the current device). Sources of one
   solve call are split in contiguous blocks across the devices. */
int openr_spf_create(const int* device_ids, int n_devices, openr_spf_ctx** out);
void openr_spf_destroy(openr_spf_ctx* ctx);

int openr_spf_set_graph(openr_spf_ctx* ctx, const openr_spf_graph* graph);

/* Minimum nh_bytes for the current graph: ceil(max distinct degree / 8), >= 1. */
int openr_spf_nh_bytes(const openr_spf_ctx* ctx, uint32_t* out_nh_bytes);

/* Distinct neighbours of src in row order (next-hop bit i -> out_nbrs[i]). */
int openr_spf_neighbor_map(const openr_spf_ctx* ctx, uint32_t src, uint32_t* out_nbrs,
                           uint32_t capacity, uint32_t* out_count);

/* Batched SPF from sources[0..n): dist [n][V]; nh [n][V][nh_bytes] (nh_bytes >=
   openr_spf_nh_bytes, or nh == NULL); tight [n][ceil(E/64)] or NULL. */
int openr_spf_solve(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n,
                    uint32_t flags, uint64_t* dist, uint8_t* nh, uint32_t nh_bytes,
                    uint64_t* tight);

/* As openr_spf_solve_ignore (ignore_ptr may be NULL: no ignore sets), plus order [n][V]:
   the index at which runSpf popped v from its queue (0 = the source), UINT32_MAX if v is
   not in the SpfResult. Always runs the exact-order kernel; pathLinks(v) = the tight[]
   in-edges of v sorted by order[u], then by row position (what LinkState needs when
   metrics can be zero). */
int openr_spf_solve_order(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n,
                          uint32_t flags, const uint32_t* ignore_ptr,
                          const uint32_t* ignore_links, uint64_t* dist, uint8_t* nh,
                          uint32_t nh_bytes, uint64_t* tight, uint32_t* order);

/* As openr_spf_solve with a per-solve ignore set: solve i ignores the links
   ignore_links[ignore_ptr[i] .. ignore_ptr[i+1]) (ignore_ptr has n+1 entries). */
int openr_spf_solve_ignore(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n,
                           uint32_t flags, const uint32_t* ignore_ptr,
                           const uint32_t* ignore_links, uint64_t* dist, uint8_t* nh,
                           uint32_t nh_bytes, uint64_t* tight);

/* Device-buffer form on device `device_index` of the context (an index into the
   device_ids given to create). All pointers are device memory; d_ignore_ptr may be
   NULL (no ignore sets); d_nh / d_tight may be NULL. `stream` is a hipStream_t
   (NULL = the context's own stream). Asynchronous: returns after enqueueing. */
/* With OPENR_SPF_EMIT_LEVELS8 / 16 the distance rows are written in level form instead:
   d_dist points to [n][V] u8 / u16 levels (level = dist / cost; all ones = not in the
   SpfResult) — the compact rows a strong-scaling rank all-gathers, 1 or 2 bytes per node
   instead of 8, emitted by the solve itself. Only for graphs on which every usable edge
   costs the same (or useLinkMetric off) and that run on the level BFS family (uniform-cost
   rows of <= 4 ELL slots, grids), with no ignore sets and no tight output: otherwise
   OPENR_SPF_ENOTSUP. A finite level above 254 in a u8 row is written as 0xFE and sets
   OPENR_SPF_STATUS_LEVEL_OVERFLOW (openr_spf_take_status): use u16 rows for such graphs. */
int openr_spf_solve_device(openr_spf_ctx* ctx, int device_index,
                           const uint32_t* d_sources, uint32_t n, uint32_t flags,
                           const uint32_t* d_ignore_ptr, const uint32_t* d_ignore_links,
                           uint64_t* d_dist, uint8_t* d_nh, uint32_t nh_bytes,
                           uint64_t* d_tight, void* stream);

/* Waits for device `device_index` to go idle, then returns the OPENR_SPF_STATUS_* bits
   its device-form calls raised since the last call (and clears them). */
int openr_spf_take_status(openr_spf_ctx* ctx, int device_index, uint32_t* out_status);

/* Per-link-failure what-if sweep (no reference API: the north-star what-if workload over
   LinkState::runSpf(src, useLinkMetric, {link}), LinkState.cpp:808-882 with the
   linksToIgnore argument getKthPaths uses at :769-779). Unit (i, j) fails links[i] for
   sources[j]; changed[i * n_sources + j] = number of nodes whose distance or next-hop
   set differs from the no-failure SPF of sources[j] (a node that becomes unreachable
   counts). A link with no tight edge in the base SPF cannot change the result: such
   units are 0 without a solve. *out_solved (nullable) = SPFs actually run (base solves
   + affected units), also added to stats.spf_runs. Links are split across devices. */
int openr_spf_whatif(openr_spf_ctx* ctx, const uint32_t* links, uint32_t n_links,
                     const uint32_t* sources, uint32_t n_sources, uint32_t flags,
                     uint32_t* changed, uint64_t* out_solved);

/* Device-buffer form (pointers are device memory; d_changed [n_links][n_sources]).
   Synchronizes `stream` once (the affected-unit count sizes the chunked solves).
   Link ids >= L are never affected (0). */
int openr_spf_whatif_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_links,
                            uint32_t n_links, const uint32_t* d_sources, uint32_t n_sources,
                            uint32_t flags, uint32_t* d_changed, void* stream,
                            uint64_t* out_solved);

/* What-if sweep with the per-unit delta (round 6): besides changed[], the nodes each
   failure changes, with their new distance and next-hop bits, i.e. the part of
   runSpf(sources[j], useLinkMetric, {links[i]}) (LinkState.cpp:808-882, SpfResult
   LinkState.h:436-443) that differs from the no-failure SPF. A consumer builds
   post-failure routes from it without solving again.
   Host form: a CSR over units u = i * n_sources + j. Unit u's entries are
   [ptr[u], ptr[u + 1]), with node ids ascending and ptr[n_units] = sum(changed).
   dist[k] is UINT64_MAX for a node the failure makes unreachable. nh[k] holds nh_bytes
   bytes in openr_spf_solve's row layout (bit b = the b-th distinct neighbour of the
   source), zero past the graph's width. nh_bytes must be >= that width.
   When sum(changed) > cap, ptr and changed are filled, the entries are not, and the call
   returns OPENR_SPF_E2BIG. The entries come from the repair's own overlays (and from the
   seeded re-solve of the few units too large for them): no second solve is run for them. */
typedef struct {
  uint64_t* ptr;     /* [n_links * n_sources + 1] */
  uint32_t* node;    /* [cap] */
  uint64_t* dist;    /* [cap] */
  uint8_t* nh;       /* [cap][nh_bytes] */
  uint64_t cap;      /* entries the caller allocated */
  uint32_t nh_bytes; /* bytes per next-hop entry */
} openr_spf_whatif_delta_t;
int openr_spf_whatif_delta(openr_spf_ctx* ctx, const uint32_t* links, uint32_t n_links,
                           const uint32_t* sources, uint32_t n_sources, uint32_t flags,
                           uint32_t* changed, openr_spf_whatif_delta_t* delta,
                           uint64_t* out_solved);

/* Device-buffer form (every buffer device memory): the same CSR, d_ptr [n_units + 1],
   with each unit's entries in the order the repair found them (not sorted). The repair
   writes into library scratch, a few slots per unit from per-wave blocks; a scan of
   changed and a gather then pack the caller's arrays. *out_total (host, nullable) =
   sum(changed). d_ptr and d_changed are always filled; when the total exceeds cap the
   entries are not, and the call returns OPENR_SPF_E2BIG (cap 0: counts and ptr only).
   Synchronizes `stream`. */
int openr_spf_whatif_delta_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_links,
                                  uint32_t n_links, const uint32_t* d_sources, uint32_t n_sources,
                                  uint32_t flags, uint32_t* d_changed, uint64_t* d_ptr,
                                  uint32_t* d_node, uint64_t* d_dist, uint8_t* d_nh, uint64_t cap,
                                  uint32_t nh_bytes, void* stream, uint64_t* out_total,
                                  uint64_t* out_solved);

/* LinkState::getKthPaths(src[i], dst[i], 1) and (.., 2) (LinkState.cpp:762-791, with
   traceOnePath :398-419) for a batch of pairs, traced on the device. Per pair, tok1 /
   tok2 [n_pairs][tok_cap] hold [n_paths, len_0, e.., len_1, e.., ...]: every path as
   its directed edge ids in src -> dest order (link = link_id[e]), paths in the
   reference's order; tokens past a row's used prefix are left unspecified. k = 2 ignores the links of the k = 1 paths. Link metrics are
   used (getKthPaths calls getSpfResult(src, true) / runSpf(src, true, ignore)). A pair
   whose paths exceed tok_cap tokens (or 255 hops) gets n_paths = 0xFFFFFFFF and the
   call returns OPENR_SPF_E2BIG after filling the others. */
int openr_spf_ksp2(openr_spf_ctx* ctx, const uint32_t* src, const uint32_t* dst, uint32_t n_pairs,
                   uint32_t tok_cap, uint32_t* tok1, uint32_t* tok2);

/* Device-buffer form: pair i = (d_sources[d_pair_row[i]], d_pair_dst[i]); the base SPF
   is solved once per listed source. Synchronizes `stream` once at the end. */
int openr_spf_ksp2_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_sources,
                          uint32_t n_sources, const uint32_t* d_pair_row,
                          const uint32_t* d_pair_dst, uint32_t n_pairs, uint32_t tok_cap,
                          uint32_t* d_tok1, uint32_t* d_tok2, void* stream);

/* Page-locked host memory for the caller-owned host buffers of the batch calls (the
   openr_spf_ksp2 token rows, solve rows): their device-to-host copies then run at link rate
   instead of through a pageable staging copy (the DecisionBenchmark G100 KSP2 update copied
   2 x 20 MB of token rows at ~2.3 GB/s). openr_spf_host_free(NULL) is a no-op. */
int openr_spf_host_alloc(size_t bytes, void** out);
void openr_spf_host_free(void* p);

/* In-place attribute patch of the mirror: the link structure —
   rows, columns, link ids — is unchanged; only attributes the reference changes on an
   existing Link / node move. Replaces a full openr_spf_set_graph at the reference's
   memo-clearing points when updateAdjacencyDatabase (LinkState.cpp:564-719) or
   decrementHolds (:500-514) changed nothing but:
     metric of directed edge e         Link::setMetricFromNode   (LinkState.cpp:195-204 getter)
     usability of link l (both edges)  Link::isUp: holds / adjacency overload (:233-236)
     overload of node x                LinkState::updateNodeOverloaded / isNodeOverloaded
   The patch is also recorded as a delta for openr_spf_refresh: the first patch after a
   refresh (or set_graph) starts a new delta, later patches with no refresh in between
   merge into it (each edge keeps its state from before the first of them). No solve may
   be in flight on the context's devices. */
typedef struct {
  uint32_t n_edges;
  const uint32_t* edge_ids;         /* [n_edges] directed edge ids */
  const uint64_t* metric;           /* [n_edges] new Link::getMetricFromNode(owner) */
  uint32_t n_links;
  const uint32_t* link_ids;         /* [n_links] */
  const uint8_t* link_up;           /* [n_links] new Link::isUp() */
  uint32_t n_nodes;
  const uint32_t* node_ids;         /* [n_nodes] */
  const uint8_t* node_overloaded;   /* [n_nodes] new isNodeOverloaded() */
} openr_spf_patch;

int openr_spf_patch_graph(openr_spf_ctx* ctx, const openr_spf_patch* patch);

/* Incremental re-SPF after openr_spf_patch_graph: rows [n] (dist, and nh / tight when
   non-NULL, laid out as openr_spf_solve writes them) hold the results of sources[0..n)
   on the graph before the delta (before the first patch since the last refresh); on
   return they hold the results on the patched graph, bit-exact with a fresh solve. Every
   refresh call of the same delta (e.g. one per batch of rows) sees the same delta. Only rows the patch can change are
   re-solved: row s is affected iff some changed directed edge u->v was tight for s
   before, or is usable with d_s(u) + w_new <= d_s(v) after (u expanding for s);
   *out_resolved (nullable) = rows re-solved (added to stats.spf_runs). Fails with
   OPENR_SPF_EINVAL when no patch followed the last set_graph. The host form splits the
   rows across devices like openr_spf_solve; the device form synchronizes `stream` once.
   Multi-device callers of the device form: the delta is per context, and any refresh
   ends its merging, so refresh the rows held on EVERY device before the next patch (a
   device whose rows skipped a delta would be refreshed against the later delta only and
   stay stale; the host LinkState mirror does this). */
int openr_spf_refresh(openr_spf_ctx* ctx, const uint32_t* sources, uint32_t n, uint32_t flags, uint64_t* dist,
                      uint8_t* nh, uint32_t nh_bytes, uint64_t* tight, uint32_t* out_resolved);
int openr_spf_refresh_device(openr_spf_ctx* ctx, int device_index, const uint32_t* d_sources, uint32_t n,
                             uint32_t flags, uint64_t* d_dist, uint8_t* d_nh, uint32_t nh_bytes,
                             uint64_t* d_tight, void* stream, uint32_t* out_resolved);

int openr_spf_get_stats(const openr_spf_ctx* ctx, openr_spf_stats_t* out);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_SPF_H */
