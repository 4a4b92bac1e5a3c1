// spf_kernels.h — device-side graph layout and kernel launchers of the SPF engine.
//
// One workgroup owns one solve at a time (persistent loop over the batch): the
// per-solve state (levels / distances, next-hop bitsets, frontier) lives in LDS,
// the CSR mirror is streamed from L2/HBM and shared by every workgroup.
// See DESIGN.md "Kernels" for the roofline accounting.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

namespace openr_spf {

// Device copy of the CSR mirror (include/openr_spf.h openr_spf_graph), packed for
// the kernels. Built once per openr_spf_set_graph on every device of the context.
struct DevGraph {
  uint32_t V = 0, E = 0, L = 0;
  uint32_t max_deg = 0;        // largest row (source expansion must fit the frontier queue)
  uint32_t est_width2 = 0;     // sampled max |level L| + |level L+1| of a BFS (ring sizing)
  uint32_t est_width1 = 0;     // sampled max |level L| (lean BFS pass: queue halves)
  uint32_t est_depth = 0;      // sampled max BFS depth (family choice, u8 level limit)
  uint32_t* row = nullptr;     // [V+1]
  uint2* row2 = nullptr;       // [V] (row[u], row[u+1]) in one 8-byte load
  uint2* row2t = nullptr;      // [V] transit row: row2[u], or an empty range when u is overloaded
                               //     (an overloaded node other than the source is never expanded)
  uint32_t* ovl_bits = nullptr;  // [ceil(V/32)] overloaded bitmap (staged into LDS)
  uint4* ellt = nullptr;       // [V] first 4 edges of each transit row (adj encoding, kEdgeDown-padded)
  uint4* ellv = nullptr;       // [ellv_rows(V)] ellt with every down / padding slot replaced by the node id V (a
                               //     level sentinel the lvl kernel keeps at 0: never tight, no flag tests);
                               //     ellv[V] = (V, V, V, V), the row of a lane past the frontier;
  uint32_t* elld = nullptr;    // [V] ellv as four signed byte deltas (v - u; 0 = no edge), or null
  // [E] erec with every row's entries sorted by (name rank of the neighbour, reverse edge):
  // for uniform cost that is the reference's pathLinks order (DijkstraQ pops equal
  // distances by name; LinkState.cpp:820-829), so the KSP tracer ranks a frame's
  // candidates by their position alone
  uint4* erecs = nullptr;
                               //     when a row has > 4 edges or a column > 127 ids away (wave pass)
  uint32_t* adj = nullptr;     // [E] col | kEdgeDown when !edge_up
  uint32_t* w = nullptr;       // [E] metric u->v (u32; usable edges are in [1, 2^31-1])
  uint64_t* w64 = nullptr;     // [E] metric u->v as the caller gave it (exact-order kernel: 0 / wrapped values)
  uint32_t* win = nullptr;     // [E] metric of the reverse edge (col -> row owner)
  uint32_t* rev = nullptr;     // [E] index of the reverse edge
  uint32_t* lid = nullptr;     // [E] undirected link id
  uint16_t* nbr = nullptr;     // [E] distinct-neighbour index of col within its row
  uint8_t* ovl = nullptr;      // [V] overloaded
  uint8_t* cls = nullptr;      // [V] source class of each node, code family (SrcClass)
  uint8_t* cls_lvl = nullptr;  // [V] source class of each node, lvl family (LvlClass)
  uint2* ledge = nullptr;      // [L] the two directed edges of each link (UINT32_MAX if unused)
  uint32_t* rank = nullptr;    // [V] name rank (pathLinks / pop-order tie-break)
  uint4* erec = nullptr;       // [E] packed edge e = u->col: {col | kEdgeDown | kNodeSink if col is
                               //     overloaded, win[e], lid[e], rev[e]} (one 16-byte load per edge)
};

constexpr uint32_t kEdgeDown = 0x80000000u;
// Sink flag of a transit row: ellt[u].x and row2t[u].x carry it when u is overloaded.
// (row2t of a sink is an empty range whose begin carries the flag, so it never loops.)
constexpr uint32_t kNodeSink = 0x40000000u;
constexpr uint32_t kBlock = 256;
// ellv slot of an ellt slot: the column, or V for a down / padding / sink-row slot
__host__ __device__ inline uint4 ellv_of(uint4 t, uint32_t V) {
  auto f = [V](uint32_t x) { return (x & kEdgeDown) ? V : x; };
  return make_uint4(f(t.x), f(t.y), f(t.z), f(t.w));
}
// elld row of an ellv row: the four slots as signed byte deltas v - u (0: V, no edge)
__host__ __device__ inline uint32_t elld_of(uint4 r, uint32_t u, uint32_t V) {
  auto d = [u, V](uint32_t x) -> uint32_t { return x >= V ? 0u : (uint32_t)(uint8_t)(int8_t)((int32_t)x - (int32_t)u); };
  return d(r.x) | (d(r.y) << 8) | (d(r.z) << 16) | (d(r.w) << 24);
}
constexpr uint32_t kBfsEdgesPerLane = 4;  // edges a lane loads ahead per pass (register prefetch)
constexpr uint32_t kBfsTargetWgs = 12;    // lvl BFS sizes its ring for this many workgroups per CU (G100: 8 -> 1.06 ms, 9..16 -> 1.02 ms)

// Next-hop bitset storage classes in LDS (chosen from the max distinct degree).
enum NhMode : int { kNhByte = 0, kNhHalf = 1, kNhW1 = 2, kNhW2 = 3, kNhW4 = 4, kNhW8 = 5, kNhNibble = 6 };
int nh_mode_for_bits(uint32_t bits);            // -1 if > 256 bits
uint32_t nh_mode_lds_bytes(int mode, uint32_t V);
uint32_t nh_words_for(int mode, uint32_t V);     // LDS dwords of V next-hop sets
bool nh_mode_single(int mode);                  // one node's set lives inside one dword
// persistent grid: workgroups that fit a CU by LDS (<= 2048 threads) x CUs, <= n
uint32_t blocks_for(uint32_t n, uint32_t lds, int num_cus, uint32_t block = 256);

struct LaunchInfo {
  uint32_t lds_bytes = 0;
  uint32_t grid = 0;
  const char* kernel = "";
};
// Launch trace (openr_spf_last_kernels): every solve launcher records the kernel it
// enqueued; the C-ABI clears the calling thread's trace at the start of each solve call.
void note_launch(const char* kernel);
void clear_launch_trace();

// Optional per-unit delta of a what-if sweep (openr_spf_whatif_delta): the nodes whose
// distance or next-hop set a unit's failure changes, with their new values. Unit u's
// entries are pool slots [off[u], off[u] + changed[u]) in no particular order; a unit
// reserves its slots with one atomic on `used`, and slots past `cap` are not written
// (used then exceeds cap: the caller reports OPENR_SPF_E2BIG).
struct WhatifDelta {
  uint32_t* off = nullptr;             // [units] (unit = link index * n_src + source index)
  uint32_t* node = nullptr;            // [cap] node id; null: no delta output
  unsigned long long* dist = nullptr;  // [cap] new distance (UINT64_MAX: not reached)
  uint8_t* nh = nullptr;               // [cap][nhb] new next-hop bits, zero padded past the graph's width
  uint32_t cap = 0, nhb = 0;
  unsigned long long* used = nullptr;  // pool cursor (device counter, zeroed by the launcher)
  __device__ uint32_t base_of(unsigned long long b) const { return b < 0xFFFFFFFFull ? (uint32_t)b : 0xFFFFFFFFu; }
};

struct SolveArgs {
  const uint32_t* sources;
  uint32_t n;
  const uint32_t* ign_ptr;    // nullable: solve i ignores ign_links[ign_ptr[i], end_i)
  const uint32_t* ign_links;
  const uint32_t* ign_end;    // nullable: end_i = ign_end[i], else ign_ptr[i + 1]
  uint64_t* dist;             // [n][V]
  uint8_t* nh;                // nullable [n][V][nh_bytes]
  uint32_t nh_bytes;
  uint64_t* tight;            // nullable [n][ceil(E/64)] (zeroed by the launcher)
  uint32_t nh_bits;           // bits that are meaningful (max distinct degree)
  uint32_t* ovf_list;         // [n * nsl] scratch: units the ring variant could not finish (re-run list)
  uint32_t* work;             // [kWorkSlots] per-class launch counters (zero at rest: kernels reset them)
  // Source classes (next-hop width): when perm != nullptr this launch solves only the
  // sources of class `cls`: solve k < part[cls] is sid = perm[part[kMaxClasses + cls] + k]
  // (part / perm in device memory, built by partition_sources or the host).
  const uint32_t* perm;
  const uint32_t* part;       // [2 * kMaxClasses]: counts, then offsets
  uint32_t cls;
  uint32_t nsl;               // next-hop slices per solve (sliced class), else 1
  uint32_t dist_only;         // code family: no next-hop output, so no next-hop bits (one class);
                              // bit 1: the KSP2 target's pull test (2) in its per-wave form (A/B)
  // nullable, honoured by dist_only code-family solves: solve sid may stop once the level
  // of target[sid] is known; nodes at the target's distance or farther, other than the
  // target, then read UINT64_MAX (a KSP trace to the target only reads nodes nearer)
  const uint32_t* target;
  // nullable, dist_only code-family solves (GENERIC kernels) only: write u16 level rows
  // [n][V] here instead of u64 distance rows (0xFFFF = unreached; dist = level * cost;
  // levels stay below V <= 65535). KSP2 second SPFs: 4x fewer bytes per pair row.
  uint16_t* lvl16;
  // lvl16 rows in tagged form when lvl_tag != 0 (KSP2 second SPFs, round 3): a node's entry
  // is (lvl_tag << lvl_shift) | level, written only when the node is settled; the unreached
  // fill is skipped, so a row costs the bytes of the nodes the (target-bounded) solve
  // reached, and an entry with another tag reads as unreached. Levels < V < 2^lvl_shift.
  uint32_t lvl_tag, lvl_shift;
  // nullable: solve sid writes its dist / nh / tight rows at row out_row[sid] instead of
  // sid (openr_spf_refresh re-solves a scattered subset of resident rows in place; the
  // launcher then leaves zeroing those tight rows to the caller)
  const uint32_t* out_row;
  unsigned long long* prof;   // profiling builds only: per-phase cycle sums (nullable)
  uint32_t* order;            // nullable [n][V]: pop index per node (exact-order kernel only)
  // nullable, level family (OPENR_SPF_EMIT_LEVELS8 / 16): level rows [n][V] of lvl_bytes
  // (1 or 2) per node here instead of the u64 distance rows (dist = level x cost; all
  // ones = unreached); a finite level a u8 row cannot hold is written 0xFE and sets
  // kStatusLevelOverflow in *status
  uint8_t* lvl_rows;
  uint32_t lvl_bytes;
  // nullable, rounds kernel with an ignore set (what-if re-solves of large units, round 4):
  // solve sid starts from base row j = seed_unit[sid] % seed_nsrc of seed_dist / seed_tight
  // (the source's SPF without the ignore set, and its tight-edge mask) instead of from
  // scratch: only the nodes whose distance the ignored links raise are re-solved
  const uint64_t* seed_dist;
  const uint64_t* seed_tight;
  const uint32_t* seed_unit;
  uint32_t seed_nsrc;
  // nullable with seed_dist: instead of writing rows, compare the solve with the base rows
  // (seed_dist, seed_nh: nh_bytes per node) and store the count of nodes whose distance or
  // next-hop bytes differ at seed_changed[seed_unit[sid]] (the what-if unit's answer)
  const uint8_t* seed_nh;
  uint32_t* seed_changed;
  WhatifDelta delta;  // with seed_changed: the unit's changed nodes and their new rows (node == null: off)
  // rounds kernel: tin_out (nullable, solves without a seed) receives each solve's tight
  // in-degree row [out_row][V] (u16); seed_tin (nullable, with seed_dist) is such a row set
  // for the base SPF, so a seeded start reads the counts instead of scanning every in-edge
  uint16_t* tin_out;
  const uint16_t* seed_tin;
  // nullable (rounds kernel, generic): the solve count is min(n, *n_dev), read on the device
  // (n sizes the grid; n_block = threads per solve, 64 / 128 / 256) -- no host round trip
  // for a count the previous kernel produced
  const uint32_t* n_dev;
  uint32_t n_block;
  unsigned long long* prof_solve;  // nullable (OPENR_SPF_PROF): rounds kernel per-solve wall-clock start / end
  uint32_t* status;
  // code-family sliced class with next-hop output: [krows][nsl][V] 29-bit chunks of the
  // sets (slice s = bits [29s, 29s + 29)); launch_bfs_code merges them into nh rows
  uint32_t* slice_tmp;
  // sliced class with next-hop output, chunked: this launch solves the class-local solves
  // [k0, k0 + krows) and slice_tmp holds krows of them (row k - k0); krows 0 = the whole class
  uint32_t k0, krows;
};
__host__ __device__ constexpr uint32_t ellv_rows(uint32_t V) { return V + 1u; }
// output row of solve sid (SolveArgs::out_row)
__host__ __device__ inline size_t out_row_of(const SolveArgs& a, uint32_t sid) {
  return a.out_row ? (size_t)a.out_row[sid] : (size_t)sid;
}
constexpr uint32_t kMaxClasses = 8;
constexpr uint32_t kCtrPerClass = 8;  // [0,1] fast launch, [2,3] re-run launch, [4] flagged solves
constexpr uint32_t kWorkSlots = kCtrPerClass * kMaxClasses;
constexpr uint32_t kStatusLevelOverflow = 1u;  // = OPENR_SPF_STATUS_LEVEL_OVERFLOW
constexpr uint32_t kFringeCtr = kCtrPerClass * (kMaxClasses - 1);  // BFS classes use < 7 blocks
constexpr uint32_t kIncrCtr = kFringeCtr + 2;                        // incremental what-if
constexpr uint32_t kExactCtr = kIncrCtr + 2;                         // exact-order kernel

// Uniform-cost BFS kernel families (spf_capi.hip picks one per graph):
//  * code (spf_bfs.hip): one packed LDS field per node = [next-hop bits | 3-bit level
//    code]; distances stored when a node is expanded. Smallest LDS footprint, best on
//    shallow graphs with wide frontiers (fabrics).
//  * lvl (spf_bfs_lvl.hip): exact u8/u16 level per node + packed next-hop sets; the
//    distance row is written coalesced at the end. Best on deep graphs (grids).
enum BfsFamily : int { kFamCode = 0, kFamLvl = 1, kNumFamilies = 2 };

// Source classes by distinct degree (next-hop bitset width).
// code family: the per-node field holds the set plus a 3-bit level code in 8 bits
// (d <= 5), 16 bits (d <= 13) or 32 bits (d <= 29); d > 29 solves in ceil(d / 29)
// slices of 29 next-hop bits, one workgroup pass per slice, merged into bytes afterwards.
enum SrcClass : int { kCls8 = 0, kCls16 = 1, kCls32 = 2, kClsSliced = 3, kNumClasses = 4 };
// lvl family: next-hop sets of 4 / 8 / 16 / 32 bits; d > 32 in 32-bit slices.
enum LvlClass : int { kLvl4 = 0, kLvl8 = 1, kLvl16 = 2, kLvl32 = 3, kLvlSliced = 4, kNumLvlClasses = 5 };
int src_class_for_degree(int family, uint32_t distinct_degree);  // -1 if > 256
int num_classes(int family);
int sliced_class(int family);
uint32_t slice_bits(int family);
// Stable within a class is not required: perm maps class-local index -> sid.
hipError_t launch_partition(const uint32_t* d_sources, uint32_t n, const uint8_t* d_node_cls, uint32_t V,
                            uint32_t* d_part, uint32_t* d_perm, hipStream_t s);

// Uniform edge cost c (all usable edges cost c, or useLinkMetric=false): BFS levels,
// sources of class a.cls of `family` (a.nsl slices for the sliced class).
hipError_t launch_bfs(int family, const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes,
                      int num_cus, hipStream_t s, LaunchInfo* info);
hipError_t launch_bfs_code(const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes, int num_cus,
                           hipStream_t s, LaunchInfo* info);
hipError_t launch_bfs_lvl(const DevGraph& g, const SolveArgs& a, uint64_t cost, int group_lanes, int num_cus,
                          hipStream_t s, LaunchInfo* info);

// General positive metrics (spf_fringe.hip): one wavefront per solve, settle-safe
// buckets of width delta = min usable metric over a fringe list, next hops pulled over
// tight in-edges. Uses a.work[kFringeCtr, +2) for dynamic scheduling.
hipError_t launch_fringe(const DevGraph& g, const SolveArgs& a, uint32_t delta, bool dist64,
                         int nh_mode, int num_cus, hipStream_t s, LaunchInfo* info);
// General positive metrics on shallow graphs (spf_rounds.hip): Bellman-Ford distance
// rounds, then next hops in Kahn order of the tight DAG. Same counters as the fringe.
hipError_t launch_rounds(const DevGraph& g, const SolveArgs& a, bool dist64, int nh_mode, int num_cus,
                         hipStream_t s, LaunchInfo* info);
uint32_t rounds_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64);

// What-if sweep (spf_sweep.hip): unit u = i * n_src + j (links[i] failed, sources[j]).
// Filter: changed[u] = 0 for every unit; units whose link has a tight edge in
// base_tight[j] are appended to (wsrc, wlink, wunit), *wcount of them.
hipError_t launch_whatif_filter(const DevGraph& g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                                uint32_t n_src, const uint64_t* base_tight, uint32_t* changed, uint32_t* wsrc,
                                uint32_t* wlink, uint32_t* wunit, uint32_t* wcount, int num_cus, hipStream_t s);
// changed[wunit[k]] = nodes whose dist / next-hop bytes differ from base row wunit[k] % n_src.
// With dl.node: also the unit's changed nodes and their new rows (WhatifDelta).
hipError_t launch_rows_compare(uint32_t n, uint32_t V, uint32_t nb, const uint64_t* dist, const uint8_t* nh,
                               const uint64_t* base_dist, const uint8_t* base_nh, const uint32_t* wunit,
                               uint32_t n_src, uint32_t* changed, const WhatifDelta& dl, int num_cus, hipStream_t s);
// What-if delta compaction: ptr[0, n] = exclusive scan of changed (tsum: one u64 per
// 4096 units of scratch), then every unit's entries from its pool slots (off) to its CSR
// slots (ptr) in node / dist / nh.
hipError_t launch_delta_scan(const uint32_t* changed, size_t n, unsigned long long* tsum, unsigned long long* ptr,
                             hipStream_t s);
hipError_t launch_delta_gather(const uint32_t* changed, size_t n, const uint32_t* off, const unsigned long long* ptr,
                               const WhatifDelta& pool, uint32_t* node, unsigned long long* dist, uint8_t* nh,
                               int num_cus, hipStream_t s);
hipError_t launch_iota(uint32_t* p, uint32_t n, int num_cus, hipStream_t s);
// Incremental what-if (spf_sweep.hip): changed[wunit[k]] for every listed unit from the
// base rows alone (no full re-solve). Uses a.work-style counters `ctr` (2 slots).
hipError_t launch_whatif_incr(const DevGraph& g, const uint32_t* wsrc, const uint32_t* wlink, const uint32_t* wunit,
                              uint32_t count, uint32_t n_src, const uint64_t* base_dist, const uint8_t* base_nh,
                              uint32_t nb, bool unit_cost, bool dist64, uint32_t* changed, uint32_t* ctr,
                              int num_cus, hipStream_t s);
uint32_t whatif_incr_lds_bytes(uint32_t V, uint32_t nb, bool dist64);
// Grouped what-if (spf_sweep.hip, the default): one workgroup per (source, chunk of links)
// stages the source's base rows (dist, next hops, tight mask) in LDS once; its wavefronts
// filter the links (no tight edge -> 0) and repair the affected ones on private overlays.
// Writes every changed[i * n_src + j]; affected[0] = affected units, affected[1] = units
// that outgrew the dirty slots (listed in ovf_*[0, affected[1]) for a re-solve). With
// dl.node, every repaired unit also writes its delta (WhatifDelta).
hipError_t launch_whatif_group(const DevGraph& g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                               uint32_t n_src, const uint64_t* base_dist, const uint8_t* base_nh,
                               const uint64_t* base_tight, const uint16_t* base_tin, uint32_t nb, bool unit_cost, bool dist64, uint32_t w_max,
                               uint32_t nh_bits, uint32_t* changed, uint32_t* changed_t, uint32_t* affected,
                               uint32_t* ovf_src, uint32_t* ovf_link, uint32_t* ovf_unit, uint32_t* ctr,
                               const WhatifDelta& dl, int num_cus, hipStream_t s);
// 0 when the grouped repair cannot run on the graph (ids, next-hop width, degree, LDS)
uint32_t whatif_group_lds_bytes(uint32_t V, uint32_t E, uint32_t nb, bool dist64, uint32_t max_deg);

// Incremental mirror updates (spf_update.hip).
// In-place attribute patch of the device mirror: each record overwrites one element of
// one DevGraph array (structure — rows, columns, link ids — never changes).
enum PatchArray : uint32_t {
  kPatchAdj = 0, kPatchW, kPatchWin, kPatchErec, kPatchEllt, kPatchRow2t, kPatchOvl, kPatchOvlBits, kPatchEllv,
  kPatchW64,  // val.x = low, val.y = high word
  kPatchElld,
  kPatchErecS,  // DevGraph::erecs (idx = sorted position)
  kNumPatchArrays
};
struct PatchRec {
  uint32_t arr, idx, pad0, pad1;
  uint4 val;  // x (u32 / u8 arrays), xy (uint2), xyzw (uint4)
};
hipError_t launch_patch_apply(const DevGraph& g, const PatchRec* recs, uint32_t n, hipStream_t s);
// One directed edge u->v whose usability / weight / tail overload changed in a patch.
struct DeltaEdge {
  uint32_t u, v, w0, w1;  // weight before / after (u32; usable metrics are i32-positive)
  uint32_t flags, pad0, pad1, pad2;
};
constexpr uint32_t kDeltaUp0 = 1u, kDeltaUp1 = 2u, kDeltaOvl0 = 4u, kDeltaOvl1 = 8u;
// Refresh filter: row i (source sources[i], distances dist[i][V] of the graph before the
// patch) is affected iff some delta edge was tight for it or may now be tight / shorter;
// affected rows are appended to alist (row index) / asrc (source), *count of them.
hipError_t launch_refresh_filter(const DeltaEdge* delta, uint32_t n_delta, const uint32_t* sources, uint32_t n,
                                 uint32_t V, const uint64_t* dist, bool unit_cost, uint32_t* alist, uint32_t* asrc,
                                 uint32_t* count, int num_cus, hipStream_t s);
// Exact second stage: of the *count_in rows the filter listed, those whose dist or next-hop
// rows the change really moves (needs the next-hop rows; nb <= 32); n_max bounds *count_in.
hipError_t launch_refresh_exact(const DevGraph& g, const DeltaEdge* delta, uint32_t n_delta, uint32_t V,
                                const uint64_t* dist, const uint8_t* nh, uint32_t nb, bool unit_cost,
                                const uint32_t* alist_in, const uint32_t* asrc_in, const uint32_t* count_in,
                                uint32_t n_max, uint32_t* alist, uint32_t* asrc, uint32_t* count, int num_cus,
                                hipStream_t s);
// rows[alist[k]][0 .. words) = 0 for k < n
hipError_t launch_zero_rows(uint64_t* rows, uint32_t words, const uint32_t* alist, uint32_t n, int num_cus,
                            hipStream_t s);

// KSP2 tracing (spf_ksp.hip), one wavefront per (src, dest) pair of a chunk.
constexpr uint32_t kKspMaxDepth = 256;  // DFS frames (hops of a traced shortest path)
constexpr uint32_t kKspArena = 1024;    // sorted pathLinks of the frames on the DFS stack
struct KspCaps {
  uint32_t frames, arena;
};
KspCaps ksp_caps(const DevGraph& g, bool full);  // small tier (occupancy) or full tier
// kind 1 writes the k = 1 links to ign_io[k * ign_cap, ign_end[k]); kind 2 ignores them.
// Small tier: retry_list != null; pairs that outgrow it are appended there (count in
// *retry_count). Full tier: retry_list == null; with `list` it traces only the chunk-local
// pairs list[0 .. *list_count).
hipError_t launch_ksp_trace(int kind, const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                            const uint32_t* pdst, uint32_t first, uint32_t n, const uint64_t* rows, uint32_t* ign_io,
                            uint32_t* ign_end, uint32_t ign_cap, uint32_t* tok, uint32_t tok_cap, uint32_t* status,
                            uint32_t* qbuf, int num_cus, hipStream_t s, unsigned long long* stats = nullptr,
                            const uint32_t* list = nullptr, const uint32_t* list_count = nullptr,
                            uint32_t* retry_list = nullptr, uint32_t* retry_count = nullptr,
                            uint32_t* work_ctr = nullptr,  // zeroed dynamic-scheduling counter (required)
                            const uint16_t* rows16 = nullptr,  // kind 2: u16 level rows (SolveArgs::lvl16)
                            uint64_t lcost = 0,   // instead of `rows`: dist = level * lcost; non-zero lcost
                                                  // also marks a uniform-cost graph (rank by name / edge)
                            uint32_t ltag = 0,    // rows16 tagged (SolveArgs::lvl_tag): tag << 8 | lvl_shift
                            // uniform cost: the sources' pathLinks lists (launch_ksp_path_lists), row
                            // prow[pair] of each. Kind 1 reads them instead of gathering from the records
                            // and rows; kind 2 reads them for the nodes its pair's row leaves at their
                            // base distance (tl_rows: the base rows the lists were built from)
                            const uint32_t* tl_off = nullptr, const uint2* tl_ent = nullptr,
                            const uint64_t* tl_rows = nullptr,
                            // kind 2: rows16 from launch_ksp_repair where rmode[k] == 0 (base fallback)
                            const uint32_t* rmode = nullptr);
// KSP2 second SPF as a repair of the base SPF (uniform cost `cost`): for chunk-local pair k
// (list[0 .. *list_count) when list is set), source srcs[k] of base row prow[k] (base_rows,
// pathLinks list offsets tl_off: launch_ksp_path_lists), dest tgts[k], ignoring
// ign_links[ign_ptr[k], ign_end[k]): rows16[k][v] = ltag | level for the nodes whose
// distance the ignored links change (lmask: unreached or at / beyond dest's level); every
// other node keeps its base distance (the k = 2 trace's `repaired` mode reads it there).
// Requires levels < lmask. A pair whose affected set outgrows a cap gets mode[k] = 1 and
// is appended to retry_list (*retry_count) for the forward solve; else mode[k] = 0.
// work_ctr: zeroed dynamic-scheduling counter.
uint32_t ksp_repair_lds_bytes(uint32_t V, uint32_t L);  // 0: the graph does not fit
hipError_t launch_ksp_repair(const DevGraph& g, const uint32_t* srcs, const uint32_t* prow, const uint32_t* tgts,
                             const uint32_t* list, const uint32_t* list_count, uint32_t n, const uint32_t* ign_ptr,
                             const uint32_t* ign_end, const uint32_t* ign_links, const uint64_t* base_rows,
                             const uint32_t* tl_off, uint64_t cost, uint16_t* rows16, uint32_t ltag, uint32_t lmask,
                             uint32_t* mode, uint32_t* retry_list, uint32_t* retry_count, uint32_t* work_ctr,
                             int num_cus, hipStream_t s);
// The k = 1 trace's pathLinks lists: for base row j (source sources[j], distances rows[j]),
// off[j][0 .. V] (V + 1 u32) and ent[j][off[v] .. off[v + 1]) = node v's tight in-edges in
// rank order as {u->v edge, link | u << 16} (ent holds E entries per source). Needs
// DevGraph::erecs and ids below 2^16 (ksp_path_lists_ok; OPENR_SPF_KSP_TL=0 turns it off).
bool ksp_path_lists_ok(const DevGraph& g);
hipError_t launch_ksp_path_lists(const DevGraph& g, const uint32_t* sources, uint32_t n_src, const uint64_t* rows,
                                 uint32_t* off, uint2* ent, int num_cus, hipStream_t s);
uint32_t ksp_stats_count();  // counters a stats buffer holds (OPENR_SPF_PROF tuning only)
uint32_t ksp_max_grid(const DevGraph& g, int num_cus);  // qbuf must hold ksp_max_grid * (V + ceil(V / 32)) u32
hipError_t launch_strided_iota(uint32_t* p, uint32_t n, uint32_t stride, int num_cus, hipStream_t s);
hipError_t launch_gather_sources(const uint32_t* sources, const uint32_t* prow, uint32_t first, uint32_t n,
                                 uint32_t* out, int num_cus, hipStream_t s);
// After the k = 1 trace of a chunk: pairs whose k = 2 answer is empty by construction get
// n_paths = 0 in tok2; the others are listed (chunk-local k, list[0 .. *count), count
// zeroed by the caller) for the second SPF and the k = 2 trace. Also writes out_src[k] =
// the pair's source for every k (launch_gather_sources).
hipError_t launch_ksp_select_pairs(const DevGraph& g, const uint32_t* sources, const uint32_t* prow,
                                   const uint32_t* pdst, uint32_t first, uint32_t n, const uint32_t* tok1,
                                   uint32_t* tok2, uint32_t tok_cap, uint32_t* out_src, uint32_t* list,
                                   uint32_t* count, int num_cus, hipStream_t s);
uint32_t ksp_lds_bytes(uint32_t V, uint32_t L, uint32_t max_deg);

// Exact-order kernel (spf_exact.hip): LinkState::runSpf's heap process replayed per solve
// (one wavefront per solve) for graphs outside the fast kernels' domain — zero or
// wrapped-negative metrics, graphs too large for their LDS layouts, next-hop sets wider
// than 256. State in LDS when a slot fits (<= kMaxLds), else in `scratch` (slot bytes each).
// tight = the edges left in pathLinks; a.order (nullable) = pop index per node.
uint64_t exact_slot_bytes(uint32_t V, uint32_t E, uint32_t L, uint32_t nh_bits);
hipError_t launch_exact(const DevGraph& g, const SolveArgs& a, const uint64_t* w64, bool use_metric, uint32_t nh_bits,
                        uint8_t* scratch, uint64_t scratch_bytes, uint32_t* order_out, uint32_t* ctr, int num_cus,
                        hipStream_t s);

// LDS footprint of each kernel for a graph (0 if it cannot fit one workgroup per CU).
uint32_t bfs_lds_bytes(int family, uint32_t V, uint32_t L, bool has_ignore, int cls);
uint32_t bfs_code_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int cls);
uint32_t bfs_lvl_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int cls);

uint32_t fringe_lds_bytes(uint32_t V, uint32_t L, bool has_ignore, int nh_mode, bool dist64);
constexpr uint32_t kMaxLds = 160 * 1024;

// OPENR_SPF_PROF=1 (tuning only): the kernels' profiling counters (BFS level loops, the
// what-if repair phases, the KSP2 trace kinds) printed to stderr after each launch
inline bool prof_enabled() {
  const char* e = std::getenv("OPENR_SPF_PROF");
  return e && e[0] == '1';
}

}  // namespace openr_spf
