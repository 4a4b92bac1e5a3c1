/* openr_adjdb.h — C-ABI of the bulk AdjacencyDatabase input path (libopenr_decision.so).
 *
 * Replaces, for a batch of KvStore "adj:" values, the per-key
 *   fbzmq::util::readThriftObjStr<thrift::AdjacencyDatabase>(value, CompactSerializer)
 * of Decision::processPublication (openr/decision/Decision.cpp:1755-1757) and the
 * LinkState::updateAdjacencyDatabase calls that follow (:1773-1777, LinkState.cpp:564-719),
 * ending in the CSR mirror the SPF engine consumes (openr_spf_graph, openr_spf.h).
 *
 * Conventions as in openr_spf.h: extern "C", plain pointers and sizes, caller-owned
 * output buffers, 0 on success and a negative errno-style code on failure with a
 * thread-local message in openr_adjdb_last_error(). No exception crosses the boundary.
 * Host-only: nothing here touches a GPU.
 */
#ifndef OPENR_ADJDB_H
#define OPENR_ADJDB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OPENR_ADJDB_EINVAL (-22)  /* bad argument */
#define OPENR_ADJDB_EBADMSG (-74) /* malformed compact-protocol value */
#define OPENR_ADJDB_ENOSPC (-28)  /* caller buffer too small */
#define OPENR_ADJDB_EINTERNAL (-5)

typedef struct openr_adjdb_batch openr_adjdb_batch;
typedef struct openr_adjdb_graph openr_adjdb_graph;

const char* openr_adjdb_last_error(void);

/* Build id of libopenr_decision.so: "<sha256/16 of its sources> <source files>"
 * (Makefile build_id; checked against the tree by openr_amd/provenance.py). */
const char* openr_decision_build_id(void);

/* Decode n compact-protocol AdjacencyDatabase values. Value i is
 * data[offsets[i] .. offsets[i+1]) (offsets has n+1 entries). n_threads = 0 uses
 * every hardware thread. A malformed value fails the whole call (EBADMSG, message
 * names the value index), matching the reference, which drops the publication key. */
int openr_adjdb_decode(const uint8_t* data, const uint64_t* offsets, uint32_t n, uint32_t n_threads,
                       openr_adjdb_batch** out);
void openr_adjdb_free(openr_adjdb_batch* batch);

typedef struct {
  uint32_t n_dbs;
  uint64_t n_adjs;
  uint64_t n_strings;    /* 2 per database + 5 per adjacency (see columns) */
  uint64_t string_bytes; /* total bytes in the string pool */
  uint64_t n_perf_events;
} openr_adjdb_info_t;
int openr_adjdb_info(const openr_adjdb_batch* batch, openr_adjdb_info_t* out);

/* Columnar export (Lsdb.thrift:71-129 field meanings). String columns hold indices
 * into str_off; string k is str_pool[str_off[k] .. str_off[k+1]). Addresses are text
 * (inet_ntop of the 4/16-byte wire value). Every pointer must be non-null. */
typedef struct {
  char* str_pool;     /* [string_bytes] */
  uint64_t* str_off;  /* [n_strings + 1] */
  /* per database [n_dbs] */
  uint32_t* node_name;
  uint32_t* area;
  uint8_t* node_overloaded;
  int32_t* node_label;
  uint64_t* adj_begin; /* [n_dbs + 1] */
  /* per adjacency [n_adjs] */
  uint32_t* other_node;
  uint32_t* if_name;
  uint32_t* other_if_name;
  uint32_t* nh_v6;
  uint32_t* nh_v4;
  int32_t* metric;
  int32_t* adj_label;
  uint8_t* adj_overloaded;
  int32_t* rtt;
  int64_t* timestamp;
  int64_t* weight;
} openr_adjdb_columns;
int openr_adjdb_export(const openr_adjdb_batch* batch, const openr_adjdb_columns* cols);

/* Re-encode database `index` (writeThriftObjStr, LinkMonitor.cpp:620). *out_len gets the
 * encoded size; ENOSPC if cap is smaller (out may be null to query the size). */
int openr_adjdb_encode(const openr_adjdb_batch* batch, uint32_t index, uint8_t* out, uint64_t cap,
                       uint64_t* out_len);

/* Build a batch from columns (the inverse of openr_adjdb_export; str_pool/str_off as
 * there, adj_begin has n_dbs+1 entries). Used to originate values the way LinkMonitor
 * does before writeThriftObjStr (LinkMonitor.cpp:620). */
int openr_adjdb_batch_from_columns(const openr_adjdb_columns* cols, uint32_t n_dbs, openr_adjdb_batch** out);

/* Encode every database of the batch back to back: value i = data[offsets[i] ..
 * offsets[i+1]). *total gets the byte count; data may be null to query it. */
int openr_adjdb_encode_all(const openr_adjdb_batch* batch, uint8_t* data, uint64_t cap, uint64_t* offsets,
                           uint64_t* total);

/* Apply every decoded database, in order, to a fresh LinkState of `area` (each stamped
 * with the area, Decision.cpp:1762) and build its CSR mirror: node ids = rank of the
 * name under std::string operator<, row order = linksFromNode() iteration order. */
int openr_adjdb_build_graph(const openr_adjdb_batch* batch, const char* area, openr_adjdb_graph** out);
void openr_adjdb_graph_free(openr_adjdb_graph* graph);

typedef struct {
  uint32_t num_nodes;
  uint32_t num_dir_edges;
  uint32_t num_links;
  uint64_t name_bytes;
} openr_adjdb_graph_info_t;
int openr_adjdb_graph_info(const openr_adjdb_graph* graph, openr_adjdb_graph_info_t* out);

/* CSR arrays in the layout of openr_spf_graph (openr_spf.h). name_pool/name_off give
 * node names by id. Every pointer must be non-null. */
int openr_adjdb_graph_export(const openr_adjdb_graph* graph, uint32_t* row_ptr /* [V+1] */, uint32_t* col /* [E] */,
                             uint64_t* metric /* [E] */, uint32_t* link_id /* [E] */, uint8_t* edge_up /* [E] */,
                             uint8_t* node_overloaded /* [V] */, uint32_t* name_rank /* [V] */,
                             char* name_pool /* [name_bytes] */, uint64_t* name_off /* [V+1] */);

#ifdef __cplusplus
}
#endif

#endif /* OPENR_ADJDB_H */
