/* openr_routes.h — batched route build over a LinkState built from AdjacencyDatabases
 * (libopenr_decision.so; the graph handle comes from openr_adjdb_build_graph).
 *
 * Replaces, for a batch of nodes, SpfSolver::buildRouteDb(node, areaLinkStates,
 * prefixState) (openr/decision/Decision.cpp:568-734) followed, with
 * OPENR_ROUTES_UCMP, by RibPolicy::applyPolicy on the unicast routes (RibPolicy.cpp:
 * 181-199; Decision.cpp applies it on every rebuild). One all-sources SPF batch on the
 * GPU engine serves every node (SpfSolver::buildRouteDbs prefetch). Every node of the
 * graph originates one synthetic loopback prefix fd00::<node id hex>/128 (node id = the
 * name rank of openr_adjdb_build_graph), as the benchmark generators give every node a
 * prefix (RoutingBenchmarkUtils.cpp:85-101).
 *
 * Conventions as in openr_adjdb.h (0 / negative errno, openr_adjdb_last_error()).
 */
#ifndef OPENR_ROUTES_H
#define OPENR_ROUTES_H

#include <stdint.h>

#include "openr_adjdb.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OPENR_ROUTES_LFA = 1u << 0,  /* SpfSolver computeLfaPaths (per-neighbour SPFs, RFC 5286) */
  OPENR_ROUTES_V4 = 1u << 1,   /* SpfSolver enableV4 */
  OPENR_ROUTES_UCMP = 1u << 2, /* RibPolicy set_weight: default_weight, neighbor_weight[v] > 0 */
};

typedef struct {
  uint64_t unicast_routes;    /* sum over nodes of RibUnicastEntry count */
  uint64_t mpls_routes;       /* node / adjacency label routes */
  uint64_t nexthops;          /* NextHopThrift entries over every unicast route */
  uint64_t weighted_nexthops; /* of them, weight > 1 (UCMP) */
  uint64_t checksum;          /* order-independent hash of (node, prefix, nexthop addr, ifName,
                                 neighbour, metric, weight) */
  double ms_build;            /* SPF prefetch + route build (+ tally, free), host wall time less ms_policy */
  double ms_policy;           /* RibPolicy application: its thread time over the host workers
                                 (OPENR_HOST_THREADS) — its share of the wall time */
} openr_routes_stats_t;

/* Route DBs of node_ids[0..n) (graph node ids). neighbor_weight (nullable) [V] by graph
 * node id: the RibPolicy neighbour weight of that node as a next hop (<= 0: none). */
int openr_routes_build(openr_adjdb_graph* graph, const uint32_t* node_ids, uint32_t n, uint32_t flags,
                       int32_t default_weight, const int32_t* neighbor_weight, openr_routes_stats_t* out);

#ifdef __cplusplus
}
#endif
#endif /* OPENR_ROUTES_H */
