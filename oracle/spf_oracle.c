/*
 * spf_oracle.c — CPU ORACLE (test infrastructure; see spf_oracle.h header).
 *
 * Restates the reference algorithm step by step on dense integer ids:
 *   node name         -> node id, with std::string order given by name_rank
 *   linksFromNode(u)  -> CSR row u, in the caller-captured iteration order
 *   Link shared_ptr   -> undirected link id (link_id[e])
 *   nextHops (names)  -> bitset over the source's distinct neighbours
 *   pathLinks         -> ordered list of directed edge ids (prevNode = row owner)
 */
#include "spf_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define U64_MAX_ ((uint64_t)~(uint64_t)0)

/* ------------------------------------------------------------------------ */
/* DijkstraQ: min-heap keyed (metric, nodeName)  — LinkState.h:483-535       */
/* Any correct priority queue yields the same pop sequence because the key   */
/* (metric, name) is a strict total order; decrease-key replaces reMake().   */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t* heap;   /* node ids */
  int32_t* pos;     /* node -> heap slot, -1 if absent */
  uint32_t size;
  const uint64_t* key;   /* current tentative metric per node */
  const uint32_t* rank;  /* name rank per node */
} dq_t;

static int dq_less(const dq_t* q, uint32_t a, uint32_t b) {
  /* DijkstraQNodeGreater (LinkState.h:488-498) inverted: smaller metric first,
     then smaller name. */
  if (q->key[a] != q->key[b]) return q->key[a] < q->key[b];
  return q->rank[a] < q->rank[b];
}

static void dq_swap(dq_t* q, uint32_t i, uint32_t j) {
  uint32_t a = q->heap[i], b = q->heap[j];
  q->heap[i] = b;
  q->heap[j] = a;
  q->pos[b] = (int32_t)i;
  q->pos[a] = (int32_t)j;
}

static void dq_up(dq_t* q, uint32_t i) {
  while (i > 0) {
    uint32_t p = (i - 1) >> 1;
    if (!dq_less(q, q->heap[i], q->heap[p])) break;
    dq_swap(q, i, p);
    i = p;
  }
}

static void dq_down(dq_t* q, uint32_t i) {
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < q->size && dq_less(q, q->heap[l], q->heap[m])) m = l;
    if (r < q->size && dq_less(q, q->heap[r], q->heap[m])) m = r;
    if (m == i) break;
    dq_swap(q, i, m);
    i = m;
  }
}

static void dq_insert(dq_t* q, uint32_t v) {
  q->heap[q->size] = v;
  q->pos[v] = (int32_t)q->size;
  q->size++;
  dq_up(q, q->size - 1);
}

static int64_t dq_extract(dq_t* q) {
  if (q->size == 0) return -1;
  uint32_t v = q->heap[0];
  q->size--;
  if (q->size > 0) {
    q->heap[0] = q->heap[q->size];
    q->pos[q->heap[0]] = 0;
    dq_down(q, 0);
  }
  q->pos[v] = -1;
  return v;
}

/* ------------------------------------------------------------------------ */
/* Workspace                                                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t V, E, nw;    /* nw = u64 words per next-hop set */
  uint64_t* dist;       /* NodeSpfResult::metric_ */
  uint8_t* settled;     /* result.count(node) */
  uint64_t* nh;         /* [V][nw] NodeSpfResult::nextHops_ */
  int32_t* nbr_idx;     /* node -> distinct neighbour index of src, -1 */
  uint32_t** pl;        /* NodeSpfResult::pathLinks_ (edge ids) */
  uint32_t* pl_len;
  uint32_t* pl_cap;
  uint32_t* order;
  dq_t q;
  int unencodable;
} ws_t;

static void ws_free(ws_t* w) {
  if (!w) return;
  if (w->pl) {
    for (uint32_t i = 0; i < w->V; ++i) free(w->pl[i]);
  }
  free(w->pl);
  free(w->pl_len);
  free(w->pl_cap);
  free(w->dist);
  free(w->settled);
  free(w->nh);
  free(w->nbr_idx);
  free(w->order);
  free(w->q.heap);
  free(w->q.pos);
  memset(w, 0, sizeof(*w));
}

static int ws_init(ws_t* w, const oracle_graph* g) {
  memset(w, 0, sizeof(*w));
  w->V = g->num_nodes;
  w->E = g->num_dir_edges;
  uint32_t maxdeg = 0;
  for (uint32_t u = 0; u < w->V; ++u) {
    uint32_t d = g->row_ptr[u + 1] - g->row_ptr[u];
    if (d > maxdeg) maxdeg = d;
  }
  w->nw = (maxdeg + 63) / 64;
  if (w->nw == 0) w->nw = 1;
  size_t V = w->V ? w->V : 1;
  w->dist = (uint64_t*)malloc(V * sizeof(uint64_t));
  w->settled = (uint8_t*)malloc(V);
  w->nh = (uint64_t*)malloc(V * w->nw * sizeof(uint64_t));
  w->nbr_idx = (int32_t*)malloc(V * sizeof(int32_t));
  w->pl = (uint32_t**)calloc(V, sizeof(uint32_t*));
  w->pl_len = (uint32_t*)calloc(V, sizeof(uint32_t));
  w->pl_cap = (uint32_t*)calloc(V, sizeof(uint32_t));
  w->order = (uint32_t*)malloc(V * sizeof(uint32_t));
  w->q.heap = (uint32_t*)malloc(V * sizeof(uint32_t));
  w->q.pos = (int32_t*)malloc(V * sizeof(int32_t));
  if (!w->dist || !w->settled || !w->nh || !w->nbr_idx || !w->pl || !w->pl_len ||
      !w->pl_cap || !w->order || !w->q.heap || !w->q.pos) {
    ws_free(w);
    return -1;
  }
  for (uint32_t i = 0; i < w->V; ++i) w->nbr_idx[i] = -1;
  w->q.key = w->dist;
  w->q.rank = NULL;
  return 0;
}

static int pl_push(ws_t* w, uint32_t v, uint32_t e) {
  if (w->pl_len[v] == w->pl_cap[v]) {
    uint32_t nc = w->pl_cap[v] ? 2 * w->pl_cap[v] : 4;
    uint32_t* p = (uint32_t*)realloc(w->pl[v], nc * sizeof(uint32_t));
    if (!p) return -1;
    w->pl[v] = p;
    w->pl_cap[v] = nc;
  }
  w->pl[v][w->pl_len[v]++] = e;
  return 0;
}

static int ignored(const uint64_t* ign, uint32_t link) {
  return ign && ((ign[link >> 6] >> (link & 63)) & 1u);
}

/* LinkState::runSpf (LinkState.cpp:808-882). Returns #settled or -1. */
static int64_t run_spf_ws(ws_t* w, const oracle_graph* g, uint32_t src,
                          int use_link_metric, const uint64_t* ign) {
  const uint32_t V = w->V, nw = w->nw;
  if (src >= V) return -1;
  for (uint32_t i = 0; i < V; ++i) {
    w->dist[i] = U64_MAX_;
    w->settled[i] = 0;
    w->q.pos[i] = -1;
    w->pl_len[i] = 0;
  }
  memset(w->nh, 0, (size_t)V * nw * sizeof(uint64_t));
  w->q.size = 0;
  w->q.rank = g->name_rank;
  w->unencodable = 0;

  /* distinct neighbour numbering of src (next-hop bit encoding) */
  uint32_t nd = 0;
  for (uint32_t e = g->row_ptr[src]; e < g->row_ptr[src + 1]; ++e) {
    uint32_t v = g->col[e];
    if (w->nbr_idx[v] < 0) w->nbr_idx[v] = (int32_t)nd++;
  }

  /* q.insertNode(thisNodeName, 0) */
  w->dist[src] = 0;
  dq_insert(&w->q, src);
  uint32_t nsettled = 0;
  int64_t popped;
  while ((popped = dq_extract(&w->q)) >= 0) {
    uint32_t u = (uint32_t)popped;
    /* result.emplace(node) — record */
    w->settled[u] = 1;
    w->order[nsettled++] = u;
    const uint64_t du = w->dist[u];
    /* overloaded non-source nodes are sinks (LinkState.cpp:831-838) */
    if (g->node_overloaded[u] && u != src) continue;
    const uint64_t* nhu = w->nh + (size_t)u * nw;
    for (uint32_t e = g->row_ptr[u]; e < g->row_ptr[u + 1]; ++e) {
      uint32_t v = g->col[e];
      /* !link->isUp() or result.count(other) or linksToIgnore.count(link) */
      if (!g->edge_up[e] || w->settled[v] || ignored(ign, g->link_id[e])) continue;
      uint64_t m = use_link_metric ? g->metric[e] : 1u;
      uint64_t cand = du + m; /* u64 arithmetic, wraps like the reference */
      if (w->q.pos[v] < 0) {
        /* q.insertNode(otherNodeName, recordedNodeMetric + metric) */
        w->dist[v] = cand;
        w->pl_len[v] = 0;
        memset(w->nh + (size_t)v * nw, 0, nw * sizeof(uint64_t));
        dq_insert(&w->q, v);
      }
      if (w->dist[v] >= cand) {
        if (w->dist[v] > cand) {
          /* reset(newMetric) + reMake() */
          w->dist[v] = cand;
          w->pl_len[v] = 0;
          memset(w->nh + (size_t)v * nw, 0, nw * sizeof(uint64_t));
          dq_up(&w->q, (uint32_t)w->q.pos[v]);
        }
        /* addPath(link, recordedNodeName) */
        if (pl_push(w, v, e)) return -1;
        /* addNextHops(recordedNodeNextHops) */
        uint64_t* nhv = w->nh + (size_t)v * nw;
        int empty = 1;
        for (uint32_t k = 0; k < nw; ++k) {
          nhv[k] |= nhu[k];
          empty &= (nhv[k] == 0);
        }
        if (empty) {
          /* directly connected node: addNextHop(otherNodeName) */
          int32_t idx = w->nbr_idx[v];
          if (idx < 0) {
            w->unencodable = 1; /* only reachable through u64 wrap-around */
          } else {
            nhv[idx >> 6] |= (uint64_t)1 << (idx & 63);
          }
        }
      }
    }
  }
  /* restore neighbour map for the next call */
  for (uint32_t e = g->row_ptr[src]; e < g->row_ptr[src + 1]; ++e) w->nbr_idx[g->col[e]] = -1;
  return nsettled;
}

static void write_nh(const ws_t* w, uint8_t* out, uint32_t nh_bytes) {
  for (uint32_t v = 0; v < w->V; ++v) {
    uint8_t* o = out + (size_t)v * nh_bytes;
    const uint64_t* s = w->nh + (size_t)v * w->nw;
    for (uint32_t b = 0; b < nh_bytes; ++b) {
      uint32_t word = b >> 3;
      o[b] = (word < w->nw) ? (uint8_t)(s[word] >> (8 * (b & 7))) : 0;
    }
  }
}

uint32_t oracle_num_distinct_neighbors(const oracle_graph* g, uint32_t src) {
  uint32_t n = 0;
  for (uint32_t e = g->row_ptr[src]; e < g->row_ptr[src + 1]; ++e) {
    int seen = 0;
    for (uint32_t f = g->row_ptr[src]; f < e; ++f) {
      if (g->col[f] == g->col[e]) {
        seen = 1;
        break;
      }
    }
    n += !seen;
  }
  return n;
}

int64_t oracle_run_spf(const oracle_graph* g, uint32_t src, int use_link_metric,
                       const uint64_t* ignore_links, uint64_t* out_dist,
                       uint8_t* out_nh, uint32_t nh_bytes, uint32_t* out_order,
                       uint32_t* out_pl_ptr, uint32_t* out_pl_edge) {
  ws_t w;
  if (!g || src >= g->num_nodes) return -1;
  if (ws_init(&w, g)) return -1;
  int64_t n = run_spf_ws(&w, g, src, use_link_metric, ignore_links);
  if (n >= 0 && w.unencodable) n = -2;
  if (n >= 0) {
    if (out_dist) {
      /* nodes absent from SpfResult report UINT64_MAX */
      for (uint32_t v = 0; v < w.V; ++v) out_dist[v] = w.settled[v] ? w.dist[v] : U64_MAX_;
    }
    if (out_nh) write_nh(&w, out_nh, nh_bytes);
    if (out_order) memcpy(out_order, w.order, (size_t)n * sizeof(uint32_t));
    if (out_pl_ptr) {
      uint32_t off = 0;
      for (uint32_t v = 0; v < w.V; ++v) {
        out_pl_ptr[v] = off;
        if (w.settled[v]) {
          if (out_pl_edge) memcpy(out_pl_edge + off, w.pl[v], w.pl_len[v] * sizeof(uint32_t));
          off += w.pl_len[v];
        }
      }
      out_pl_ptr[w.V] = off;
    }
  }
  ws_free(&w);
  return n;
}

/* ------------------------------------------------------------------------ */
/* traceOnePath (LinkState.cpp:398-419) as an explicit-stack DFS             */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t node;
  uint32_t it;     /* next pathLinks index to try */
  uint32_t taken;  /* edge taken towards the next frame */
} frame_t;

/* Returns path length (>=0) written into path[] in src->dest order, or -1
   when no path (std::nullopt). visited = bitmask over link ids. */
static int64_t trace_one_path(const ws_t* w, const oracle_graph* g,
                              const uint32_t* owner, uint32_t src, uint32_t dest,
                              uint64_t* visited, frame_t* stack, uint32_t* path) {
  if (src == dest) return 0; /* LinkState::Path{} */
  uint32_t sp = 0;
  stack[sp].node = dest;
  stack[sp].it = 0;
  sp = 1;
  while (sp > 0) {
    frame_t* f = &stack[sp - 1];
    if (f->node == src) {
      /* success: frames [dest, p1, ..., src]; taken links from dest upward */
      uint32_t len = sp - 1;
      for (uint32_t i = 0; i < len; ++i) path[len - 1 - i] = stack[i].taken;
      return len;
    }
    int pushed = 0;
    while (f->it < w->pl_len[f->node]) {
      uint32_t e = w->pl[f->node][f->it++];
      uint32_t link = g->link_id[e];
      /* linksToIgnore.insert(pathLink.link).second */
      if (!((visited[link >> 6] >> (link & 63)) & 1u)) {
        visited[link >> 6] |= (uint64_t)1 << (link & 63);
        f->taken = e;
        stack[sp].node = owner[e]; /* pathLink.prevNode */
        stack[sp].it = 0;
        sp++;
        pushed = 1;
        break;
      }
    }
    if (!pushed) sp--; /* exhausted: std::nullopt to the caller frame */
  }
  return -1;
}

/* Per-thread buffers of getKthPaths (allocated once, reused across pairs). */
typedef struct {
  ws_t w;
  size_t lw;
  uint64_t* ignore;
  uint64_t* visited;
  uint32_t* owner;
  frame_t* stack;
  uint32_t* path;
  uint32_t* cur_ptr;   /* paths of the current level */
  uint32_t* cur_edges;
} ksp_ctx;

static void ksp_free(ksp_ctx* c) {
  free(c->ignore);
  free(c->visited);
  free(c->owner);
  free(c->stack);
  free(c->path);
  free(c->cur_ptr);
  free(c->cur_edges);
  ws_free(&c->w);
  memset(c, 0, sizeof(*c));
}

static int ksp_init(ksp_ctx* c, const oracle_graph* g) {
  memset(c, 0, sizeof(*c));
  if (ws_init(&c->w, g)) return -1;
  const uint32_t L = g->num_links, V = g->num_nodes, E = g->num_dir_edges;
  c->lw = (L + 63) / 64 + 1;
  c->ignore = (uint64_t*)calloc(c->lw, sizeof(uint64_t));
  c->visited = (uint64_t*)calloc(c->lw, sizeof(uint64_t));
  c->owner = (uint32_t*)malloc((E ? E : 1) * sizeof(uint32_t));
  c->stack = (frame_t*)malloc(((size_t)V + 1) * sizeof(frame_t));
  c->path = (uint32_t*)malloc(((size_t)V + 1) * sizeof(uint32_t));
  c->cur_ptr = (uint32_t*)malloc(((size_t)E + 2) * sizeof(uint32_t));
  c->cur_edges = (uint32_t*)malloc(((size_t)E * 2 + (size_t)V + 1) * sizeof(uint32_t));
  if (!c->ignore || !c->visited || !c->owner || !c->stack || !c->path || !c->cur_ptr || !c->cur_edges) {
    ksp_free(c);
    return -1;
  }
  for (uint32_t u = 0; u < V; ++u)
    for (uint32_t e = g->row_ptr[u]; e < g->row_ptr[u + 1]; ++e) c->owner[e] = u;
  return 0;
}

/* getKthPaths (LinkState.cpp:762-791): level i < k ignores the links of every path
   found at levels < i; the paths of level k are left in cur_ptr / cur_edges.
   Returns the number of paths or -1. */
static int64_t kth_paths_ctx(ksp_ctx* c, const oracle_graph* g, uint32_t src, uint32_t dest, uint32_t k) {
  memset(c->ignore, 0, c->lw * sizeof(uint64_t));
  uint32_t npaths = 0;
  for (uint32_t level = 1; level <= k; ++level) {
    int any_ignore = 0;
    for (size_t i = 0; i < c->lw; ++i) any_ignore |= (c->ignore[i] != 0);
    /* linksToIgnore.empty() ? getSpfResult(src, true) : runSpf(src, true, ignore) */
    if (run_spf_ws(&c->w, g, src, 1, any_ignore ? c->ignore : NULL) < 0) return -1;
    npaths = 0;
    c->cur_ptr[0] = 0;
    if (c->w.settled[dest]) {
      memset(c->visited, 0, c->lw * sizeof(uint64_t));
      for (;;) {
        int64_t len = trace_one_path(&c->w, g, c->owner, src, dest, c->visited, c->stack, c->path);
        if (len <= 0) break; /* while (path && !path->empty()) */
        memcpy(c->cur_edges + c->cur_ptr[npaths], c->path, (size_t)len * sizeof(uint32_t));
        c->cur_ptr[npaths + 1] = c->cur_ptr[npaths] + (uint32_t)len;
        npaths++;
      }
    }
    if (level < k) {
      for (uint32_t i = 0; i < c->cur_ptr[npaths]; ++i) {
        uint32_t link = g->link_id[c->cur_edges[i]];
        c->ignore[link >> 6] |= (uint64_t)1 << (link & 63);
      }
    }
  }
  return npaths;
}

int64_t oracle_kth_paths(const oracle_graph* g, uint32_t src, uint32_t dest,
                         uint32_t k, uint32_t* out_path_ptr, uint32_t max_paths,
                         uint32_t* out_edges, uint32_t max_edges) {
  if (!g || k < 1 || src >= g->num_nodes || dest >= g->num_nodes) return -1;
  ksp_ctx c;
  if (ksp_init(&c, g)) return -1;
  int64_t npaths = kth_paths_ctx(&c, g, src, dest, k);
  int64_t result = -1;
  if (npaths >= 0 && (uint64_t)npaths <= max_paths && c.cur_ptr[npaths] <= max_edges) {
    if (out_path_ptr) memcpy(out_path_ptr, c.cur_ptr, ((size_t)npaths + 1) * sizeof(uint32_t));
    if (out_edges) memcpy(out_edges, c.cur_edges, (size_t)c.cur_ptr[npaths] * sizeof(uint32_t));
    result = npaths;
  }
  ksp_free(&c);
  return result;
}

/* Token row [n_paths, len_0, e.., len_1, e.., ...] (openr_spf_ksp2 layout); a row that
   does not fit gets n_paths = 0xFFFFFFFF. */
static void write_tokens(const ksp_ctx* c, uint32_t npaths, uint32_t* tok, uint32_t cap) {
  if (1u + npaths + c->cur_ptr[npaths] > cap) {
    tok[0] = 0xFFFFFFFFu;
    return;
  }
  uint32_t pos = 0;
  tok[pos++] = npaths;
  for (uint32_t i = 0; i < npaths; ++i) {
    const uint32_t len = c->cur_ptr[i + 1] - c->cur_ptr[i];
    tok[pos++] = len;
    memcpy(tok + pos, c->cur_edges + c->cur_ptr[i], (size_t)len * sizeof(uint32_t));
    pos += len;
  }
}

typedef struct {
  const oracle_graph* g;
  const uint32_t *src, *dst;
  uint32_t n, tid, nthreads, tok_cap;
  uint32_t *tok1, *tok2;
  int rc;
} ksp_job_t;

static void* ksp_worker(void* arg) {
  ksp_job_t* j = (ksp_job_t*)arg;
  ksp_ctx c;
  if (ksp_init(&c, j->g)) {
    j->rc = -1;
    return NULL;
  }
  for (uint32_t i = j->tid; i < j->n; i += j->nthreads) {
    for (uint32_t k = 1; k <= 2; ++k) {
      int64_t np = kth_paths_ctx(&c, j->g, j->src[i], j->dst[i], k);
      if (np < 0) {
        j->rc = -1;
        break;
      }
      write_tokens(&c, (uint32_t)np, (k == 1 ? j->tok1 : j->tok2) + (size_t)i * j->tok_cap, j->tok_cap);
    }
  }
  ksp_free(&c);
  return NULL;
}

int oracle_ksp2_batch(const oracle_graph* g, const uint32_t* src, const uint32_t* dst, uint32_t n,
                      uint32_t tok_cap, uint32_t* tok1, uint32_t* tok2, int nthreads) {
  if (!g || tok_cap < 1 || (n && (!src || !dst || !tok1 || !tok2))) return -1;
  for (uint32_t i = 0; i < n; ++i)
    if (src[i] >= g->num_nodes || dst[i] >= g->num_nodes) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ksp_job_t jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (ksp_job_t){g, src, dst, n, (uint32_t)t, (uint32_t)nthreads, tok_cap, tok1, tok2, 0};
    if (t > 0) pthread_create(&th[t], NULL, ksp_worker, &jobs[t]);
  }
  ksp_worker(&jobs[0]);
  int rc = jobs[0].rc;
  for (int t = 1; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Per-link-failure what-if counts: runSpf(src, use, {link}) vs runSpf(src)  */
/* ------------------------------------------------------------------------ */
typedef struct {
  const oracle_graph* g;
  const uint32_t *links, *sources;
  uint32_t n_links, n_sources, tid, nthreads;
  int use_link_metric;
  uint32_t* changed;
  int rc;
  uint64_t* digest;   /* nullable: per-unit delta digest (oracle_whatif_delta_digest) */
  uint32_t nh_bytes;
} whatif_job_t;

/* splitmix64 finaliser (Steele et al.): the mixing step of the delta digest */
static uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* hash of one delta entry: node, new distance, new next-hop bytes in 8-byte chunks
   (little-endian, zero past nh_bytes) -- the layout openr_spf_whatif_delta writes */
static uint64_t delta_entry_hash(uint32_t v, uint64_t d, const uint64_t* nh, uint32_t nw, uint32_t nh_bytes) {
  uint64_t h = mix64((uint64_t)v ^ 0xD1B54A32D192ED03ull);
  h = mix64(h ^ d);
  for (uint32_t k = 0; k < (nh_bytes + 7) / 8; ++k) {
    uint64_t c = k < nw ? nh[k] : 0;
    const uint32_t bytes = nh_bytes - 8 * k;
    if (bytes < 8) c &= (((uint64_t)1) << (8 * bytes)) - 1;
    h = mix64(h ^ c);
  }
  return h;
}

static void* whatif_worker(void* arg) {
  whatif_job_t* j = (whatif_job_t*)arg;
  const oracle_graph* g = j->g;
  ws_t w;
  if (ws_init(&w, g)) {
    j->rc = -1;
    return NULL;
  }
  const uint32_t V = g->num_nodes, nw = w.nw;
  const size_t lw = (g->num_links + 63) / 64 + 1;
  uint64_t* base_d = (uint64_t*)malloc((size_t)(V ? V : 1) * sizeof(uint64_t));
  uint64_t* base_nh = (uint64_t*)malloc((size_t)(V ? V : 1) * nw * sizeof(uint64_t));
  uint64_t* ign = (uint64_t*)calloc(lw, sizeof(uint64_t));
  if (!base_d || !base_nh || !ign) j->rc = -1;
  for (uint32_t s = j->tid; s < j->n_sources && !j->rc; s += j->nthreads) {
    const uint32_t src = j->sources[s];
    if (run_spf_ws(&w, g, src, j->use_link_metric, NULL) < 0) {
      j->rc = -1;
      break;
    }
    for (uint32_t v = 0; v < V; ++v) base_d[v] = w.settled[v] ? w.dist[v] : U64_MAX_;
    memcpy(base_nh, w.nh, (size_t)V * nw * sizeof(uint64_t));
    for (uint32_t i = 0; i < j->n_links; ++i) {
      const uint32_t l = j->links[i];
      ign[l >> 6] |= (uint64_t)1 << (l & 63);
      if (run_spf_ws(&w, g, src, j->use_link_metric, ign) < 0) j->rc = -1;
      ign[l >> 6] = 0;
      uint32_t cnt = 0;
      uint64_t dig = 0;
      for (uint32_t v = 0; v < V; ++v) {
        const uint64_t d = w.settled[v] ? w.dist[v] : U64_MAX_;
        int diff = d != base_d[v];
        for (uint32_t k = 0; k < nw && !diff; ++k) diff = w.nh[(size_t)v * nw + k] != base_nh[(size_t)v * nw + k];
        cnt += (uint32_t)diff;
        if (diff && j->digest) dig += delta_entry_hash(v, d, w.nh + (size_t)v * nw, nw, j->nh_bytes);
      }
      j->changed[(size_t)i * j->n_sources + s] = cnt;
      if (j->digest) j->digest[(size_t)i * j->n_sources + s] = dig;
    }
  }
  free(base_d);
  free(base_nh);
  free(ign);
  ws_free(&w);
  return NULL;
}

static int whatif_run(const oracle_graph* g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                      uint32_t n_sources, int use_link_metric, uint32_t* changed, uint64_t* digest,
                      uint32_t nh_bytes, int nthreads) {
  if (!g) return -1;
  for (uint32_t i = 0; i < n_links; ++i)
    if (links[i] >= g->num_links) return -1;
  for (uint32_t i = 0; i < n_sources; ++i)
    if (sources[i] >= g->num_nodes) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  whatif_job_t jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (whatif_job_t){g, links, sources, n_links, n_sources, (uint32_t)t, (uint32_t)nthreads,
                             use_link_metric, changed, 0, digest, nh_bytes};
    if (t > 0) pthread_create(&th[t], NULL, whatif_worker, &jobs[t]);
  }
  whatif_worker(&jobs[0]);
  int rc = jobs[0].rc;
  for (int t = 1; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  return rc;
}

int oracle_whatif(const oracle_graph* g, const uint32_t* links, uint32_t n_links, const uint32_t* sources,
                  uint32_t n_sources, int use_link_metric, uint32_t* changed, int nthreads) {
  return whatif_run(g, links, n_links, sources, n_sources, use_link_metric, changed, NULL, 0, nthreads);
}

int oracle_whatif_delta_digest(const oracle_graph* g, const uint32_t* links, uint32_t n_links,
                               const uint32_t* sources, uint32_t n_sources, int use_link_metric,
                               uint32_t* changed, uint64_t* digest, uint32_t nh_bytes, int nthreads) {
  if (!digest) return -1;
  return whatif_run(g, links, n_links, sources, n_sources, use_link_metric, changed, digest, nh_bytes, nthreads);
}

/* ------------------------------------------------------------------------ */
/* Multi-threaded all-sources driver (CPU baseline)                          */
/* ------------------------------------------------------------------------ */
typedef struct {
  const oracle_graph* g;
  const uint32_t* sources;
  uint32_t n, tid, nthreads;
  int use_link_metric;
  uint64_t* dist;
  uint8_t* nh;
  uint32_t nh_bytes;
  int rc;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  ws_t w;
  if (ws_init(&w, j->g)) {
    j->rc = -1;
    return NULL;
  }
  const uint32_t V = j->g->num_nodes;
  for (uint32_t i = j->tid; i < j->n; i += j->nthreads) {
    if (run_spf_ws(&w, j->g, j->sources[i], j->use_link_metric, NULL) < 0) {
      j->rc = -1;
      break;
    }
    if (j->dist) {
      uint64_t* d = j->dist + (size_t)i * V;
      for (uint32_t v = 0; v < V; ++v) d[v] = w.settled[v] ? w.dist[v] : U64_MAX_;
    }
    if (j->nh) write_nh(&w, j->nh + (size_t)i * V * j->nh_bytes, j->nh_bytes);
  }
  ws_free(&w);
  return NULL;
}

int oracle_all_sources(const oracle_graph* g, const uint32_t* sources, uint32_t n,
                       int use_link_metric, uint64_t* dist, uint8_t* nh,
                       uint32_t nh_bytes, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (job_t){g, sources, n, (uint32_t)t, (uint32_t)nthreads, use_link_metric,
                      dist, nh, nh_bytes, 0};
    if (t > 0) pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  worker(&jobs[0]);
  int rc = jobs[0].rc;
  for (int t = 1; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  return rc;
}
