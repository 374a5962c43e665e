/*
 * keto_oracle.c -- CPU restatement of Ory Keto's check / expand semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU
 * baseline ("port") for the MI355X engine in keto_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU reference -- never as a product path.
 *
 * It follows the reference Go engine (paths relative to /root/reference):
 *   internal/check/engine.go:54-80    CheckIsMember / CheckRelationTuple, depth clamp
 *   internal/check/engine.go:183-207  checkIsAllowed: group[direct(d-1), expand(d), rewrite|err]
 *   internal/check/engine.go:148-177  checkDirect: exact tuple exists -> IsMember
 *   internal/check/engine.go:87-145   checkExpandSubject: rows in shard order, pages of 100,
 *                                     mark-visited-then-skip, "..." and SubjectIDs skipped
 *   internal/check/engine.go:209-229  astRelationFor: unknown ns / no relations -> no rewrite,
 *                                     undeclared relation -> error "relation not found"
 *   internal/check/rewrites.go:30-260 rewrite / inverted / computed (same depth) / TTU (d-1)
 *   internal/check/binop.go:15-70     or / and
 *   internal/check/checkgroup/concurrent_checkgroup.go:104-120  first Err|IsMember wins, else NotMember
 *   internal/x/graph/graph_utils.go:35-50  visited set scoping (created by the first expand)
 *   internal/expand/engine.go:35-104  BuildTree
 *   internal/persistence/sql/relationtuples.go:203-244  rows = filter + shard_id order
 *
 * Two evaluation policies are provided (SURVEY.md section 8a "order-sensitivity contract"):
 *   KO_POLICY_CANONICAL  -- the schedule-free semantics: the checkIsAllowed recursion evaluated
 *                           without visited pruning, memoised on (node, depth).  On rewrite-free
 *                           graphs this equals "BFS-first-mark" bounded reachability.
 *   KO_POLICY_DFS        -- one concrete Go schedule: fully sequential DFS in Add order, sharing
 *                           the reference's visited sets and its page-tail marking.
 * A query is schedule-invariant when both agree; parity is bit-exact on those.
 *
 * Data model: every string/UUID is pre-interned by the caller into dense u32 ids (namespaces,
 * relations, objects/subject-ids share one UUID space exactly as in the reference).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KO_SUBJECT_ID 0xFFFFFFFFu
#define SET_BIT 0x80000000u
#define NONE 0xFFFFFFFFu
#define LOOKUP 0xFFFFFFFEu

enum { KO_N = 0, KO_M = 1, KO_ERR = 2, KO_U = 3 };
enum { KO_POLICY_CANONICAL = 0, KO_POLICY_DFS = 1 };
enum { RW_OR = 0, RW_AND = 1, RW_COMPUTED = 2, RW_TTU = 3, RW_NOT = 4 };
enum { KO_ERR_NONE = 0, KO_ERR_RELATION_NOT_FOUND = 1, KO_ERR_NOT_IMPLEMENTED = 2, KO_ERR_REWRITE_CYCLE = 3 };

typedef struct { uint32_t ns, obj, rel, sns, sobj, srel; } ko_tuple;
typedef struct { int32_t kind, rel, crel, first, count; } ko_rw;

/* ---------------------------------------------------------------- hash map: (u64,u64) -> u32 */
typedef struct { uint64_t a, b; uint32_t v, used; } slot_t;
typedef struct { slot_t* s; uint64_t cap, n; } tmap;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL; x ^= x >> 27; x *= 0x94d049bb133111ebULL; x ^= x >> 31;
  return x;
}
static uint64_t hkey(uint64_t a, uint64_t b) { return mix64(a * 0x9E3779B97F4A7C15ULL ^ mix64(b)); }

static void tmap_init(tmap* m, uint64_t cap) {
  uint64_t c = 16; while (c < cap * 2) c <<= 1;
  m->s = (slot_t*)calloc(c, sizeof(slot_t)); m->cap = c; m->n = 0;
}
static void tmap_free(tmap* m) { free(m->s); m->s = NULL; m->cap = m->n = 0; }
static slot_t* tmap_find_slot(slot_t* s, uint64_t cap, uint64_t a, uint64_t b) {
  uint64_t i = hkey(a, b) & (cap - 1);
  for (;;) {
    if (!s[i].used || (s[i].a == a && s[i].b == b)) return &s[i];
    i = (i + 1) & (cap - 1);
  }
}
static void tmap_grow(tmap* m) {
  uint64_t nc = m->cap * 2; slot_t* ns = (slot_t*)calloc(nc, sizeof(slot_t));
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->s[i].used) *tmap_find_slot(ns, nc, m->s[i].a, m->s[i].b) = m->s[i];
  free(m->s); m->s = ns; m->cap = nc;
}
/* returns pointer to value; *found tells whether it existed. */
static uint32_t* tmap_put(tmap* m, uint64_t a, uint64_t b, int* found) {
  if ((m->n + 1) * 2 > m->cap) tmap_grow(m);
  slot_t* sl = tmap_find_slot(m->s, m->cap, a, b);
  if (sl->used) { *found = 1; return &sl->v; }
  sl->used = 1; sl->a = a; sl->b = b; sl->v = 0; m->n++; *found = 0; return &sl->v;
}
static const uint32_t* tmap_get(const tmap* m, uint64_t a, uint64_t b) {
  if (!m->cap) return NULL;
  slot_t* sl = tmap_find_slot(m->s, m->cap, a, b);
  return sl->used ? &sl->v : NULL;
}

/* ---------------------------------------------------------------- index */
typedef struct {
  uint32_t wildcard_rel, page_size;
  /* tuples as given (shard order) */
  ko_tuple* tup; uint64_t n_tup, cap_tup;
  /* nodes: (ns,obj,rel) triples; node id = index */
  uint32_t *nd_ns, *nd_obj, *nd_rel; uint32_t n_nodes, cap_nodes;
  tmap node_map;
  /* CSR rows in shard order and per-row sorted copy for exact-tuple lookups */
  uint64_t* row_off; uint32_t* row_subj; uint32_t* row_sorted;
  int finalized;
  /* program */
  uint32_t n_ns; uint8_t* ns_has_rel;
  tmap rel_map;        /* (ns, rel) -> rewrite root + 1 (0 = declared without rewrite) */
  ko_rw* rw; uint32_t n_rw; int32_t* child; uint32_t n_child;
} ko_index;

static uint32_t node_intern(ko_index* ix, uint32_t ns, uint32_t obj, uint32_t rel) {
  int found;
  uint32_t* v = tmap_put(&ix->node_map, ((uint64_t)ns << 32) | rel, obj, &found);
  if (found) return *v;
  if (ix->n_nodes == ix->cap_nodes) {
    ix->cap_nodes = ix->cap_nodes ? ix->cap_nodes * 2 : 1024;
    ix->nd_ns = (uint32_t*)realloc(ix->nd_ns, ix->cap_nodes * 4);
    ix->nd_obj = (uint32_t*)realloc(ix->nd_obj, ix->cap_nodes * 4);
    ix->nd_rel = (uint32_t*)realloc(ix->nd_rel, ix->cap_nodes * 4);
  }
  uint32_t id = ix->n_nodes++;
  ix->nd_ns[id] = ns; ix->nd_obj[id] = obj; ix->nd_rel[id] = rel;
  *v = id;
  return id;
}
static uint32_t node_find(const ko_index* ix, uint32_t ns, uint32_t obj, uint32_t rel) {
  const uint32_t* v = tmap_get(&ix->node_map, ((uint64_t)ns << 32) | rel, obj);
  return v ? *v : NONE;
}

ko_index* ko_index_new(uint32_t wildcard_rel, uint32_t page_size) {
  ko_index* ix = (ko_index*)calloc(1, sizeof(ko_index));
  ix->wildcard_rel = wildcard_rel;
  ix->page_size = page_size ? page_size : 100; /* persister.go:38 defaultPageSize */
  tmap_init(&ix->node_map, 1024);
  tmap_init(&ix->rel_map, 64);
  return ix;
}

void ko_index_free(ko_index* ix) {
  if (!ix) return;
  free(ix->tup); free(ix->nd_ns); free(ix->nd_obj); free(ix->nd_rel);
  tmap_free(&ix->node_map); tmap_free(&ix->rel_map);
  free(ix->row_off); free(ix->row_subj); free(ix->row_sorted);
  free(ix->ns_has_rel); free(ix->rw); free(ix->child);
  free(ix);
}

int ko_index_add_tuples(ko_index* ix, const ko_tuple* t, uint64_t n) {
  if (ix->finalized) return -1;
  if (ix->n_tup + n > ix->cap_tup) {
    uint64_t c = ix->cap_tup ? ix->cap_tup : 1024;
    while (c < ix->n_tup + n) c *= 2;
    ix->tup = (ko_tuple*)realloc(ix->tup, c * sizeof(ko_tuple)); ix->cap_tup = c;
  }
  memcpy(ix->tup + ix->n_tup, t, n * sizeof(ko_tuple)); ix->n_tup += n;
  return 0;
}

static int cmp_u32(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b; return x < y ? -1 : x > y;
}

typedef struct { ko_index* ix; uint32_t v0, v1; } sort_arg;
static void* sort_worker(void* p) {
  sort_arg* a = (sort_arg*)p;
  ko_index* ix = a->ix;
  uint64_t b0 = ix->row_off[a->v0], e0 = ix->row_off[a->v1];
  memcpy(ix->row_sorted + b0, ix->row_subj + b0, (e0 - b0) * 4);
  for (uint32_t v = a->v0; v < a->v1; v++) {
    uint64_t b = ix->row_off[v], e = ix->row_off[v + 1];
    if (e - b > 1) qsort(ix->row_sorted + b, e - b, 4, cmp_u32);
  }
  return NULL;
}
static void build_sorted(ko_index* ix, int nthreads) {
  ix->row_sorted = (uint32_t*)malloc((ix->row_off[ix->n_nodes] + 1) * 4);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pthread_t th[64]; sort_arg args[64];
  for (int t = 0; t < nthreads; t++) {
    args[t].ix = ix;
    args[t].v0 = (uint32_t)((uint64_t)ix->n_nodes * t / nthreads);
    args[t].v1 = (uint32_t)((uint64_t)ix->n_nodes * (t + 1) / nthreads);
    pthread_create(&th[t], NULL, sort_worker, &args[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* Interns all triples, then lays rows out per node keeping tuple (shard) order. */
int ko_index_finalize(ko_index* ix) {
  if (ix->finalized) return -1;
  uint32_t* lhs = (uint32_t*)malloc((ix->n_tup + 1) * 4);
  uint32_t* sub = (uint32_t*)malloc((ix->n_tup + 1) * 4);
  for (uint64_t i = 0; i < ix->n_tup; i++) {
    const ko_tuple* t = &ix->tup[i];
    lhs[i] = node_intern(ix, t->ns, t->obj, t->rel);
    if (t->sns == KO_SUBJECT_ID) sub[i] = t->sobj & ~SET_BIT;
    else sub[i] = SET_BIT | node_intern(ix, t->sns, t->sobj, t->srel);
  }
  ix->row_off = (uint64_t*)calloc((uint64_t)ix->n_nodes + 1, 8);
  for (uint64_t i = 0; i < ix->n_tup; i++) ix->row_off[lhs[i] + 1]++;
  for (uint32_t v = 0; v < ix->n_nodes; v++) ix->row_off[v + 1] += ix->row_off[v];
  uint64_t* fill = (uint64_t*)malloc(((uint64_t)ix->n_nodes + 1) * 8);
  memcpy(fill, ix->row_off, ((uint64_t)ix->n_nodes + 1) * 8);
  ix->row_subj = (uint32_t*)malloc((ix->n_tup + 1) * 4);
  for (uint64_t i = 0; i < ix->n_tup; i++) ix->row_subj[fill[lhs[i]]++] = sub[i];
  free(fill); free(lhs); free(sub);
  build_sorted(ix, 1);
  ix->finalized = 1;
  return 0;
}

/* Import an already laid-out row index (used by bench.py's CPU baseline on the big synthetic
 * graph): node triples, CSR offsets and tagged subjects in shard order. */
ko_index* ko_index_from_csr(uint32_t wildcard_rel, uint32_t n_nodes, const uint32_t* nd_ns,
                            const uint32_t* nd_obj, const uint32_t* nd_rel, const uint64_t* row_off,
                            const uint32_t* row_subj, int with_node_map, int nthreads) {
  ko_index* ix = ko_index_new(wildcard_rel, 100);
  ix->cap_nodes = n_nodes ? n_nodes : 1;
  ix->nd_ns = (uint32_t*)malloc(ix->cap_nodes * 4);
  ix->nd_obj = (uint32_t*)malloc(ix->cap_nodes * 4);
  ix->nd_rel = (uint32_t*)malloc(ix->cap_nodes * 4);
  if (with_node_map) {
    tmap_free(&ix->node_map);
    tmap_init(&ix->node_map, n_nodes);
    for (uint32_t v = 0; v < n_nodes; v++) node_intern(ix, nd_ns[v], nd_obj[v], nd_rel[v]);
  } else { /* node ids given directly (rewrite-free node-level queries only) */
    memcpy(ix->nd_ns, nd_ns, (size_t)n_nodes * 4); memcpy(ix->nd_obj, nd_obj, (size_t)n_nodes * 4);
    memcpy(ix->nd_rel, nd_rel, (size_t)n_nodes * 4); ix->n_nodes = n_nodes;
  }
  ix->row_off = (uint64_t*)malloc(((uint64_t)n_nodes + 1) * 8);
  memcpy(ix->row_off, row_off, ((uint64_t)n_nodes + 1) * 8);
  uint64_t ne = row_off[n_nodes];
  ix->row_subj = (uint32_t*)malloc((ne + 1) * 4);
  memcpy(ix->row_subj, row_subj, ne * 4);
  build_sorted(ix, nthreads);
  ix->finalized = 1;
  return ix;
}

uint32_t ko_index_n_nodes(const ko_index* ix) { return ix->n_nodes; }
uint64_t ko_index_n_rows(const ko_index* ix) { return ix->finalized ? ix->row_off[ix->n_nodes] : 0; }

/* Namespace program: ns_has_rel[ns] = namespace configured with >=1 relation
 * (engine.go:219-221); rel entries (ns, rel, root) declare relations, root = -1 for none. */
int ko_set_program(ko_index* ix, uint32_t n_ns, const uint8_t* ns_has_rel, uint32_t n_rel,
                   const uint32_t* rel_ns, const uint32_t* rel_rel, const int32_t* rel_root,
                   uint32_t n_rw, const int32_t* rw5, uint32_t n_child, const int32_t* child) {
  free(ix->ns_has_rel); free(ix->rw); free(ix->child);
  tmap_free(&ix->rel_map); tmap_init(&ix->rel_map, n_rel + 8);
  ix->n_ns = n_ns;
  ix->ns_has_rel = (uint8_t*)calloc(n_ns + 1, 1);
  if (n_ns) memcpy(ix->ns_has_rel, ns_has_rel, n_ns);
  for (uint32_t i = 0; i < n_rel; i++) {
    int found; uint32_t* v = tmap_put(&ix->rel_map, rel_ns[i], rel_rel[i], &found);
    *v = (uint32_t)(rel_root[i] + 1);
  }
  ix->n_rw = n_rw; ix->rw = (ko_rw*)malloc((n_rw + 1) * sizeof(ko_rw));
  if (n_rw) memcpy(ix->rw, rw5, n_rw * sizeof(ko_rw));
  ix->n_child = n_child; ix->child = (int32_t*)malloc((n_child + 1) * 4);
  if (n_child) memcpy(ix->child, child, n_child * 4);
  return 0;
}

/* astRelationFor (engine.go:209-229): returns 0 = no rewrite, 1 = rewrite (*root set), -1 = error */
static int relation_for(const ko_index* ix, uint32_t ns, uint32_t rel, int32_t* root) {
  if (ns >= ix->n_ns || !ix->ns_has_rel[ns]) return 0; /* unknown ns or no relations */
  const uint32_t* v = tmap_get(&ix->rel_map, ns, rel);
  if (!v) return -1; /* relation %q not found */
  if (*v == 0) return 0;
  *root = (int32_t)*v - 1;
  return 1;
}

/* ---------------------------------------------------------------- evaluation */
typedef struct { tmap m; } vset;

typedef struct {
  const ko_index* ix;
  uint32_t subj;          /* tagged query subject; NONE for an unknown subject set */
  int policy;
  int32_t err;
  tmap memo;              /* canonical: (node-triple, d) -> result+1, 0xFF = in progress */
  uint64_t rows_opened, edges_read, probes;
} ctx_t;

typedef struct { uint32_t ns, obj, rel; } trip;

static int direct(ctx_t* c, trip n, uint32_t node, int d) {
  if (d < 0) return KO_U;
  c->probes++;
  if (node == NONE || c->subj == NONE) return KO_N;
  const ko_index* ix = c->ix;
  uint64_t lo = ix->row_off[node], hi = ix->row_off[node + 1];
  while (lo < hi) { /* binary search == SQL index lookup (sqlite.up.sql:22-27) */
    uint64_t mid = (lo + hi) >> 1; uint32_t v = ix->row_sorted[mid];
    if (v == c->subj) return KO_M;
    if (v < c->subj) lo = mid + 1; else hi = mid;
  }
  (void)n;
  return KO_N;
}

static int cia(ctx_t* c, trip n, uint32_t node, int d, vset* scope);

static int is_decisive(int r) { return r == KO_M || r == KO_ERR; }

/* checkExpandSubject (engine.go:87-145) */
static int expand_subject(ctx_t* c, uint32_t node, int d, vset* scope) {
  if (d < 0) return KO_U;
  const ko_index* ix = c->ix;
  if (node == NONE) return KO_N;
  uint64_t b = ix->row_off[node], e = ix->row_off[node + 1];
  c->rows_opened++;
  int res = KO_N, decided = 0;
  if (c->policy == KO_POLICY_CANONICAL) {
    for (uint64_t i = b; i < e; i++) {
      uint32_t s = ix->row_subj[i]; c->edges_read++;
      if (!(s & SET_BIT)) continue;
      uint32_t sn = s & ~SET_BIT;
      if (ix->nd_rel[sn] == ix->wildcard_rel) continue;
      trip ch = {ix->nd_ns[sn], ix->nd_obj[sn], ix->nd_rel[sn]};
      int r = cia(c, ch, sn, d - 1, NULL);
      if (is_decisive(r)) return r;
    }
    return KO_N;
  }
  /* DFS policy: graph.InitVisited -- reuse the scope, else create one for this subtree */
  vset own; int mine = 0;
  if (!scope) { tmap_init(&own.m, 64); scope = &own; mine = 1; }
  for (uint64_t i = b; i < e; i++) {
    if (decided && ((i - b) % ix->page_size) == 0) break; /* g.Done() checked at page end */
    uint32_t s = ix->row_subj[i]; c->edges_read++;
    int found; tmap_put(&scope->m, s, 0, &found); /* CheckAndAddVisited marks first */
    if (found) continue;
    if (!(s & SET_BIT)) continue;
    uint32_t sn = s & ~SET_BIT;
    if (ix->nd_rel[sn] == ix->wildcard_rel) continue;
    if (decided) continue; /* page tail: marked, its check is never consumed */
    trip ch = {ix->nd_ns[sn], ix->nd_obj[sn], ix->nd_rel[sn]};
    int r = cia(c, ch, sn, d - 1, scope);
    if (is_decisive(r)) { res = r; decided = 1; }
  }
  if (mine) tmap_free(&own.m);
  return res;
}

static int eval_rw(ctx_t* c, int32_t idx, trip n, int d, vset* scope);

/* checkTupleToSubjectSet (rewrites.go:205-260): every SubjectSet row (any relation, also "...")
 * of (ns,obj,ttu.rel) -> checkIsAllowed(set.ns, set.obj, computed, d-1); no visited marking. */
static int ttu(ctx_t* c, trip n, uint32_t rel, uint32_t crel, int d, vset* scope) {
  if (d < 0) return KO_U;
  const ko_index* ix = c->ix;
  uint32_t node = node_find(ix, n.ns, n.obj, rel);
  if (node == NONE) return KO_N;
  c->rows_opened++;
  for (uint64_t i = ix->row_off[node]; i < ix->row_off[node + 1]; i++) {
    uint32_t s = ix->row_subj[i]; c->edges_read++;
    if (!(s & SET_BIT)) continue;
    uint32_t sn = s & ~SET_BIT;
    trip ch = {ix->nd_ns[sn], ix->nd_obj[sn], crel};
    int r = cia(c, ch, LOOKUP, d - 1, scope);
    if (is_decisive(r)) return r;
  }
  return KO_N;
}

static int eval_child(ctx_t* c, int32_t idx, trip n, int d, vset* scope) {
  const ko_rw* w = &c->ix->rw[idx];
  switch (w->kind) {
    case RW_OR: case RW_AND: return eval_rw(c, idx, n, d, scope);
    case RW_COMPUTED: { /* rewrites.go:167-193: same depth */
      if (d < 0) return KO_U;
      trip ch = {n.ns, n.obj, (uint32_t)w->rel};
      return cia(c, ch, LOOKUP, d, scope);
    }
    case RW_TTU: return ttu(c, n, (uint32_t)w->rel, (uint32_t)w->crel, d, scope);
    case RW_NOT: { /* rewrites.go:95-159 */
      if (d < 0) return KO_U;
      if (w->count != 1) { c->err = KO_ERR_NOT_IMPLEMENTED; return KO_ERR; }
      int r = eval_child(c, c->ix->child[w->first], n, d, scope);
      if (r == KO_M) return KO_N;
      if (r == KO_N) return KO_M;
      return r;
    }
    default: c->err = KO_ERR_NOT_IMPLEMENTED; return KO_ERR;
  }
}

/* checkSubjectSetRewrite + or/and (rewrites.go:30-93, binop.go:15-70) */
static int eval_rw(ctx_t* c, int32_t idx, trip n, int d, vset* scope) {
  if (d < 0) return KO_U;
  const ko_rw* w = &c->ix->rw[idx];
  if (w->kind != RW_OR && w->kind != RW_AND) { c->err = KO_ERR_NOT_IMPLEMENTED; return KO_ERR; }
  if (w->count == 0) return KO_N;
  for (int32_t k = 0; k < w->count; k++) {
    int r = eval_child(c, c->ix->child[w->first + k], n, d, scope);
    if (w->kind == RW_OR) { if (is_decisive(r)) return r; }
    else { if (r == KO_ERR) return KO_ERR; if (r != KO_M) return KO_N; }
  }
  return w->kind == RW_OR ? KO_N : KO_M;
}

/* checkIsAllowed (engine.go:183-207) */
static int cia(ctx_t* c, trip n, uint32_t node, int d, vset* scope) {
  if (d < 0) return KO_U;
  const ko_index* ix = c->ix;
  uint32_t* memo = NULL;
  if (c->policy == KO_POLICY_CANONICAL) {
    int found;
    memo = tmap_put(&c->memo, ((uint64_t)n.ns << 32) | n.rel, ((uint64_t)n.obj << 32) | (uint32_t)d, &found);
    if (found) {
      if (*memo == 0xFF) { c->err = KO_ERR_REWRITE_CYCLE; return KO_ERR; }
      return (int)*memo - 1;
    }
    *memo = 0xFF;
  }
  if (node == LOOKUP) node = node_find(ix, n.ns, n.obj, n.rel);
  int r = direct(c, n, node, d - 1);
  if (!is_decisive(r)) {
    r = expand_subject(c, node, d, scope);
    if (!is_decisive(r)) {
      int32_t root = -1;
      int k = relation_for(ix, n.ns, n.rel, &root);
      if (k < 0) { c->err = KO_ERR_RELATION_NOT_FOUND; r = KO_ERR; }
      else if (k > 0) { r = eval_rw(c, root, n, d, scope); if (!is_decisive(r)) r = KO_N; }
      else r = KO_N; /* group: Unknown collapses to NotMember */
    }
  }
  if (memo) {
    /* memo may have moved on growth: re-find */
    int found;
    uint32_t* m2 = tmap_put(&c->memo, ((uint64_t)n.ns << 32) | n.rel, ((uint64_t)n.obj << 32) | (uint32_t)d, &found);
    *m2 = (uint32_t)r + 1;
  }
  return r;
}

static int clamp_depth(int rest, int global) {
  if (rest <= 0 || global < rest) rest = global; /* engine.go:68-70 */
  return rest;
}

static uint32_t subject_tag(const ko_index* ix, const ko_tuple* q) {
  if (q->sns == KO_SUBJECT_ID) return q->sobj & ~SET_BIT;
  uint32_t sn = node_find(ix, q->sns, q->sobj, q->srel);
  return sn == NONE ? NONE : (SET_BIT | sn);
}

typedef struct { uint64_t rows_opened, edges_read, probes; } ko_stats;

static int check_one(const ko_index* ix, const ko_tuple* q, uint32_t root_node, uint32_t subj_tag, int rest_depth,
                     int global, int policy, int32_t* err, ko_stats* st) {
  ctx_t c; memset(&c, 0, sizeof c);
  c.ix = ix; c.policy = policy; c.subj = subj_tag == LOOKUP ? subject_tag(ix, q) : subj_tag;
  if (policy == KO_POLICY_CANONICAL) tmap_init(&c.memo, 64);
  trip root = {q->ns, q->obj, q->rel};
  int r = cia(&c, root, root_node, clamp_depth(rest_depth, global), NULL);
  if (policy == KO_POLICY_CANONICAL) tmap_free(&c.memo);
  if (err) *err = r == KO_ERR ? (c.err ? c.err : KO_ERR_NOT_IMPLEMENTED) : KO_ERR_NONE;
  if (st) { st->rows_opened += c.rows_opened; st->edges_read += c.edges_read; st->probes += c.probes; }
  if (r == KO_ERR) return KO_ERR;
  return r == KO_M ? KO_M : KO_N; /* CheckIsMember: allowed <=> IsMember */
}

/* returns 0 = not allowed, 1 = allowed, 2 = error (code in *err) */
int ko_check(const ko_index* ix, const ko_tuple* q, int rest_depth, int global, int policy, int32_t* err) {
  if (!ix->finalized) return -1;
  return check_one(ix, q, LOOKUP, LOOKUP, rest_depth, global, policy, err, NULL);
}

typedef struct {
  const ko_index* ix; const ko_tuple* q; const uint32_t* qnode; const uint32_t* qsubj;
  const int32_t* depth; uint64_t n; int global, policy; uint8_t* out; int32_t* err;
  uint64_t next; pthread_mutex_t* mu; ko_stats st;
} batch_arg;

static void* batch_worker(void* p) {
  batch_arg* a = (batch_arg*)p;
  ko_stats mine = {0, 0, 0};  /* per-thread counters, added once: no lock per check */
  for (;;) {
    pthread_mutex_lock(a->mu);
    uint64_t i0 = a->next; a->next += 64;
    pthread_mutex_unlock(a->mu);
    if (i0 >= a->n) break;
    uint64_t i1 = i0 + 64 < a->n ? i0 + 64 : a->n;
    for (uint64_t i = i0; i < i1; i++) {
      int32_t e = 0; ko_tuple qq; uint32_t rn = LOOKUP, sg = LOOKUP;
      if (a->q) qq = a->q[i];
      else {
        uint32_t v = a->qnode[i];
        qq.ns = a->ix->nd_ns[v]; qq.obj = a->ix->nd_obj[v]; qq.rel = a->ix->nd_rel[v];
        qq.sns = qq.sobj = qq.srel = 0;
        rn = v; sg = a->qsubj[i];
      }
      ko_stats st = {0, 0, 0};
      a->out[i] = (uint8_t)check_one(a->ix, &qq, rn, sg, a->depth[i], a->global, a->policy, &e, &st);
      if (a->err) a->err[i] = e;
      mine.rows_opened += st.rows_opened; mine.edges_read += st.edges_read; mine.probes += st.probes;
    }
  }
  pthread_mutex_lock(a->mu);
  a->st.rows_opened += mine.rows_opened; a->st.edges_read += mine.edges_read; a->st.probes += mine.probes;
  pthread_mutex_unlock(a->mu);
  return NULL;
}

static int run_batch(batch_arg* a, int nthreads, uint64_t* stats3) {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  a->mu = &mu; a->next = 0; memset(&a->st, 0, sizeof a->st);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, a);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  if (stats3) { stats3[0] = a->st.rows_opened; stats3[1] = a->st.edges_read; stats3[2] = a->st.probes; }
  return 0;
}

/* Batch of string-level queries (already interned). */
int ko_check_batch(const ko_index* ix, const ko_tuple* q, const int32_t* depth, uint64_t n, int global,
                   int policy, int nthreads, uint8_t* out, int32_t* err, uint64_t* stats3) {
  if (!ix->finalized) return -1;
  batch_arg a; memset(&a, 0, sizeof a);
  a.ix = ix; a.q = q; a.depth = depth; a.n = n; a.global = global; a.policy = policy; a.out = out; a.err = err;
  return run_batch(&a, nthreads, stats3);
}

/* Batch of node-level queries (root node id + tagged subject), for the synthetic graphs. */
int ko_check_nodes_batch(const ko_index* ix, const uint32_t* qnode, const uint32_t* qsubj, const int32_t* depth,
                         uint64_t n, int global, int policy, int nthreads, uint8_t* out, uint64_t* stats3) {
  if (!ix->finalized) return -1;
  batch_arg a; memset(&a, 0, sizeof a);
  a.ix = ix; a.qnode = qnode; a.qsubj = qsubj; a.depth = depth; a.n = n; a.global = global; a.policy = policy;
  a.out = out;
  return run_batch(&a, nthreads, stats3);
}

/* ---------------------------------------------------------------- expand (expand/engine.go:35-104)
 * Output: pre-order records of 6 int32 {type, is_set, ns, obj, rel, n_children};
 * type 1 = union, 2 = leaf.  SubjectID: is_set=0, obj=id, ns=rel=-1. */
typedef struct { int32_t* buf; int64_t cap, n; int overflow; } tbuf;

static int64_t emit(tbuf* t, int type, uint32_t subj, const ko_index* ix) {
  int64_t at = t->n;
  if ((t->n + 1) * 6 > t->cap) { t->overflow = 1; t->n++; return at; }
  int32_t* r = t->buf + t->n * 6;
  r[0] = type;
  if (subj & SET_BIT) { uint32_t v = subj & ~SET_BIT; r[1] = 1; r[2] = ix->nd_ns[v]; r[3] = ix->nd_obj[v]; r[4] = ix->nd_rel[v]; }
  else { r[1] = 0; r[2] = -1; r[3] = (int32_t)subj; r[4] = -1; }
  r[5] = 0;
  t->n++;
  return at;
}

/* returns 1 if a node was emitted, 0 for nil */
static int build_tree(const ko_index* ix, uint32_t subj, int d, int global, tmap* visited, tbuf* t) {
  d = clamp_depth(d, global); /* re-applied at every level (engine.go:37-39) */
  if (!(subj & SET_BIT)) { emit(t, 2, subj, ix); return 1; }
  int found; tmap_put(visited, subj, 0, &found);
  if (found) return 0;
  uint32_t v = subj & ~SET_BIT;
  uint64_t b = ix->row_off[v], e = ix->row_off[v + 1];
  if (b == e) return 0;
  if (d <= 1) { emit(t, 2, subj, ix); return 1; }
  int64_t me = emit(t, 1, subj, ix);
  int32_t nch = 0;
  for (uint64_t i = b; i < e; i++) {
    uint32_t s = ix->row_subj[i];
    if (!build_tree(ix, s, d - 1, global, visited, t)) emit(t, 2, s, ix);
    nch++;
  }
  if (!t->overflow) t->buf[me * 6 + 5] = nch;
  return 1;
}

/* Expand a subject set (sns,sobj,srel) or a subject id (sns == KO_SUBJECT_ID, id in sobj).
 * Returns the number of records (0 = nil tree), or -(needed) if cap is too small. */
int64_t ko_expand(const ko_index* ix, uint32_t sns, uint32_t sobj, uint32_t srel, int rest_depth, int global,
                  int32_t* buf, int64_t cap_records) {
  if (!ix->finalized) return -1;
  tbuf t = {buf, cap_records * 6, 0, 0};
  uint32_t subj;
  if (sns == KO_SUBJECT_ID) subj = sobj & ~SET_BIT;
  else {
    uint32_t v = node_find(ix, sns, sobj, srel);
    if (v == NONE) return 0; /* no rows anywhere: BuildTree returns nil */
    subj = SET_BIT | v;
  }
  tmap visited; tmap_init(&visited, 64);
  int ok = build_tree(ix, subj, rest_depth, global, &visited, &t);
  tmap_free(&visited);
  if (!ok) return 0;
  return t.overflow ? -t.n : t.n;
}

/* ko_expand with the root given as a node id (an index built without a node map, e.g. the synthetic
 * graphs' group#member roots, whose node id equals their object id). */
int64_t ko_expand_node(const ko_index* ix, uint32_t node, int rest_depth, int global, int32_t* buf,
                       int64_t cap_records) {
  if (!ix->finalized || node >= ix->n_nodes) return -1;
  tbuf t = {buf, cap_records * 6, 0, 0};
  tmap visited; tmap_init(&visited, 64);
  int ok = build_tree(ix, SET_BIT | node, rest_depth, global, &visited, &t);
  tmap_free(&visited);
  if (!ok) return 0;
  return t.overflow ? -t.n : t.n;
}

/* Batch of ko_expand_node over `n` root nodes on `nthreads` threads (the C5 CPU baseline: every tree is
 * built into a per-thread buffer, as BuildTree's result would be serialised, then dropped).  counts[i] =
 * records of root i (0 = nil).  Returns 0, or -1 if a buffer could not be allocated. */
typedef struct {
  const ko_index* ix; const uint32_t* node; const int32_t* depth; uint64_t n; int global; int64_t* counts;
  uint64_t next; pthread_mutex_t* mu; int fail;
} expand_arg;

static void* expand_worker(void* p) {
  expand_arg* a = (expand_arg*)p;
  int64_t cap = 1 << 16;
  int32_t* buf = (int32_t*)malloc((size_t)cap * 6 * sizeof(int32_t));
  for (;;) {
    pthread_mutex_lock(a->mu);
    uint64_t i0 = a->next; a->next += 16;
    pthread_mutex_unlock(a->mu);
    if (i0 >= a->n || !buf) break;
    uint64_t i1 = i0 + 16 < a->n ? i0 + 16 : a->n;
    for (uint64_t i = i0; i < i1 && buf; i++) {
      int64_t r = ko_expand_node(a->ix, a->node[i], a->depth[i], a->global, buf, cap);
      while (r < 0 && r != -1) { /* grow to the size it asked for and rebuild */
        cap = -r + 1024;
        free(buf);
        buf = (int32_t*)malloc((size_t)cap * 6 * sizeof(int32_t));
        if (!buf) break;
        r = ko_expand_node(a->ix, a->node[i], a->depth[i], a->global, buf, cap);
      }
      a->counts[i] = r;
    }
  }
  if (!buf) { pthread_mutex_lock(a->mu); a->fail = 1; pthread_mutex_unlock(a->mu); }
  free(buf);
  return NULL;
}

int ko_expand_nodes_batch(const ko_index* ix, const uint32_t* node, const int32_t* depth, uint64_t n, int global,
                          int nthreads, int64_t* counts) {
  if (!ix->finalized) return -1;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  expand_arg a = {ix, node, depth, n, global, counts, 0, &mu, 0};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, expand_worker, &a);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  return a.fail ? -1 : 0;
}
