// kg_check.hip -- batched permission checks on gfx950.
//
// Replaces the reference's per-request recursion (internal/check/engine.go:54-207 +
// checkgroup/concurrent_checkgroup.go) with a batch pipeline, one HIP stream:
//
//   k_resolve   request mapping (uuid_mapping.go:180-238 analogue on dense ids): (ns,obj,rel) ->
//               node via the device node map, depth clamp (engine.go:68-70), routing:
//                 DONE    node has no rows and its relation has no rewrite -> NotMember
//                 LIGHT   every node reachable through subject sets is rewrite-free
//                 GENERAL a rewrite / undeclared relation is reachable (rewrite interpreter)
//   k_light     one wave64 per query, frontier + visited set in LDS: level-synchronous BFS over
//               the set-adjacency CSR.  Level k holds nodes at rest depth D-k; each is probed for
//               the exact tuple (checkDirect at d-1 >= 0) and, when D-k >= 2, expanded
//               (checkExpandSubject's children at d-1).  On rewrite-free nodes the reference's
//               group semantics reduce to "a path of <= D-1 subject-set hops to a node holding
//               the tuple" -- SURVEY.md 8a; BFS marks every node at its shallowest depth, which
//               is the schedule-free answer.  Early exit on the first hit (group: first
//               IsMember wins, concurrent_checkgroup.go:104-115).
//   k_heavy     one workgroup (256 lanes) per query whose visited set overflowed LDS: same
//               algorithm, visited bitmap + BFS list in HBM (per-slot), block-wide edge split.
//   k_general   rewrite interpreter (kg_interp.hip).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kg_bfs.h"
#include "kg_internal.h"
#include "kg_interp.h"
#include "kg_snapshot.h"

namespace kg {

// Counters: [0] rows_opened [1] edges_read [2] probes [3] frontier_hbm [4] light [5] heavy [6] general
enum { ST_ROWS = 0, ST_EDGES, ST_PROBES, ST_FHBM, ST_LIGHT, ST_HEAVY, ST_GENERAL, ST_LROWS, ST_LEDGES, ST_LPROBES, ST_N };

// Device-side counters/heads (zeroed per batch).
struct Ctl {
  uint32_t light_count, gen_count, heavy_count, giant_count;
  uint32_t heavy_head, giant_head, gen_head, pad0;
  uint32_t heads[8 * 32];  // per-XCD dequeue heads, one 128-B line each
  unsigned long long st[ST_N];
  InterpCtl ic;
};

// ------------------------------------------------------------------ k_resolve
__global__ __launch_bounds__(256) void k_resolve(DevSnap s, const kg_query* __restrict__ q, uint32_t n,
                                                 int32_t global, RQuery* __restrict__ rq, uint8_t* __restrict__ out,
                                                 uint32_t* __restrict__ err, uint32_t* light_list,
                                                 uint32_t* gen_list, Ctl* ctl) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < n;
  uint32_t route = ROUTE_DONE;
  if (valid) {
    kg_query x = q[i];
    uint32_t node = nmap_find(s, x.t.ns, x.t.rel, x.t.obj);
    uint32_t subj;
    if (x.t.sns == KG_SUBJECT_ID) {
      subj = x.t.sobj < 0x7FFFFFFFu ? x.t.sobj : NONE;
    } else {
      uint32_t sn = nmap_find(s, x.t.sns, x.t.srel, x.t.sobj);
      subj = sn == NONE ? NONE : (SET_BIT | sn);
    }
    int32_t d = x.max_depth;
    if (d <= 0 || global < d) d = global;  // engine.go:68-70
    const uint8_t rf = relflag(s, x.t.ns, x.t.rel);
    if (node == NONE) {
      route = rf ? ROUTE_GENERAL : ROUTE_DONE;
    } else {
      bool impure = s.nflags && (s.nflags[node] & NF_IMPURE);
      route = impure ? ROUTE_GENERAL : ROUTE_LIGHT;
    }
    rq[i] = RQuery{node, subj, d, route};
    if (route == ROUTE_DONE) {
      out[i] = KG_NOT_MEMBER;
      if (err) err[i] = KG_ERR_NONE;
    }
  }
  wave_append(valid && route == ROUTE_LIGHT, i, light_list, &ctl->light_count);
  wave_append(valid && route == ROUTE_GENERAL, i, gen_list, &ctl->gen_count);
}

// ------------------------------------------------------------------ k_light
constexpr int LWAVES = 4;  // waves per workgroup (256 threads)

// Dequeue one work index; per-XCD heads over [0, count) split into 8 ranges.
__device__ __forceinline__ uint32_t dequeue(uint32_t* heads, uint32_t count, uint32_t& head_sel, uint32_t head0) {
  while (head_sel < head0 + 8) {
    uint32_t h = head_sel & 7;
    uint32_t lo = (uint32_t)((uint64_t)count * h / 8), hi = (uint32_t)((uint64_t)count * (h + 1) / 8);
    uint32_t k = atomicAdd(&heads[h * 32], 1u);
    if (lo + k < hi) return lo + k;
    head_sel++;
  }
  return NONE;
}

__global__ __launch_bounds__(256) void k_light(DevSnap s, const RQuery* __restrict__ rq,
                                               const uint32_t* __restrict__ light_list, uint8_t* __restrict__ out,
                                               uint32_t* __restrict__ err, uint32_t* heavy_list, Ctl* ctl) {
  __shared__ WaveLds lds_all[LWAVES];
  const int wave = threadIdx.x >> 6, lane = lane_id();
  LdsStore st{&lds_all[wave]};
  const uint32_t count = ctl->light_count;
  const uint32_t head0 = blockIdx.x & 7;  // XCD label (speed only, never correctness)
  uint32_t head_sel = head0;
  BfsStats bs;
  unsigned long long st_done = 0;
  for (;;) {
    uint32_t li = 0;
    if (lane == 0) li = dequeue(ctl->heads, count, head_sel, head0);
    li = __shfl(li, 0, 64);
    if (li == NONE) break;
    const uint32_t qi = light_list[li];
    const RQuery q = rq[qi];
    st.reset();
    uint32_t n = 0;
    wave_add_roots(st, lane == 0, q.node, n);
    const int r = wave_bfs_run(s, st, n, q.depth, q.subj, bs);
    if (r == BFS_OVERFLOW) {
      if (lane == 0) heavy_list[atomicAdd(&ctl->heavy_count, 1u)] = qi;
    } else if (lane == 0) {
      out[qi] = r == BFS_M ? KG_IS_MEMBER : KG_NOT_MEMBER;
      if (err) err[qi] = KG_ERR_NONE;
      st_done++;
    }
  }
  if (lane == 0) {
    atomicAdd(&ctl->st[ST_LROWS], bs.rows);
    atomicAdd(&ctl->st[ST_LEDGES], bs.edges);
    atomicAdd(&ctl->st[ST_LPROBES], bs.probes);
    atomicAdd(&ctl->st[ST_LIGHT], st_done);
  }
}

// ------------------------------------------------------------------ k_heavy
// One 256-lane workgroup per overflowed query.  Per-slot HBM state: visited bitmap (n_nodes bits)
// and the BFS list (cap entries).  A query whose list would exceed cap is forwarded to the
// "giant" pass (same kernel, one slot, cap = n_nodes).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t wt;
  uint32_t e = wave_excl_scan(x, &wt);
  if (lane == 0) wsum[wave] = wt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < 4; w++) {
    uint32_t v = wsum[w];
    if (w < wave) off += v;
    tot += v;
  }
  *total = tot;
  __syncthreads();
  return e + off;
}

__global__ __launch_bounds__(256) void k_heavy(DevSnap s, const RQuery* __restrict__ rq, const uint32_t* hlist,
                                               const uint32_t* hcount_p, uint32_t* hhead, uint8_t* __restrict__ out,
                                               uint32_t* __restrict__ err, uint32_t* bitmaps, uint64_t words_per_slot,
                                               uint32_t* lists, uint64_t cap, uint32_t* giant_list,
                                               uint32_t* giant_count, Ctl* ctl) {
  __shared__ uint32_t sh_qi, sh_n, sh_hit, sh_over;
  __shared__ uint32_t pref[256];
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x;
  uint32_t* bm = bitmaps + (uint64_t)blockIdx.x * words_per_slot;
  uint32_t* list = lists + (uint64_t)blockIdx.x * cap;
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_fh = 0, st_done = 0;
  const uint32_t hcount = *hcount_p;
  for (;;) {
    if (tid == 0) sh_qi = atomicAdd(hhead, 1u);
    __syncthreads();
    const uint32_t hi = sh_qi;
    if (hi >= hcount) break;
    const uint32_t qi = hlist[hi];
    const RQuery q = rq[qi];
    if (tid == 0) {
      list[0] = q.node;
      atomicOr(&bm[q.node >> 5], 1u << (q.node & 31));
      sh_n = 1;
      sh_hit = 0;
      sh_over = 0;
    }
    __syncthreads();
    uint32_t lvl_b = 0, lvl_e = 1;
    for (int k = 0;; k++) {
      const int d = q.depth - k;
      if (d < 1) break;
      const bool expand = d >= 2;
      for (uint32_t base = lvl_b; base < lvl_e; base += 256) {
        const uint32_t i = base + tid;
        const bool valid = i < lvl_e;
        const uint32_t node = valid ? list[i] : 0;
        uint64_t rb = 0, re = 0;
        if (valid && expand) {
          rb = s.adj_off[node];
          re = s.adj_off[node + 1];
        }
        if (valid && dset_probe(s, node, q.subj)) sh_hit = 1;
        if (tid == 0) {
          uint32_t nv = min(256u, lvl_e - base);
          st_probes += nv;
          st_fh += nv;
          if (expand) st_rows += nv;
        }
        uint32_t total;
        const uint32_t excl = block_excl_scan(expand ? (uint32_t)(re - rb) : 0u, wsum, &total);
        pref[tid] = excl;
        __syncthreads();
        if (sh_hit) break;
        if (tid == 0) st_edges += total;
        for (uint32_t eb = 0; eb < total; eb += 256) {
          const uint32_t e = eb + tid;
          if (e < total) {
            int own = owner_search(pref, 256, e);
            uint64_t src = 0;
            // rb of the owner: recompute from its node (owner lane's rb is in another wave)
            uint32_t onode = list[base + own];
            src = s.adj_off[onode] + (e - pref[own]);
            uint32_t child = s.adj[src];
            uint32_t bit = 1u << (child & 31);
            uint32_t old = atomicOr(&bm[child >> 5], bit);
            if (!(old & bit)) {
              uint32_t pos = atomicAdd(&sh_n, 1u);
              if (pos < cap) list[pos] = child;
              else sh_over = 1;
            }
          }
        }
        __syncthreads();
        if (sh_over) break;
      }
      __syncthreads();
      if (sh_hit || sh_over) break;
      lvl_b = lvl_e;
      lvl_e = sh_n;
      if (lvl_b == lvl_e) break;
    }
    __syncthreads();
    const uint32_t n_list = (uint32_t)min((uint64_t)sh_n, cap);
    if (tid == 0) {
      if (sh_over && !sh_hit) {
        giant_list[atomicAdd(giant_count, 1u)] = qi;
      } else {
        out[qi] = sh_hit ? KG_IS_MEMBER : KG_NOT_MEMBER;
        if (err) err[qi] = KG_ERR_NONE;
        st_done++;
      }
    }
    // clear this query's bits (every set bit in a touched word belongs to this query); after an
    // overflow some set bits have no list entry, so the whole slot bitmap is cleared instead
    if (sh_over) {
      for (uint64_t w = tid; w < words_per_slot; w += 256) bm[w] = 0u;
    } else {
      for (uint32_t i = tid; i < n_list; i += 256) atomicAnd(&bm[list[i] >> 5], 0u);
    }
    __syncthreads();
  }
  if (tid == 0) {
    atomicAdd(&ctl->st[ST_ROWS], st_rows);
    atomicAdd(&ctl->st[ST_EDGES], st_edges);
    atomicAdd(&ctl->st[ST_PROBES], st_probes);
    atomicAdd(&ctl->st[ST_FHBM], st_fh);
    atomicAdd(&ctl->st[ST_HEAVY], st_done);
  }
}

// ------------------------------------------------------------------ synthetic queries
__global__ void k_synth_queries(SynthLayout L, DevSnap s, uint64_t seed, uint32_t n, kg_query* q) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t doc = (uint32_t)(shash(seed, i, 7) % L.n_docs);
  int32_t md = (int32_t)(shash(seed, i, 8) % 11);  // 0 (-> global) or 1..10
  uint32_t user = NONE;
  uint32_t rel = L.rel_viewer, start = doc;
  if (L.preset == 1) {  // C3: view / edit / share, walks start at viewer / editor / owner rows
    const uint32_t k = (uint32_t)(shash(seed, i, 11) % 3);
    rel = k == 0 ? L.rel_view : (k == 1 ? L.rel_edit : L.rel_share);
    const uint32_t want = (uint32_t)(shash(seed, i, 12) % 3);
    const uint32_t wrel = want == 0 ? L.rel_viewer : (want == 1 ? L.rel_editor : L.rel_owner);
    for (uint32_t b = 0; b < L.n_blocks; b++)
      if (L.b[b].ns == L.ns_doc && L.b[b].rel == wrel) start = L.b[b].node0 + doc;
  }
  if ((i & 1) == 0) {  // positive: walk down random rows until a subject id
    uint32_t cur = start;
    for (int step = 0; step < 16; step++) {
      uint64_t b = s.row_off[cur], e = s.row_off[cur + 1];
      if (e == b) break;
      uint32_t sub = s.row_subj[b + shash(seed, ((uint64_t)i << 8) | step, 9) % (e - b)];
      if (!(sub & SET_BIT)) {
        user = sub;
        break;
      }
      cur = sub & ~SET_BIT;
    }
  }
  if (user == NONE) user = L.user_obj0 + (uint32_t)(shash(seed, i, 10) % L.n_users);
  kg_query x;
  x.t.ns = L.ns_doc;
  x.t.obj = doc;
  x.t.rel = rel;
  x.t.sns = KG_SUBJECT_ID;
  x.t.sobj = user;
  x.t.srel = 0;
  x.max_depth = md;
  q[i] = x;
}

int synth_queries(Snapshot* s, uint64_t seed, size_t n, kg_query* d_q) {
  if (!s->is_synth) return set_error(-2, "kg_synth_queries needs a synthetic snapshot");
  HIPC(hipSetDevice(s->device));
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_synth_queries, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s->stream, s->synth, s->ds,
                     seed, (uint32_t)n, d_q);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s->stream));
  return 0;
}

// ------------------------------------------------------------------ batch driver
static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int check_batch_device(Snapshot* s, const kg_query* d_q, size_t n, int32_t global_max_depth, uint8_t* d_out,
                       uint32_t* d_err, kg_stats* stats, hipStream_t stream) {
  if (global_max_depth < 1) global_max_depth = 5;  // config.schema.json:308-315 default
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  // scratch: rq[n] | light[n] | gen[n] | heavy[n] | giant[n] | p2[n] | Ctl
  size_t off_rq = 0, off_light = align_up(off_rq + n * sizeof(RQuery)), off_gen = align_up(off_light + n * 4),
         off_heavy = align_up(off_gen + n * 4), off_giant = align_up(off_heavy + n * 4),
         off_p2 = align_up(off_giant + n * 4), off_ctl = align_up(off_p2 + n * 4),
         total = align_up(off_ctl + sizeof(Ctl));
  if (total > s->scratch_bytes) {
    if (s->scratch) hipFree(s->scratch);
    s->scratch = nullptr;
    s->scratch_bytes = 0;
    HIPC(hipMalloc(&s->scratch, total));
    s->scratch_bytes = total;
  }
  char* base = (char*)s->scratch;
  RQuery* rq = (RQuery*)(base + off_rq);
  uint32_t* light = (uint32_t*)(base + off_light);
  uint32_t* gen = (uint32_t*)(base + off_gen);
  uint32_t* heavy = (uint32_t*)(base + off_heavy);
  uint32_t* giant = (uint32_t*)(base + off_giant);
  uint32_t* p2 = (uint32_t*)(base + off_p2);
  Ctl* ctl = (Ctl*)(base + off_ctl);
  // heavy pool: H slots of (bitmap + cap list) + one giant slot (bitmap + n_nodes list)
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  const uint64_t words = (nn + 31) / 32 + 1;
  const uint64_t cap_h = std::min<uint64_t>(nn, 4u << 20);
  const uint32_t H = (uint32_t)std::min<uint64_t>(2 * (uint64_t)s->n_cu, std::max<uint64_t>(
                                                      1, (8ull << 30) / ((words + cap_h) * 4)));
  const size_t pool = ((size_t)H * (words + cap_h) + (words + nn)) * 4;
  if (pool > s->heavy_pool_bytes) {
    if (s->heavy_pool) hipFree(s->heavy_pool);
    s->heavy_pool = nullptr;
    s->heavy_pool_bytes = 0;
    HIPC(hipMalloc(&s->heavy_pool, pool));
    HIPC(hipMemsetAsync(s->heavy_pool, 0, pool, stream));  // bitmaps start clear and are left clear
    s->heavy_pool_bytes = pool;
  }
  uint32_t* hb = (uint32_t*)s->heavy_pool;
  uint32_t* hl = hb + (size_t)H * words;
  uint32_t* gb = hl + (size_t)H * cap_h;
  uint32_t* gl = gb + words;

  hipEvent_t e0 = nullptr, e1 = nullptr, l0 = nullptr, l1 = nullptr;
  if (stats) {
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    HIPC(hipEventCreate(&l0));
    HIPC(hipEventCreate(&l1));
    HIPC(hipEventRecord(e0, stream));
  }
  HIPC(hipMemsetAsync(ctl, 0, sizeof(Ctl), stream));
  if (n) {
    hipLaunchKernelGGL(k_resolve, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, s->ds, d_q, (uint32_t)n,
                       global_max_depth, rq, d_out, d_err, light, gen, ctl);
    HIPC(hipGetLastError());
    const uint32_t light_grid = (uint32_t)std::min<uint64_t>((uint64_t)s->n_cu * 6, (n + 3) / 4 + 8);
    if (stats) HIPC(hipEventRecord(l0, stream));
    hipLaunchKernelGGL(k_light, dim3(light_grid), dim3(256), 0, stream, s->ds, rq, light, d_out, d_err, heavy, ctl);
    HIPC(hipGetLastError());
    if (stats) HIPC(hipEventRecord(l1, stream));
    hipLaunchKernelGGL(k_heavy, dim3(H), dim3(256), 0, stream, s->ds, rq, heavy, &ctl->heavy_count, &ctl->heavy_head,
                       d_out, d_err, hb, words, hl, cap_h, giant, &ctl->giant_count, ctl);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_heavy, dim3(1), dim3(256), 0, stream, s->ds, rq, giant, &ctl->giant_count, &ctl->giant_head,
                       d_out, d_err, gb, words, gl, nn, giant /*never overflows*/, &ctl->pad0, ctl);
    HIPC(hipGetLastError());
    if (s->has_program) {
      InterpCtl ic{};
      ic.gen_count = &ctl->gen_count;
      ic.p2_list = p2;
      ic.st_general = &ctl->st[ST_GENERAL];
      ic.st_rows = &ctl->st[ST_ROWS];
      ic.st_edges = &ctl->st[ST_EDGES];
      ic.st_probes = &ctl->st[ST_PROBES];
      HIPC(hipMemcpyAsync(&ctl->ic, &ic, sizeof ic, hipMemcpyHostToDevice, stream));
      if (launch_general(s, d_q, rq, gen, &ctl->gen_count, &ctl->ic, d_out, d_err, stream)) return -1;
    }
  }
  if (stats) {
    HIPC(hipEventRecord(e1, stream));
    HIPC(hipEventSynchronize(e1));
    float ms = 0, lms = 0;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    if (n) HIPC(hipEventElapsedTime(&lms, l0, l1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipEventDestroy(l0);
    hipEventDestroy(l1);
    Ctl h;
    HIPC(hipMemcpy(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    stats->rows_opened = h.st[ST_ROWS] + h.st[ST_LROWS];
    stats->edges_read = h.st[ST_EDGES] + h.st[ST_LEDGES];
    stats->direct_probes = h.st[ST_PROBES] + h.st[ST_LPROBES];
    stats->light_rows_opened = h.st[ST_LROWS];
    stats->light_edges_read = h.st[ST_LEDGES];
    stats->light_probes = h.st[ST_LPROBES];
    stats->light_ms = lms;
    stats->frontier_hbm = h.st[ST_FHBM];
    stats->n_light = h.st[ST_LIGHT];
    stats->n_heavy = h.st[ST_HEAVY];
    stats->n_general = h.st[ST_GENERAL];
    stats->kernel_ms = ms;
  }
  return 0;
}

}  // namespace kg
