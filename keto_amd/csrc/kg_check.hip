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
#include <cstdlib>
#include <cstring>

#include "kg_bfs.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_interp.h"
#include "kg_snapshot.h"

namespace kg {

// Counters: [0] rows_opened [1] edges_read [2] probes [3] frontier_hbm [4] light [5] heavy [6] general
enum { ST_ROWS = 0, ST_EDGES, ST_PROBES, ST_FHBM, ST_LIGHT, ST_HEAVY, ST_GENERAL, ST_LROWS, ST_LEDGES, ST_LPROBES,
       ST_MEDIUM, ST_BROWS, ST_BEDGES, ST_BACK, ST_NOHOLD, ST_LSTEPS, ST_LWAVES, ST_LTICKS, ST_N };
static_assert(ST_N <= 32, "per-XCD counter shards hold 32 counters");

// Device-side counters/heads (zeroed per batch).
struct Ctl {
  uint32_t light_count, gen_count, heavy_count, giant_count;
  uint32_t heavy_head, giant_head, gen_head, pad0;
  uint32_t medium_count, medium_head, light2_count, pad1;
  uint32_t back_head, fwd_count, back2_head, back2_count;  // k_back<64> / k_back<256> lists and heads
  uint32_t heads[8 * 32];   // per-XCD dequeue heads, one 128-B line each (k_light<16>)
  uint32_t heads2[8 * 32];  // (k_light<64>)
  uint32_t light8[8 * 32];  // per-XCD shard sizes of the light list (k_resolve appends)
  unsigned long long st[ST_N];
  unsigned long long st8[8][32];  // per-XCD shards of the hot counters (block-reduced adds)
  // k_stream2 wave span on the device clock, per XCD shard (one 128-B line each): max of ~start
  // (= the earliest start), latest end, longest wave -- workgroup-reduced atomicMax on a zeroed block
  unsigned long long tmax8[8][16];
  InterpCtl ic;
};

// One device-scope atomic on a single word costs ~11 ns at the memory side and one word saturates
// near 90 M updates/s (MI355X_MICROARCH.md, "dequeue"/"fanin"): counters and list appends are
// reduced per workgroup and spread over 8 per-XCD shards.

// Adds v[k] (summed over the workgroup) to counter shard (blockIdx & 7) of stat idx[k].
// Every thread of the workgroup must call it.
template <int N>
__device__ void block_stats(Ctl* ctl, const int (&idx)[N], const unsigned long long (&v)[N]) {
  __shared__ unsigned long long red[4][N];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < N; k++) {
    unsigned long long x = v[k];
    for (int off = 32; off; off >>= 1) x += __shfl_xor(x, off, 64);
    if (lane == 0) red[wave][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    const unsigned long long t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (t) atomicAdd(&ctl->st8[blockIdx.x & 7][idx[threadIdx.x]], t);
  }
  __syncthreads();
}

// Workgroup max of three values (wave-uniform per wave) into XCD shard (blockIdx & 7) of
// ctl->tmax8: one device atomic per workgroup and value.  Every thread must call it.
__device__ void block_max3(Ctl* ctl, unsigned long long a, unsigned long long b, unsigned long long c) {
  __shared__ unsigned long long red[4][3];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[wave][0] = a;
    red[wave][1] = b;
    red[wave][2] = c;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long m = 0;
    for (int w = 0; w < 4; w++) m = max(m, red[w][threadIdx.x]);
    atomicMax(&ctl->tmax8[blockIdx.x & 7][threadIdx.x], m);
  }
  __syncthreads();
}

// Workgroup-aggregated append (one atomic per workgroup).  Every thread must call it.
__device__ void block_append(bool pred, uint32_t val, uint32_t* list, uint32_t* count) {
  __shared__ uint32_t wcnt[4], bbase;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(pred);
  if (lane == 0) wcnt[wave] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    bbase = t ? atomicAdd(count, t) : 0u;
  }
  __syncthreads();
  uint32_t off = bbase;
  for (int w = 0; w < wave; w++) off += wcnt[w];
  if (pred) list[off + lanes_below(m)] = val;
  __syncthreads();
}

// Workgroup-aggregated append of LQuery records (one atomic per workgroup).  The workgroup's records
// are packed in LDS first and leave as one contiguous run of 8-B words: a lane storing its own 24-B
// record would make each store instruction span 24 B x 64 lanes in three partial passes.
// back_cap != 0: the run fills the shard from its end instead -- entries [back_cap - c - t, back_cap - c)
// for the c records appended that way before it (the stream tier's work order, k_resolve).
// Every thread must call it (256 threads).
__device__ void block_append_lq(bool pred, const LQuery& v, LQuery* list, uint32_t* count, uint32_t back_cap = 0) {
  static_assert(sizeof(LQuery) == 24, "LQuery is three 8-B words");
  __shared__ uint32_t wcnt[4], bbase;
  __shared__ LQuery s_lq[256];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(pred);
  if (lane == 0) wcnt[wave] = __popcll(m);
  __syncthreads();
  const uint32_t t = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
  if (threadIdx.x == 0) bbase = t ? atomicAdd(count, t) : 0u;
  uint32_t li = 0;
  for (int w = 0; w < wave; w++) li += wcnt[w];
  if (pred) s_lq[li + lanes_below(m)] = v;
  __syncthreads();
  const uint2* src = reinterpret_cast<const uint2*>(s_lq);
  uint2* dst = reinterpret_cast<uint2*>(list + (back_cap ? back_cap - bbase - t : bbase));
  for (uint32_t k = threadIdx.x; k < 3 * t; k += 256) dst[k] = src[k];
  __syncthreads();
}

// ------------------------------------------------------------------ k_resolve
// lq_list != nullptr (stream variant 15, k_stream4): light-routed queries go to the stream tier as
// LQuery records in 8 shards of lq_cap entries (shard blockIdx & 7) and skip rq[i]; only queries
// that later tiers read by index (GENERAL) are written to rq.
__global__ __launch_bounds__(256) void k_resolve(DevSnap s, const kg_query* __restrict__ q, uint32_t n,
                                                 uint32_t n_base, const uint32_t* __restrict__ n_extra,
                                                 int32_t global, RQuery* __restrict__ rq, uint8_t* __restrict__ out,
                                                 uint32_t* __restrict__ err, uint32_t* light_list,
                                                 uint32_t* gen_list, int no_holder_filter, Ctl* ctl,
                                                 LQuery* lq_list, uint32_t lq_cap, uint32_t big_len, int32_t big_depth) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // n: capacity (list strides); with a formula split the live count is n_base + *n_extra
  bool valid = i < (n_extra ? n_base + *n_extra : n);
  uint32_t route = ROUTE_DONE;
  bool did_probe = false, no_holder = false;
  LQuery lq{};
  if (valid) {
    kg_query x = q[i];
    // node map and (for a subject id) holder hash: the first slots of both are loaded together,
    // so the common case is one round trip for both lookups
    const bool key_ok = nmap_key_ok(x.t.ns, x.t.rel, x.t.obj);
    const uint64_t key = nmap_key(x.t.ns, x.t.rel, x.t.obj);
    const uint64_t ni = hash_home(key, s.nmap_n);
    const bool sid = x.t.sns == KG_SUBJECT_ID;
    uint32_t subj = sid ? (x.t.sobj < 0x7FFFFFFFu ? x.t.sobj : NONE) : NONE;
    const bool want_h = no_holder_filter && sid && subj != NONE;
    // no-holder test for a subject id: one bit of the holder bitmap (36 MB at 1 B tuples, stays in
    // the Infinity Cache) instead of a random line of the holder hash
    const bool use_bits = want_h && s.hbits != nullptr;
    const uint64_t hi = mix64(subj) & s.hmask;
    HSlot h0{};
    uint32_t hw = 0;
    if (use_bits) hw = subj < s.hbits_n ? s.hbits[subj >> 5] : 0u;
    else if (want_h) h0 = s.hslots[hi];
    // without a namespace program nothing can end as an error, so a subject that no row holds is
    // NotMember whatever the root: the bit (an Infinity-Cache hit) is read first and such a query
    // never touches the node map (~13 % of the C2 batch; one random HBM line each)
    const bool unheld = no_holder_filter == 2 && use_bits && !s.relflags && !((hw >> (subj & 31)) & 1u);
    NSlot n0{};
    if (key_ok && !unheld) n0 = s.nmap[ni];
    uint32_t node = NONE, rb = 0, rl = 0, rsig = 0xFFFFFFFFu, nfl = 0;
    if (unheld) {
      no_holder = true;
    } else if (key_ok) {
      // (no pointer to the register copy n0: a pointer that may address private memory puts n0 in
      // scratch -- 40 B stored and reloaded per query, ~40 % of this kernel's HBM writes)
      NSlot v = n0;
      bool found = n0.key == key;
      if (!found && n0.key != EMPTY64) {
        const NSlot* sl = nmap_slot(s, key, hash_next(ni, s.nmap_n));
        if (sl) {
          v = *sl;
          found = true;
        }
      }
      if (found) {
        node = v.node;
        rb = v.beg;
        rl = v.len;
        rsig = v.sig;
        nfl = (uint32_t)(v.pad1 & 0xFFu);
      }
    }
    if (!sid) {
      uint32_t sn = nmap_find(s, x.t.sns, x.t.srel, x.t.sobj);
      subj = sn == NONE ? NONE : (SET_BIT | sn);
    }
    int32_t d = x.max_depth;
    if (d <= 0 || global < d) d = global;  // engine.go:68-70
    const uint8_t rf = relflag(s, x.t.ns, x.t.rel);
    if (node == NONE) {
      // a materialised union relation without a node for this object: none of its components has a
      // node either (the node exists as soon as one does), so every branch is NotMember
      const bool virt = s.virt && x.t.ns < s.n_ns && x.t.rel < s.n_rel && s.virt[(size_t)x.t.ns * s.n_rel + x.t.rel];
      route = rf && !virt ? ROUTE_GENERAL : ROUTE_DONE;
    } else {
      // the node's flags ride in its node-map slot (a random nflags read per query otherwise)
      bool impure = s.nflags && (nfl & NF_IMPURE);
      route = impure ? ROUTE_GENERAL : ROUTE_LIGHT;
    }
    bool member = false;
    if (route == ROUTE_LIGHT) {
      // the root's checkDirect(D-1) (D >= 1 always) is thread-parallel here: a direct tuple or a
      // depth that cannot reach any child (D < 2) finishes the query before the wave tier.  The
      // row signature in the node-map slot rules out most misses without touching dset.
      // an unset holder bit rules the probe out as well (the exact tuple would make subj a holder)
      const bool nobit = use_bits && !((hw >> (subj & 31)) & 1u);
      did_probe = subj != NONE && !nobit && sig_maybe(rsig, subj_sig(subj));
      member = did_probe && dset_probe(s, node, subj);
      if (member || d < 2 || rl == 0) route = ROUTE_DONE;
      // a subject that no row holds cannot be reached from any root (checkDirect never hits)
      if (route == ROUTE_LIGHT && no_holder_filter) {
        const uint32_t cnt = use_bits ? ((hw >> (subj & 31)) & 1u)
                             : want_h ? (h0.key == subj ? h0.count
                                                        : (h0.key == NONE ? 0u : holders_find(s, subj).y))
                                      : holders_find(s, subj).y;
        if (cnt == 0) {
          route = ROUTE_DONE;
          no_holder = true;
        }
      }
    }
    // rq is read only through the tier lists, so finished queries skip it (their 24 B never leave the CU)
    if (route == ROUTE_GENERAL || (route == ROUTE_LIGHT && !lq_list)) rq[i] = RQuery{node, subj, d, route, rb, rl};
    lq = LQuery{i, node, subj, d, rb, rl};
    // every result starts as NotMember / no error (coalesced here): the tiers after this one store
    // only what differs (k_stream2 writes IsMember bytes only)
    out[i] = member ? KG_IS_MEMBER : KG_NOT_MEMBER;
    if (err) err[i] = KG_ERR_NONE;
  }
  {
    const int idx[2] = {ST_PROBES, ST_NOHOLD};
    const unsigned long long v[2] = {(valid && did_probe) ? 1ull : 0ull, no_holder ? 1ull : 0ull};
    block_stats<2>(ctl, idx, v);
  }
  // light list: 8 shards of capacity n (shard = blockIdx & 7), dequeued by k_light per XCD
  const uint32_t h = blockIdx.x & 7;
  if (lq_list && big_len) {
    // work order for the stream tier (kg_snapshot_tune "stream_order"): queries whose root row has >=
    // big_len set edges and depth >= big_depth fill each shard from the front, the rest from the back,
    // and waves dequeue front-first -- the likely-long walks start early instead of holding the
    // launch's tail
    const bool big = lq.len >= big_len && lq.depth >= big_depth;
    LQuery* const sh = lq_list + (size_t)h * lq_cap;
    block_append_lq(valid && route == ROUTE_LIGHT && big, lq, sh, &ctl->light8[h * 32]);
    block_append_lq(valid && route == ROUTE_LIGHT && !big, lq, sh, &ctl->light8[h * 32 + 16], lq_cap);
  } else if (lq_list)
    block_append_lq(valid && route == ROUTE_LIGHT, lq, lq_list + (size_t)h * lq_cap, &ctl->light8[h * 32]);
  else block_append(valid && route == ROUTE_LIGHT, i, light_list + (size_t)h * n, &ctl->light8[h * 32]);
  block_append(valid && route == ROUTE_GENERAL, i, gen_list, &ctl->gen_count);
}

// ------------------------------------------------------------------ k_light
constexpr int LWAVES = 4;  // waves per workgroup (256 threads)

// LDS of one light group (W lanes = one query): visited hash of EXPANDED nodes and the BFS list
// with inlined rows.  Nodes of the last level that can still be probed (rest depth 1) are probed
// on discovery and never stored, so the list only holds nodes that will be expanded.
template <int W, int VLOG2, int LIST>
struct LightLds {
  static constexpr int VIS = 1 << VLOG2;
  uint32_t vis[VIS];
  uint32_t node[LIST];
  uint32_t beg[LIST];
  uint32_t len[LIST];
  uint32_t pref[W];
};

// Bounded LDS hash insert.  The list cap keeps the table <= ~63% full (each step adds at most W
// before the cap check), so the bound is a safety net: a full table reports "fresh" and the
// caller's cap check turns the query into an overflow instead of spinning.
template <int VLOG2>
__device__ __forceinline__ bool lx_insert(uint32_t* vis, uint32_t key) {
  constexpr uint32_t VIS = 1u << VLOG2;
  uint32_t h = (key * 2654435761u) >> (32 - VLOG2);
  for (uint32_t p = 0; p < VIS; p++) {
    uint32_t old = atomicCAS(&vis[h], NONE, key);
    if (old == NONE) return true;
    if (old == key) return false;
    h = (h + 1) & (VIS - 1);
  }
  return true;
}

// Lane-group primitives: a wave64 holds 64/W independent groups of W lanes.
template <int W>
struct Group {
  int lane, gl, gb;  // wave lane, lane within the group, first wave lane of the group
  __device__ __forceinline__ Group() : lane(lane_id()), gl(lane_id() & (W - 1)), gb(lane_id() & ~(W - 1)) {}
  __device__ __forceinline__ uint64_t ballot(bool p) const {
    const uint64_t m = __ballot(p);
    return W == 64 ? m : (m >> gb) & ((1ull << W) - 1);
  }
  __device__ __forceinline__ uint32_t below(uint64_t m) const { return __popcll(m & ((1ull << gl) - 1)); }
  __device__ __forceinline__ uint32_t excl_scan(uint32_t x, uint32_t* total) const {
    uint32_t v = x;
#pragma unroll
    for (int off = 1; off < W; off <<= 1) {
      const uint32_t y = __shfl_up(v, off, W);
      if (gl >= off) v += y;
    }
    *total = __shfl(v, W - 1, W);
    return v - x;
  }
};

// One query, one group of W lanes.  Level k (rest depth d = D-k >= 2) holds the nodes to expand:
// every one of them was already probed (checkDirect at d-1) when it was discovered.  Children
// discovered in one W-edge step are probed in the NEXT step, together with that step's row loads
// (adjx: children + their own rows inline), so each step is one HBM round trip.
// Returns BFS_M / BFS_N / BFS_OVERFLOW.
template <int W, int VLOG2, int LIST>
__device__ __forceinline__ int light_query(const DevSnap& s, LightLds<W, VLOG2, LIST>& L, const Group<W>& g,
                                           const RQuery& q, BfsStats& bs) {
  constexpr int VIS = 1 << VLOG2;
  for (int i = g.gl * 4; i < VIS; i += W * 4) *reinterpret_cast<uint4*>(&L.vis[i]) = make_uint4(NONE, NONE, NONE, NONE);
  // the root was probed by k_resolve (checkDirect(D-1) missed, D >= 2, non-empty row)
  __builtin_amdgcn_wave_barrier();
  if (g.gl == 0) {
    lx_insert<VLOG2>(L.vis, q.node);
    L.node[0] = q.node;
    L.beg[0] = q.beg;
    L.len[0] = q.len;
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t lvl_b = 0, lvl_e = 1, n = 1;
  const uint32_t qsig = subj_sig(q.subj);
  bool pend = false;
  uint32_t pend_node = 0;
  for (int k = 0; lvl_b < lvl_e; k++) {
    const int d = q.depth - k;     // >= 2: expand; children sit at d-1 >= 1 and get probed
    const bool keep = d - 1 >= 2;  // children will themselves be expanded -> list them
    for (uint32_t base = lvl_b; base < lvl_e; base += W) {
      const uint32_t i = base + g.gl;
      const bool valid = i < lvl_e;
      const uint32_t b = valid ? L.beg[i] : 0u;
      const uint32_t ln = valid ? L.len[i] : 0u;
      bs.rows += __popcll(g.ballot(valid));
      uint32_t total;
      const uint32_t excl = g.excl_scan(ln, &total);
      L.pref[g.gl] = excl;
      __builtin_amdgcn_wave_barrier();
      bs.edges += total;
      for (uint32_t eb = 0; eb < total; eb += W) {
        const uint32_t e = eb + g.gl;
        const bool act = e < total;
        const int own = act ? owner_search(L.pref, W, e) : 0;
        const uint32_t ob = __shfl(b, own, W);
        AdjX x{NONE, 0, 0, 0};
        if (act) x = s.adjx[ob + (e - L.pref[own])];
        const bool h = pend && dset_probe(s, pend_node, q.subj);  // previous step's children
        if (g.ballot(h)) return BFS_M;
        // children of this step: probed once per node when they will be expanded (first-mark
        // dedup), unconditionally on the last level (no visited state is kept for it)
        if (keep) {
          const bool fresh = act && lx_insert<VLOG2>(L.vis, x.node);
          const uint64_t m = g.ballot(fresh);
          const uint32_t cnt = __popcll(m);
          if (n + cnt > LIST) return BFS_OVERFLOW;  // the next tier redoes the query
          if (fresh) {
            const uint32_t at = n + g.below(m);
            L.node[at] = x.node;
            L.beg[at] = x.begin;
            L.len[at] = x.len;
          }
          n += cnt;
          pend = fresh;
        } else {
          pend = act;
        }
        pend = pend && sig_maybe(x.sig, qsig);  // the signature rules out most misses
        pend_node = x.node;
        bs.probes += __popcll(g.ballot(pend));
      }
      __builtin_amdgcn_wave_barrier();
    }
    lvl_b = lvl_e;
    lvl_e = n;
    if (!keep) break;
  }
  const bool h = pend && dset_probe(s, pend_node, q.subj);
  return g.ballot(h) ? BFS_M : BFS_N;
}

// A work list: either 8 shards (shard h = list[h*cap, h*cap + counts[32*h])) or one list of
// counts[0] entries split into 8 ranges.  Range h is drained first by workgroups of XCD label h.
struct WorkList {
  const uint32_t* list;
  const uint32_t* counts;
  uint32_t cap;
  uint32_t sharded;
  __device__ void range(uint32_t h, uint32_t& b, uint32_t& e) const {
    if (sharded) {
      b = h * cap;
      e = b + counts[h * 32];
    } else {
      const uint32_t c = counts[0];
      b = (uint32_t)((uint64_t)c * h / 8);
      e = (uint32_t)((uint64_t)c * (h + 1) / 8);
    }
  }
};

// Dequeue up to `want` consecutive work items for a wave from per-XCD heads.  Returns the first
// list position (NONE when every range is drained) and the number taken.
__device__ __forceinline__ uint32_t dequeue_n(const WorkList& wl, uint32_t* heads, uint32_t& head_sel, uint32_t head0,
                                              uint32_t want, uint32_t& got, uint32_t ranges = 8) {
  while (head_sel < head0 + ranges) {
    const uint32_t h = head_sel & 7;
    uint32_t lo, hi;
    wl.range(h, lo, hi);
    const uint32_t k = atomicAdd(&heads[h * 32], want);
    if (lo + k < hi) {
      got = min(want, hi - (lo + k));
      return lo + k;
    }
    head_sel++;
  }
  got = 0;
  return NONE;
}

// Light tiers: k_light<16,...> runs four queries per wave (most light queries touch ~10 edges);
// its overflow goes to k_light<64,...> (one query per wave, 4x the LDS), whose overflow goes to
// the workgroup tier.  The groups of a wave advance in lockstep, one query each per round.
template <int W, int VLOG2, int LIST>
__global__ __launch_bounds__(256) void k_light(DevSnap s, const RQuery* __restrict__ rq, WorkList wl,
                                               uint32_t* heads, uint8_t* __restrict__ out,
                                               uint32_t* __restrict__ err, uint32_t* next_list, uint32_t* next_count,
                                               Ctl* ctl) {
  constexpr int G = 256 / W, GW = 64 / W;  // groups per workgroup / per wave
  __shared__ LightLds<W, VLOG2, LIST> lds_all[G];
  const Group<W> g;
  LightLds<W, VLOG2, LIST>& L = lds_all[threadIdx.x / W];
  const uint32_t head0 = blockIdx.x & 7;  // XCD label (speed only, never correctness)
  uint32_t head_sel = head0;
  BfsStats bs;
  unsigned long long st_done = 0;
  for (;;) {
    uint32_t first = 0, got = 0;
    if (g.lane == 0) first = dequeue_n(wl, heads, head_sel, head0, GW, got);
    first = __shfl(first, 0, 64);
    got = __shfl(got, 0, 64);
    if (first == NONE) break;
    const uint32_t gi = g.lane / W;
    if (gi < got) {
      const uint32_t qi = wl.list[first + gi];
      const RQuery q = rq[qi];
      const int r = light_query<W, VLOG2, LIST>(s, L, g, q, bs);
      __builtin_amdgcn_wave_barrier();
      if (g.gl == 0) {
        if (r == BFS_OVERFLOW) {
          next_list[atomicAdd(next_count, 1u)] = qi;
        } else {
          out[qi] = r == BFS_M ? KG_IS_MEMBER : KG_NOT_MEMBER;
          if (err) err[qi] = KG_ERR_NONE;
          st_done++;
        }
      }
    }
  }
  // group-uniform counters: count each group once (its lane 0); the narrow tier has its own
  // counters (roofline of k_light<16>), the wide tier adds to the shared ones
  const bool lead = g.gl == 0;
  const int idx[4] = {W == 16 ? ST_LROWS : ST_ROWS, W == 16 ? ST_LEDGES : ST_EDGES, W == 16 ? ST_LPROBES : ST_PROBES,
                      ST_LIGHT};
  const unsigned long long v[4] = {lead ? bs.rows : 0ull, lead ? bs.edges : 0ull, lead ? bs.probes : 0ull, st_done};
  block_stats<4>(ctl, idx, v);
}

// ------------------------------------------------------------------ k_stream
// The stream tier: one wave runs up to Q queries at once over ONE FIFO of row entries
// (adjx begin, length, slot | generation | rest depth).  Every step takes the next 64 edges from
// the FIFO head -- whatever queries they belong to -- so lanes stay busy however small the
// queries are, and a finished query's slot is refilled at once (no lockstep rounds).
//   * per query, FIFO order is BFS order (children are appended after every entry of the
//     current level), so first-mark dedup marks each node at its shallowest depth, exactly as in
//     k_light; the visited hash of a slot holds its expanded nodes
//   * children found in one step are probed (checkDirect) in the next, together with that
//     step's adjx loads: one HBM round trip per step for both
//   * a query ends on a hit (IsMember), when it has no FIFO entry and no pending probe left
//     (NotMember), or on overflow (visited cap, FIFO full, a row longer than LONG_ROW), which
//     hands it to the next tier to be redone there
//   * a finished slot bumps its generation: its FIFO entries and pending probes become stale
constexpr uint32_t LONG_ROW = 2048;  // rows longer than this go to a wider tier
constexpr uint32_t SF_HIT = 1, SF_OVER = 2;

// 1 inserted, 0 present, -1 table full (bounded)
template <int VLOG2>
__device__ __forceinline__ int lx_insert3(uint32_t* vis, uint32_t key) {
  constexpr uint32_t VIS = 1u << VLOG2;
  uint32_t h = (key * 2654435761u) >> (32 - VLOG2);
  for (uint32_t p = 0; p < VIS; p++) {
    const uint32_t old = atomicCAS(&vis[h], NONE, key);
    if (old == NONE) return 1;
    if (old == key) return 0;
    h = (h + 1) & (VIS - 1);
  }
  return -1;
}

// Visited sets of the stream tier's slots (nodes a query has expanded), two layouts:
//   SlotVis<Q, VLOG2>   one table of 2^VLOG2 u32 keys per slot, cleared when the slot is freed;
//                       a query may expand 5/8 of its table
//   WaveVis<VLOG2, CAP> ONE table of 2^VLOG2 64-bit keys valid | generation (26) | slot (5) | node
//                       shared by the wave's slots: small queries use little, so a single query may
//                       expand up to CAP nodes as long as the live entries stay <= 5/8 of the table.
//                       Entries of a finished query (an older generation of their slot) count as
//                       free and are reclaimed by later inserts; nothing is cleared.  A reclaim can
//                       let a node be inserted twice (expanded twice: extra work, same answer), but
//                       a node is never reported present unless this query inserted it.
template <int Q, int VLOG2>
struct SlotVis {
  static constexpr uint32_t VIS = 1u << VLOG2, INS_CAP = VIS * 5 / 8;
  uint32_t vis[Q * VIS];
  __device__ void init(int lane) {
    for (int i = lane; i < Q * (int)VIS; i += 64) vis[i] = NONE;
  }
  __device__ int insert(uint32_t slot, uint32_t, uint32_t node, const uint32_t*) {
    return lx_insert3<VLOG2>(&vis[slot * VIS], node);
  }
  __device__ void release(uint32_t slot, uint32_t, int lane) {
    for (int i = lane; i < (int)VIS; i += 64) vis[slot * VIS + i] = NONE;
  }
};

template <int VLOG2, int CAP>
struct WaveVis {
  static constexpr uint32_t VT = 1u << VLOG2, INS_CAP = CAP, LIVE_CAP = VT * 5 / 8;
  unsigned long long vt[VT];
  uint32_t live;
  __device__ void init(int lane) {
    for (int i = lane; i < (int)VT; i += 64) vt[i] = 0ull;
    if (lane == 0) live = 0;
  }
  __device__ int insert(uint32_t slot, uint32_t gen, uint32_t node, const uint32_t* s_gen) {
    if (*(volatile uint32_t*)&live >= LIVE_CAP) return -1;
    const unsigned long long key =
        (1ull << 63) | ((unsigned long long)(gen & 0x3FFFFFFu) << 37) | ((unsigned long long)slot << 32) | node;
    uint32_t h = ((node ^ (slot * 0x9E3779B9u)) * 2654435761u) >> (32 - VLOG2);
    for (uint32_t p = 0; p < VT; p++) {
      unsigned long long cur = vt[h];
      for (;;) {
        if (cur == key) return 0;
        if (cur != 0ull) {  // a live entry of some slot (its generation is current): probe on
          const uint32_t es = (uint32_t)(cur >> 32) & 31u, eg = (uint32_t)(cur >> 37) & 0x3FFFFFFu;
          if (eg == (s_gen[es] & 0x3FFFFFFu)) break;
        }
        const unsigned long long old = atomicCAS(&vt[h], cur, key);
        if (old == cur) {
          atomicAdd(&live, 1u);
          return 1;
        }
        cur = old;
      }
      h = (h + 1) & (VT - 1);
    }
    return -1;
  }
  __device__ void release(uint32_t, uint32_t inserted, int lane) {
    if (lane == 0) atomicSub(&live, inserted);
  }
};

template <int Q, class Vis, int QC>
struct StreamLds {
  Vis V;
  uint32_t e_beg[QC], e_len[QC], e_meta[QC];  // meta = slot (4 | 5) | generation (12) | rest depth (16 | 15)
  uint32_t pref[64];
  uint32_t s_qi[Q], s_subj[Q], s_gen[Q], s_cnt[Q], s_ins[Q], s_flag[Q];
  uint32_t s_edg[Q];  // edges scheduled for the slot's query (per-query edge budget)
};

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan<DppOr>(v), 63);
}

template <int Q, class Vis, int QC, int CHUNK>
__global__ __launch_bounds__(256) void k_stream(DevSnap s, const RQuery* __restrict__ rq, WorkList wl,
                                                uint32_t* heads, uint8_t* __restrict__ out,
                                                uint32_t* __restrict__ err, uint32_t* next_list,
                                                uint32_t* next_count, Ctl* ctl, uint32_t ecap) {
  using Lds = StreamLds<Q, Vis, QC>;
  constexpr uint32_t INS_CAP = Vis::INS_CAP;  // expanded nodes per query
  // FIFO entry meta = slot (SB bits) | generation (12) | rest depth (DB bits)
  constexpr int SB = Q <= 16 ? 4 : 5, DB = 32 - SB - 12;
  constexpr uint32_t DMASK = (1u << DB) - 1, QMASK = Q == 32 ? 0xFFFFFFFFu : (1u << Q) - 1;
  static_assert(Q <= 32, "slots are the bits of one u32 mask");
  const uint64_t t_start = wall_clock64();
  static_assert(CHUNK <= 64, "one chunk entry per lane");
  __shared__ Lds lds_all[4];
  Lds& L = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint32_t head0 = blockIdx.x & 7;  // XCD label (speed only, never correctness)
  uint32_t head_sel = head0;
  L.V.init(lane);
  if (lane < Q) {
    L.s_gen[lane] = 0;
    L.s_flag[lane] = 0;
    L.s_cnt[lane] = 0;
    L.s_ins[lane] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;  // wave-uniform: slots holding a query
  bool drained = false;  // the work list is exhausted (the local chunk may still hold entries)
  uint32_t c_left = 0, c_pos = 0;  // wave-local chunk: entries left, next entry
  uint32_t cq_qi = 0, cq_node = 0, cq_subj = 0, cq_beg = 0, cq_len = 0;  // lane i: chunk entry i
  int32_t cq_depth = 0;
  uint32_t head = 0, tail = 0, head_off = 0;
  bool pend = false;  // per lane: a child of the previous step awaiting its probe
  uint32_t pend_node = 0, pend_slot = 0, pend_gen = 0;
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
  for (;;) {
    // ---- refill free slots (their root entries need FIFO room)
    const uint32_t freem = ~active & QMASK;
    const uint32_t want = __popc(freem);
    if (want && !drained && (tail - head) + want <= QC) {
      // the wave pulls CHUNK consecutive list entries per dequeue (one device-scope atomic on the
      // per-XCD heads per CHUNK queries) and stages their RQuery records in lanes, so a refill
      // costs shuffles instead of two dependent HBM round trips
      if (c_left == 0) {
        uint32_t got = 0, first = 0;
        if (lane == 0) first = dequeue_n(wl, heads, head_sel, head0, CHUNK, got);
        first = __shfl(first, 0, 64);
        c_left = __shfl(got, 0, 64);
        c_pos = 0;
        if (first == NONE) {
          drained = true;
        } else if ((uint32_t)lane < c_left) {  // lane i stages chunk entry i (two dependent loads per chunk)
          cq_qi = wl.list[first + lane];
          const RQuery q = rq[cq_qi];
          cq_node = q.node;
          cq_subj = q.subj;
          cq_depth = q.depth;
          cq_beg = q.beg;
          cq_len = q.len;
        }
      }
      const uint32_t got = min(want, c_left);
      if (got) {
        // lane = slot: the free slot of rank r (among free slots) takes chunk entry c_pos + r
        const uint32_t r = __popc(freem & (lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu));
        const bool mine = lane < Q && ((freem >> (lane & 31)) & 1u) && r < got;
        const int src = mine ? (int)(c_pos + r) : lane;
        const uint32_t qi = __shfl(cq_qi, src, 64), qnode = __shfl(cq_node, src, 64),
                       qsubj = __shfl(cq_subj, src, 64), qbeg = __shfl(cq_beg, src, 64),
                       qlen = __shfl(cq_len, src, 64);
        const int32_t qdepth = __shfl(cq_depth, src, 64);
        c_pos += got;
        c_left -= got;
        if (mine) {
          const uint32_t slot = lane;
          const uint32_t gen = L.s_gen[slot];
          const bool over = qdepth > (int32_t)DMASK || qlen > LONG_ROW || qlen > ecap;
          L.s_qi[slot] = qi;
          L.s_subj[slot] = qsubj;
          L.s_flag[slot] = over ? SF_OVER : 0u;
          L.s_cnt[slot] = 1;
          L.s_edg[slot] = qlen;
          L.s_ins[slot] = L.V.insert(slot, gen, qnode, L.s_gen) > 0 ? 1u : 0u;
          const uint32_t at = (tail + r) % QC;
          L.e_beg[at] = qbeg;
          L.e_len[at] = over ? 0u : qlen;
          L.e_meta[at] = (slot << (32 - SB)) | ((gen & 0xFFF) << DB) | (uint32_t)(over ? 2 : qdepth);
        }
        active |= (uint32_t)__ballot(mine);
        tail += got;
      }
    }
    if (active == 0 && ((drained && c_left == 0) || tail == head)) {
      if (drained && c_left == 0) break;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- window: up to 64 FIFO entries from the head
    const uint32_t avail = tail - head;
    uint32_t ebeg = 0, elen = 0, emeta = 0;
    bool live = false;
    if ((uint32_t)lane < avail) {
      const uint32_t at = (head + lane) % QC;
      emeta = L.e_meta[at];
      const uint32_t sl = emeta >> (32 - SB);
      live = ((active >> sl) & 1) && ((emeta >> DB) & 0xFFF) == (L.s_gen[sl] & 0xFFF) &&
             (L.s_flag[sl] & (SF_HIT | SF_OVER)) == 0;
      ebeg = L.e_beg[at];
      elen = live ? L.e_len[at] : 0u;
      if (lane == 0) {
        ebeg += head_off;
        elen = live ? elen - head_off : 0u;
      }
    }
    uint32_t total;
    const uint32_t excl = wave_excl_scan(elen, &total);
    // owner of edge e = the non-empty entry starting at or below e: entries mark their start in
    // L.pref (start position -> entry lane + 1) and a DPP max-scan spreads the marks
    L.pref[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t taken = min(total, 64u);
    if (elen > 0 && excl < taken) L.pref[excl] = (uint32_t)lane + 1;
    const bool consumed = (uint32_t)lane < avail && excl + elen <= taken;
    const uint32_t ncons = __popcll(__ballot(consumed));  // a prefix of the window
    if (consumed && live) {
      atomicSub(&L.s_cnt[emeta >> (32 - SB)], 1u);
      st_rows++;
    }
    {
      const uint32_t ex_n = (uint32_t)__builtin_amdgcn_readlane((int)excl, ncons & 63);
      if (ncons < avail && ncons < 64 && ex_n < taken) head_off = (ncons == 0 ? head_off : 0u) + (taken - ex_n);
      else if (ncons > 0) head_off = 0;
    }
    // ---- this step's edges; previous step's probes in flight together with them
    __builtin_amdgcn_wave_barrier();
    const bool act = (uint32_t)lane < taken;
    const int own = ((int)wave_incl_scan<DppMax>(L.pref[lane]) - 1) & 63;
    const uint32_t ob = __shfl(ebeg, own, 64);
    const uint32_t om = __shfl(emeta, own, 64);
    const uint32_t ox = __shfl(excl, own, 64);
    AdjX x{NONE, 0, 0, 0};
    if (act) x = s.adjx[ob + ((uint32_t)lane - ox)];
    const bool pvalid = pend && L.s_gen[pend_slot] == pend_gen;
    const bool h = pvalid && dset_probe(s, pend_node, L.s_subj[pend_slot]);
    st_probes += pvalid ? 1 : 0;
    if (h) atomicOr(&L.s_flag[pend_slot], SF_HIT);
    head += ncons;
    st_edges += (lane == 0) ? taken : 0u;
    st_steps += (lane == 0) ? 1u : 0u;
    // ---- children: kept (rest >= 2, non-empty set row) ones are marked + appended; every new
    // child is probed next step
    const uint32_t slot = om >> (32 - SB), d = om & DMASK;
    const bool keepc = act && d >= 3 && x.len > 0;
    bool fresh = false;
    if (keepc) {
      const int r = x.len > LONG_ROW ? -1 : L.V.insert(slot, L.s_gen[slot], x.node, L.s_gen);
      if (r != 0) {
        const uint32_t k = r > 0 ? atomicAdd(&L.s_ins[slot], 1u) : INS_CAP;
        if (k >= INS_CAP || atomicAdd(&L.s_edg[slot], x.len) + x.len > ecap) atomicOr(&L.s_flag[slot], SF_OVER);
        else fresh = true;
      }
    }
    const uint64_t am = __ballot(fresh);
    const uint32_t room = QC - (tail - head);
    const uint32_t pos = __popcll(am & ((1ull << lane) - 1));
    bool appended = false;
    if (fresh) {
      if (pos < room) {
        const uint32_t at = (tail + pos) % QC;
        L.e_beg[at] = x.begin;
        L.e_len[at] = x.len;
        L.e_meta[at] = (om & ~DMASK) | (d - 1);
        atomicAdd(&L.s_cnt[slot], 1u);
        appended = true;
      } else {
        atomicOr(&L.s_flag[slot], SF_OVER);
      }
    }
    tail += min((uint32_t)__popcll(am), room);
    pend = act && (keepc ? appended : true) && sig_maybe(x.sig, subj_sig(L.s_subj[slot]));
    pend_node = x.node;
    pend_slot = slot;
    pend_gen = act ? L.s_gen[slot] : 0u;
    // ---- finished queries
    const uint32_t pslots = wave_or(pend ? 1u << slot : 0u);
    __builtin_amdgcn_wave_barrier();
    bool done = false;
    if (lane < Q && ((active >> lane) & 1)) {
      const uint32_t f = L.s_flag[lane];
      if (f & SF_HIT) {
        done = true;
        out[L.s_qi[lane]] = KG_IS_MEMBER;
        if (err) err[L.s_qi[lane]] = KG_ERR_NONE;
        st_done++;
      } else if (f & SF_OVER) {
        done = true;
        next_list[atomicAdd(next_count, 1u)] = L.s_qi[lane];
      } else if (L.s_cnt[lane] == 0 && !((pslots >> lane) & 1)) {
        done = true;
        out[L.s_qi[lane]] = KG_NOT_MEMBER;
        if (err) err[L.s_qi[lane]] = KG_ERR_NONE;
        st_done++;
      }
      if (done) L.s_gen[lane]++;  // stale: its FIFO entries and pending probes
    }
    const uint32_t freed = (uint32_t)__ballot(done) & QMASK;
    if (freed) {
      active &= ~freed;
      for (uint32_t m = freed; m; m &= m - 1) {
        const uint32_t sl = __ffs(m) - 1;
        L.V.release(sl, L.s_ins[sl], lane);
      }
      if (pend && ((freed >> pend_slot) & 1)) pend = false;
    }
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long life = lane == 0 ? wall_clock64() - t_start : 0ull;
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ k_stream2 (variant 9, default)
// The stream tier cut for issue rate.  PMC on k_stream (variant 8) showed a step of 64 edges costing
// ~1,060 wave instructions, 435 of them SALU exec-mask and loop bookkeeping of divergent code (the
// CAS-probing visited table, per-lane retry loops, conditional LDS atomics) and the waves parked on
// memory only 68 % of their life: the kernel was as much issue- as latency-bound.  Same algorithm
// (one FIFO of row entries shared by 32 query slots, BFS order per query, children probed one step
// after discovery together with the next edge gathers), but:
//   * the visited set is a DIRECT-MAPPED cache of keys valid | gen | slot | node with blind writes --
//     no probing, no CAS, no retry loop.  It may forget a node (a collision evicts it), which can
//     only make a node be expanded again (extra work, same answer: expanding a node again at a
//     smaller rest depth explores a subset of what its first expansion did); it never reports a
//     node present that this query did not insert (the key holds the slot and its generation)
//   * FIFO entries are 8 bytes (row begin | len 11 | slot 5 | gen 9 | rest depth 7) and the
//     per-slot state is one word (gen | HIT | OVER): ~7 KiB of LDS per wave, 5 workgroups per CU
//     (20 waves) instead of 3 (12)
//   * the step is straight-line, predicated code: no data-dependent loops (a probe chain past the
//     first dset bucket -- rare at load <= 0.25 -- takes a wave-uniform slow path)
//   * k_resolve pre-writes every result as NotMember and every err as 0 (coalesced), so this tier
//     stores only IsMember bytes
constexpr uint32_t S2_LONG = 2047;  // longest row a FIFO entry can hold (11-bit length)
constexpr uint32_t S2_GEN = 0x1FF, S2_DMAX = 127;
constexpr uint32_t S2_HIT = 1u << 30, S2_OVER = 1u << 31;

template <int VLOG2, int QC, int EPL>
struct Stream2Lds {
  unsigned long long vt[1 << VLOG2];  // direct-mapped visited cache (0 = empty)
  uint32_t e_beg[QC], e_meta[QC];     // FIFO ring
  uint32_t pref[64 * EPL + 1];        // edge-owner marks (+1 dummy)
  uint32_t s_state[32], s_qi[32], s_subj[32], s_sig[32], s_cnt[32], s_ins[32], s_edg[32];
};

__device__ __forceinline__ uint32_t s2_meta(uint32_t len, uint32_t slot, uint32_t gen, uint32_t depth) {
  return len | (slot << 11) | ((gen & S2_GEN) << 16) | (depth << 25);
}

// checkDirect probe, first bucket inline; a chain past a full first bucket (rare at load <= 0.25)
// is walked by the lanes that need it under a wave-uniform branch.
__device__ __forceinline__ bool dset_probe_fast(const DevSnap& s, bool want, uint32_t node, uint32_t subj) {
  const uint64_t key = dset_key(node, subj);
  const uint64_t b = hash_home(key, s.dset_nb);
  bool hit = false, more = false;
  if (want) {
    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(s.dset + b * DSET_BUCKET);
    hit = a.x == key || a.y == key;
    more = !hit && a.y != EMPTY64;
  }
  if (__ballot(more)) {
    if (more) hit = dset_probe(s, node, subj);  // from the first bucket again: exact, rarely run
  }
  return hit;
}

template <int VLOG2, int QC, int CHUNK, int INS_CAP, int EPL>
__global__ __launch_bounds__(256) void k_stream2(DevSnap s, const RQuery* __restrict__ rq, WorkList wl, uint32_t* heads,
                                                 uint8_t* __restrict__ out, uint32_t* next_list, uint32_t* next_count,
                                                 Ctl* ctl, uint32_t ecap, uint32_t chunk, uint32_t ranges) {
  using Lds = Stream2Lds<VLOG2, QC, EPL>;
  constexpr uint32_t WIN = 64u * EPL;  // edges per step: EPL per lane
  constexpr uint32_t VT = 1u << VLOG2;
  static_assert(QC <= 256 && (QC & (QC - 1)) == 0, "FIFO ring of <= 256 entries (9-bit generations stay unique)");
  static_assert(CHUNK <= 64, "one chunk entry per lane");
  const uint64_t t_start = wall_clock64();
  __shared__ Lds lds_all[4];
  Lds& L = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  // XCD label: the first range this wave drains.  With ranges < 8 (stream_steal) correctness needs
  // every label in the grid (the launch keeps grid >= 8), else some range is never drained.
  const uint32_t head0 = blockIdx.x & 7;
  uint32_t head_sel = head0;
  for (uint32_t i = lane; i < VT; i += 64) L.vt[i] = 0ull;
  if (lane < 32) {
    L.s_state[lane] = 0;
    L.s_cnt[lane] = 0;
    L.s_ins[lane] = 0;
    L.s_edg[lane] = 0;
  }
  if (lane == 0) L.pref[WIN] = 0;
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;   // wave-uniform: slots holding a query
  bool drained = false;  // the work list is exhausted (the local chunk may still hold entries)
  uint32_t c_left = 0, c_pos = 0;
  uint32_t cq_qi = 0, cq_node = 0, cq_subj = 0, cq_beg = 0, cq_len = 0;
  int32_t cq_depth = 0;
  uint32_t head = 0, tail = 0, head_off = 0;
  bool pend[EPL];
  uint32_t pend_node[EPL], pend_slot[EPL], pend_gen[EPL];
#pragma unroll
  for (int hf = 0; hf < EPL; hf++) {
    pend[hf] = false;
    pend_node[hf] = pend_slot[hf] = pend_gen[hf] = 0;
  }
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
  for (;;) {
    // ---- refill free slots (their root entries need FIFO room)
    const uint32_t freem = ~active;
    const uint32_t want = __popc(freem);
    if (want && !drained && (tail - head) + want <= QC) {
      if (c_left == 0) {
        uint32_t got = 0, first = 0;
        // chunk (kg_snapshot_tune "stream_chunk", <= CHUNK): one dequeue costs three dependent
        // round trips (head atomic, list, rq), so small chunks stall the step loop (guided
        // self-scheduling toward the free-slot count measured 5.3 -> 3.2 x 10^9 checks/s)
        // ranges (kg_snapshot_tune "stream_steal"): how many XCD ranges a wave dequeues from; once
        // the list drains every wave walks them, one atomic each on 8 hot words
        if (lane == 0) first = dequeue_n(wl, heads, head_sel, head0, chunk, got, ranges);
        first = __shfl(first, 0, 64);
        c_left = __shfl(got, 0, 64);
        c_pos = 0;
        if (first == NONE) {
          drained = true;
        } else if ((uint32_t)lane < c_left) {
          cq_qi = wl.list[first + lane];
          const RQuery q = rq[cq_qi];
          cq_node = q.node;
          cq_subj = q.subj;
          cq_depth = q.depth;
          cq_beg = q.beg;
          cq_len = q.len;
        }
      }
      const uint32_t got = min(want, c_left);
      if (got) {
        const uint32_t r = __popc(freem & (lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu));
        const bool mine = lane < 32 && ((freem >> (lane & 31)) & 1u) && r < got;
        const int src = mine ? (int)(c_pos + r) : lane;
        const uint32_t qi = __shfl(cq_qi, src, 64), qnode = __shfl(cq_node, src, 64), qsubj = __shfl(cq_subj, src, 64),
                       qbeg = __shfl(cq_beg, src, 64), qlen = __shfl(cq_len, src, 64);
        const int32_t qdepth = __shfl(cq_depth, src, 64);
        c_pos += got;
        c_left -= got;
        if (mine) {
          const uint32_t slot = lane, gen = L.s_state[slot] & S2_GEN;  // freed slots hold a fresh generation
          const bool over = qdepth > (int32_t)S2_DMAX || qlen > S2_LONG || qlen > ecap;
          L.s_qi[slot] = qi;
          L.s_edg[slot] = qlen;
          L.s_subj[slot] = qsubj;
          L.s_sig[slot] = subj_sig(qsubj);
          L.s_cnt[slot] = 1;
          L.s_ins[slot] = 0;
          L.s_state[slot] = over ? (gen | S2_OVER) : gen;
          // the root counts as visited (a cycle back to it is not expanded again)
          const unsigned long long key =
              (1ull << 63) | ((unsigned long long)gen << 37) | ((unsigned long long)slot << 32) | qnode;
          L.vt[((qnode * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (gen * 0xC2B2AE3Du)) >> (32 - VLOG2)] = key;
          const uint32_t at = (tail + r) & (QC - 1);
          L.e_beg[at] = qbeg;
          L.e_meta[at] = s2_meta(over ? 0u : qlen, slot, gen, over ? 2u : (uint32_t)qdepth);
        }
        active |= (uint32_t)__ballot(mine);
        tail += got;
      }
    }
    if (active == 0 && ((drained && c_left == 0) || tail == head)) {
      if (drained && c_left == 0) break;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- window: up to 64 FIFO entries from the head, up to WIN edges of them
    const uint32_t avail = tail - head;
    uint32_t ebeg = 0, elen = 0, emeta = 0;
    bool live = false;
    if ((uint32_t)lane < avail) {
      const uint32_t at = (head + lane) & (QC - 1);
      emeta = L.e_meta[at];
      ebeg = L.e_beg[at];
      const uint32_t sl = (emeta >> 11) & 31u;
      const uint32_t st = L.s_state[sl];
      live = ((active >> sl) & 1u) && (st == ((emeta >> 16) & S2_GEN));  // current generation, no HIT/OVER
      elen = live ? (emeta & 0x7FFu) : 0u;
      if (lane == 0) {
        ebeg += head_off;
        elen = live ? elen - head_off : 0u;
      }
    }
    uint32_t total;
    const uint32_t excl = wave_excl_scan(elen, &total);
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) L.pref[lane + 64 * hf] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t taken = min(total, WIN);
    L.pref[(elen > 0 && excl < taken) ? excl : WIN] = (uint32_t)lane + 1;
    const bool consumed = (uint32_t)lane < avail && excl + elen <= taken;
    const uint32_t ncons = __popcll(__ballot(consumed));  // a prefix of the window
    if (consumed && live) atomicSub(&L.s_cnt[(emeta >> 11) & 31u], 1u);
    st_rows += (consumed && live) ? 1u : 0u;
    {
      const uint32_t ex_n = (uint32_t)__builtin_amdgcn_readlane((int)excl, ncons & 63);
      if (ncons < avail && ncons < 64 && ex_n < taken) head_off = (ncons == 0 ? head_off : 0u) + (taken - ex_n);
      else if (ncons > 0) head_off = 0;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- this step's edge gathers (edge lane + 64 hf of the window) and the previous step's probes,
    // all issued before any of them is waited on
    AdjX x[EPL];
    uint32_t om[EPL];
    uint32_t carry = 0;  // the last edge owner mark of the earlier part of the window
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) {
      const uint32_t m = max(wave_incl_scan<DppMax>(L.pref[lane + 64 * hf]), carry);
      if (EPL > 1) carry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
      const int own = ((int)m - 1) & 63;
      const uint32_t ob = __shfl(ebeg, own, 64);
      om[hf] = __shfl(emeta, own, 64);
      const uint32_t ox = __shfl(excl, own, 64);
      const uint32_t e = (uint32_t)lane + 64u * hf;
      x[hf] = AdjX{NONE, 0, 0, 0};
      if (e < taken) x[hf] = s.adjx[ob + (e - ox)];
    }
    bool pvalid[EPL], hit[EPL];
    uint64_t pkey[EPL];
    ulonglong2 pb[EPL];
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) {
      pvalid[hf] = pend[hf] && L.s_state[pend_slot[hf]] == pend_gen[hf];
      pkey[hf] = dset_key(pend_node[hf], L.s_subj[pend_slot[hf]]);
      pb[hf] = make_ulonglong2(EMPTY64, EMPTY64);
      if (pvalid[hf]) pb[hf] = *reinterpret_cast<const ulonglong2*>(s.dset + hash_home(pkey[hf], s.dset_nb) * DSET_BUCKET);
    }
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) {
      // checkDirect probe, first bucket; a chain past a full first bucket (rare at load <= 0.25) is
      // walked by the lanes that need it under a wave-uniform branch
      hit[hf] = pvalid[hf] && (pb[hf].x == pkey[hf] || pb[hf].y == pkey[hf]);
      const bool more = pvalid[hf] && !hit[hf] && pb[hf].y != EMPTY64;
      if (__ballot(more)) {
        if (more) hit[hf] = dset_probe(s, pend_node[hf], L.s_subj[pend_slot[hf]]);
      }
      st_probes += pvalid[hf] ? 1u : 0u;
    }
    head += ncons;
    st_edges += (lane == 0) ? taken : 0u;
    st_steps += (lane == 0) ? 1u : 0u;
    // ---- children: kept ones (rest >= 2 after the hop, non-empty set row) are marked + appended;
    // every child new to the query is probed next step.  Part hf = 0 first: FIFO order stays BFS order
    bool npend[EPL];
    uint32_t nslot[EPL], ngen[EPL];
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) {
      const bool act = (uint32_t)lane + 64u * hf < taken;
      const AdjX& xc = x[hf];
      const uint32_t slot = (om[hf] >> 11) & 31u, d = om[hf] >> 25, g = (om[hf] >> 16) & S2_GEN;
      const bool keepc = act && d >= 3 && xc.len > 0;
      const bool longrow = keepc && xc.len > S2_LONG;
      const unsigned long long key =
          (1ull << 63) | ((unsigned long long)g << 37) | ((unsigned long long)slot << 32) | xc.node;
      const uint32_t hv = ((xc.node * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (g * 0xC2B2AE3Du)) >> (32 - VLOG2);
      const unsigned long long old = keepc ? L.vt[hv] : 0ull;
      const bool fresh = keepc && !longrow && old != key;
      if (fresh) L.vt[hv] = key;
      // INS_CAP 0: no per-query cap on expanded nodes (the edge budget ecap still bounds a query),
      // which saves a returning LDS atomic on the step's dependent chain
      const uint32_t k = (INS_CAP && fresh) ? atomicAdd(&L.s_ins[slot], 1u) : 0u;
      const bool ok = fresh && (INS_CAP == 0 || k < (uint32_t)INS_CAP);
      const uint64_t am = __ballot(ok);
      const uint32_t room = QC - (tail - head);
      const uint32_t pos = __popcll(am & ((1ull << lane) - 1));
      const bool appended = ok && pos < room;
      // edge budget (kg_snapshot_tune "stream_ecap"): a query whose enqueued rows pass it goes on to
      // the backward / grid tiers instead of holding its wave's FIFO
      const bool overbudget = appended && ecap != 0xFFFFFFFFu && atomicAdd(&L.s_edg[slot], xc.len) + xc.len > ecap;
      if (appended) {
        const uint32_t at = (tail + pos) & (QC - 1);
        L.e_beg[at] = xc.begin;
        L.e_meta[at] = xc.len | (om[hf] & 0x01FFF800u) | ((d - 1) << 25);
        atomicAdd(&L.s_cnt[slot], 1u);
      }
      if (longrow || (fresh && !appended) || overbudget) atomicOr(&L.s_state[slot], S2_OVER);  // visited cap, FIFO full, budget
      tail += min((uint32_t)__popcll(am), room);
      npend[hf] = act && (keepc ? appended : true) && sig_maybe(xc.sig, L.s_sig[slot]);
      nslot[hf] = slot;
      ngen[hf] = g;
      __builtin_amdgcn_wave_barrier();
    }
    uint32_t pmask = 0;
#pragma unroll
    for (int hf = 0; hf < EPL; hf++) {
      if (hit[hf]) atomicOr(&L.s_state[pend_slot[hf]], S2_HIT);
      pend[hf] = npend[hf];
      pend_node[hf] = x[hf].node;
      pend_slot[hf] = nslot[hf];
      pend_gen[hf] = ngen[hf];
      pmask |= pend[hf] ? 1u << nslot[hf] : 0u;
    }
    // ---- finished queries
    const uint32_t pslots = wave_or(pmask);
    __builtin_amdgcn_wave_barrier();
    bool done = false;
    if (lane < 32 && ((active >> lane) & 1u)) {
      const uint32_t st = L.s_state[lane];
      if (st & S2_HIT) {
        done = true;
        out[L.s_qi[lane]] = KG_IS_MEMBER;  // NotMember was pre-written by k_resolve
        st_done++;
      } else if (st & S2_OVER) {
        done = true;
        next_list[atomicAdd(next_count, 1u)] = L.s_qi[lane];
      } else if (L.s_cnt[lane] == 0 && !((pslots >> lane) & 1u)) {
        done = true;
        st_done++;
      }
      if (done) L.s_state[lane] = ((st & S2_GEN) + 1u) & S2_GEN;  // stale: its FIFO entries and probes
    }
    const uint32_t freed = (uint32_t)__ballot(done);
    active &= ~freed;
#pragma unroll
    for (int hf = 0; hf < EPL; hf++)
      if (pend[hf] && ((freed >> pend_slot[hf]) & 1u)) pend[hf] = false;
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t_end = wall_clock64(), life = lane == 0 ? t_end - t_start : 0ull;
  block_max3(ctl, ~(unsigned long long)t_start, t_end, t_end - t_start);
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ k_stream4 (variant 15)
// k_stream2's algorithm (one FIFO of row entries shared by 32 query slots, BFS order per query, a
// direct-mapped visited cache with blind writes, children probed one step after discovery) with the
// step's dependent chain and the work distribution reworked:
//   * work comes as LQuery records (k_resolve writes the resolved query into the list itself), and a
//     dequeue is PIPELINED over steps: step t issues the head atomic, step t+1 issues the coalesced
//     record load, the records are used from step t+2 on -- both round trips hide under the steps'
//     gathers, so chunks can be small (kg_snapshot_tune "stream_chunk") and the waves finish
//     together instead of the last few running one 64-query chunk each (k_stream2's tail)
//   * per-slot bookkeeping without returning LDS atomics: a query is finished when the FIFO position
//     of its last appended entry (s_last, an atomicMax) lies behind the head -- no decrement per
//     consumed entry and no increment per append; the edge budget is an atomicAdd read once, at the
//     step's finish check (a query past it is retired in the same step)
//   * the range bounds of the 8 per-XCD list shards are read once, into lanes 0..7
//   * queries handed on write their RQuery for the next tiers (k_resolve no longer does)
constexpr uint32_t S4_CHUNK = 64;

template <int VLOG2, int QC>
struct Stream4Lds {
  unsigned long long vt[1 << VLOG2];  // direct-mapped visited cache (0 = empty)
  uint32_t e_beg[QC], e_meta[QC];     // FIFO ring
  uint32_t pref[65];                  // edge-owner marks (+1 dummy)
  uint32_t s_state[32], s_qi[32], s_subj[32], s_sig[32], s_last[32], s_edg[32];
  uint32_t s_node[32], s_depth[32], s_beg[32], s_len[32];
};

struct LqList {
  const LQuery* list;
  const uint32_t* counts;  // shard h: counts[32 h] records from list[h * cap] (the front run) and
                           // counts[32 h + 16] ending at list[(h + 1) * cap] (the back run, k_resolve)
  uint32_t cap;
};

template <int VLOG2, int QC>
__global__ __launch_bounds__(256) void k_stream4(DevSnap s, LqList wl, uint32_t* heads, uint8_t* __restrict__ out,
                                                 RQuery* __restrict__ rq, uint32_t* next_list, uint32_t* next_count,
                                                 Ctl* ctl, uint32_t ecap, uint32_t chunk, uint32_t ranges,
                                                 uint32_t tail_ecap, uint32_t big_chunk) {
  using Lds = Stream4Lds<VLOG2, QC>;
  constexpr uint32_t WIN = 64u;
  constexpr uint32_t VT = 1u << VLOG2;
  static_assert(QC <= 256 && (QC & (QC - 1)) == 0, "FIFO ring of <= 256 entries (9-bit generations stay unique)");
  const uint64_t t_start = wall_clock64();
  __shared__ Lds lds_all[4];
  Lds& L = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  // XCD label: the first range this wave drains (the launch keeps grid >= 8 so every range is drained)
  const uint32_t head0 = blockIdx.x & 7;
  uint32_t head_sel = head0;
  for (uint32_t i = lane; i < VT; i += 64) L.vt[i] = 0ull;
  if (lane < 32) {
    L.s_state[lane] = 0;
    L.s_last[lane] = 0;
    L.s_edg[lane] = 0;
  }
  if (lane == 0) L.pref[WIN] = 0;
  // shard sizes, final before this kernel starts: lanes 0..7
  const uint32_t shard_b = lane < 8 ? wl.counts[lane * 32] : 0u;  // front run (all of it without an order)
  const uint32_t shard_n = lane < 8 ? shard_b + wl.counts[lane * 32 + 16] : 0u;
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;  // wave-uniform: slots holding a query
  // dequeue pipeline (wave-uniform state): 0 idle, 1 head atomic in flight (tk, lane 0), 2 records staged
  uint32_t pf = 0, tk = 0, st_got = 0;
  uint32_t claim = chunk, last_k = 0;  // size of the claim in flight; end of this wave's last claim in the shard
  bool exhausted = false;  // every range this wave drains is empty
  LQuery sq{};             // staged chunk (lane k: record k)
  uint32_t c_left = 0, c_pos = 0;
  LQuery cq{};             // current chunk
  uint32_t head = 0, tail = 0, head_off = 0;
  bool pend = false;
  uint32_t pend_node = 0, pend_slot = 0, pend_gen = 0;
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
  for (;;) {
    // ---- the staged chunk (loaded at least one step ago) becomes the current one
    if (c_left == 0 && pf == 2) {
      cq = sq;
      c_left = st_got;
      c_pos = 0;
      pf = 0;
    }
    // ---- refill free slots (their root entries need FIFO room)
    const uint32_t freem = ~active;
    const uint32_t want = __popc(freem);
    const uint32_t got = min(want, c_left);
    if (got && (tail - head) + got <= QC) {
      const uint32_t r = __popc(freem & (lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu));
      const bool mine = lane < 32 && ((freem >> (lane & 31)) & 1u) && r < got;
      const int src = mine ? (int)(c_pos + r) : lane;
      const uint32_t qi = __shfl(cq.qi, src, 64), qnode = __shfl(cq.node, src, 64), qsubj = __shfl(cq.subj, src, 64),
                     qbeg = __shfl(cq.beg, src, 64), qlen = __shfl(cq.len, src, 64);
      const int32_t qdepth = __shfl(cq.depth, src, 64);
      c_pos += got;
      c_left -= got;
      if (mine) {
        const uint32_t slot = lane, gen = L.s_state[slot] & S2_GEN;  // freed slots hold a fresh generation
        const bool over = qdepth > (int32_t)S2_DMAX || qlen > S2_LONG || qlen > ecap;
        const uint32_t at = tail + r;
        L.s_qi[slot] = qi;
        L.s_subj[slot] = qsubj;
        L.s_sig[slot] = subj_sig(qsubj);
        L.s_node[slot] = qnode;
        L.s_depth[slot] = (uint32_t)qdepth;
        L.s_beg[slot] = qbeg;
        L.s_len[slot] = qlen;
        L.s_edg[slot] = qlen;
        L.s_last[slot] = at;
        L.s_state[slot] = over ? (gen | S2_OVER) : gen;
        // the root counts as visited (a cycle back to it is not expanded again)
        const unsigned long long key =
            (1ull << 63) | ((unsigned long long)gen << 37) | ((unsigned long long)slot << 32) | qnode;
        L.vt[((qnode * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (gen * 0xC2B2AE3Du)) >> (32 - VLOG2)] = key;
        L.e_beg[at & (QC - 1)] = qbeg;
        L.e_meta[at & (QC - 1)] = s2_meta(over ? 0u : qlen, slot, gen, over ? 2u : (uint32_t)qdepth);
      }
      active |= (uint32_t)__ballot(mine);
      tail += got;
    }
    // ---- advance the dequeue pipeline (nothing here is waited for in this step)
    if (pf == 1) {
      const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);  // issued a step ago
      const uint32_t h = head_sel & 7;
      const uint32_t lo = h * wl.cap, hi = lo + (uint32_t)__builtin_amdgcn_readlane((int)shard_n, (int)h);
      if (lo + k < hi) {
        st_got = min(claim, hi - (lo + k));
        last_k = k + claim;
        // position p of the shard's order: the front run, then the back run at the shard's end
        const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)shard_b, (int)h), p = k + (uint32_t)lane;
        if ((uint32_t)lane < st_got) sq = wl.list[lo + (p < nb ? p : p + (wl.cap - (hi - lo)))];
        pf = 2;
      } else {
        pf = 0;
        last_k = 0;
        if (++head_sel >= head0 + ranges) exhausted = true;
      }
    }
    if (pf == 0 && !exhausted) {
      // the front run of a shard (stream_order) is dequeued in small claims: a 64-query chunk of it
      // would put 64 long walks on one wave
      const uint32_t nbh = (uint32_t)__builtin_amdgcn_readlane((int)shard_b, (int)(head_sel & 7));
      claim = (big_chunk && last_k < nbh) ? big_chunk : chunk;
      if (lane == 0) tk = atomicAdd(&heads[(head_sel & 7) * 32], claim);
      pf = 1;
    }
    if (active == 0) {
      if (exhausted && pf == 0 && c_left == 0) break;
      head = tail;  // no query holds the FIFO: whatever is left in it is stale
      head_off = 0;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- window: up to 64 FIFO entries from the head, up to WIN edges of them
    // Every load of the step below is unconditional (lanes without work read a valid dummy slot) and
    // predicated afterwards: a load inside a branch whose value is merged after the branch makes the
    // compiler wait for it inside the branch -- k_stream2's gather was waited for before its probe
    // load was even issued, two serial memory round trips per step.
    const uint32_t avail = tail - head;
    const uint32_t at0 = (head + lane) & (QC - 1);
    uint32_t emeta = L.e_meta[at0], ebeg = L.e_beg[at0];
    const uint32_t sl0 = (emeta >> 11) & 31u;
    const uint32_t st0 = L.s_state[sl0];
    // the previous step's children: probe validity and keys (LDS reads independent of the gathers)
    const uint32_t pst = L.s_state[pend_slot], psubj = L.s_subj[pend_slot];
    const bool inwin = (uint32_t)lane < avail;
    const bool live = inwin && ((active >> sl0) & 1u) && (st0 == ((emeta >> 16) & S2_GEN));  // no HIT/OVER
    uint32_t elen = live ? (emeta & 0x7FFu) : 0u;
    if (lane == 0) {
      ebeg += head_off;
      elen = live ? elen - head_off : 0u;
    }
    if (!inwin) emeta = 0;
    const bool pvalid = pend && pst == pend_gen;
    const uint64_t pkey = dset_key(pend_node, psubj);
    uint32_t total;
    const uint32_t excl = wave_excl_scan(elen, &total);
    L.pref[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t taken = min(total, WIN);
    L.pref[(elen > 0 && excl < taken) ? excl : WIN] = (uint32_t)lane + 1;
    const bool consumed = (uint32_t)lane < avail && excl + elen <= taken;
    const uint32_t ncons = __popcll(__ballot(consumed));  // a prefix of the window
    st_rows += (consumed && live) ? 1u : 0u;
    {
      const uint32_t ex_n = (uint32_t)__builtin_amdgcn_readlane((int)excl, ncons & 63);
      if (ncons < avail && ncons < 64 && ex_n < taken) head_off = (ncons == 0 ? head_off : 0u) + (taken - ex_n);
      else if (ncons > 0) head_off = 0;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- this step's edge gathers and the previous step's probes, all issued before any wait
    const uint32_t m = wave_incl_scan<DppMax>(L.pref[lane]);
    const int own = ((int)m - 1) & 63;
    const uint32_t ob = __shfl(ebeg, own, 64);
    const uint32_t om = __shfl(emeta, own, 64);
    const uint32_t ox = __shfl(excl, own, 64);
    const bool act = (uint32_t)lane < taken;
    const AdjX x = s.adjx[act ? ob + ((uint32_t)lane - ox) : 0u];  // adjx[0] exists (n_set_edges + 1)
    const ulonglong2 pb =
        *reinterpret_cast<const ulonglong2*>(s.dset + (pvalid ? hash_home(pkey, s.dset_nb) : 0ull) * DSET_BUCKET);
    const uint32_t slot = (om >> 11) & 31u, d = om >> 25, g = (om >> 16) & S2_GEN;
    const uint32_t ssig = L.s_sig[slot];  // LDS, under the gathers' latency
    head += ncons;
    st_edges += (lane == 0) ? taken : 0u;
    st_steps += (lane == 0) ? 1u : 0u;
    // checkDirect probe, first bucket; a chain past a full first bucket (rare at load <= 0.25) is
    // walked by the lanes that need it under a wave-uniform branch
    bool hit = pvalid && (pb.x == pkey || pb.y == pkey);
    {
      const bool more = pvalid && !hit && pb.y != EMPTY64;
      if (__ballot(more)) {
        if (more) hit = dset_probe(s, pend_node, (uint32_t)pkey);
      }
    }
    st_probes += pvalid ? 1u : 0u;
    // ---- children: kept ones (rest >= 2 after the hop, non-empty set row) are marked + appended;
    // every child new to the query is probed next step
    const bool keepc = act && d >= 3 && x.len > 0;  // x of an inactive lane is adjx[0]: never used
    const bool longrow = keepc && x.len > S2_LONG;
    const unsigned long long key =
        (1ull << 63) | ((unsigned long long)g << 37) | ((unsigned long long)slot << 32) | x.node;
    const uint32_t hv = ((x.node * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (g * 0xC2B2AE3Du)) >> (32 - VLOG2);
    const unsigned long long old = keepc ? L.vt[hv] : 0ull;
    const bool fresh = keepc && !longrow && old != key;
    if (fresh) L.vt[hv] = key;
    const uint64_t am = __ballot(fresh);
    const uint32_t room = QC - (tail - head);
    const uint32_t pos = __popcll(am & ((1ull << lane) - 1));
    const bool appended = fresh && pos < room;
    if (appended) {
      const uint32_t at = tail + pos;
      L.e_beg[at & (QC - 1)] = x.begin;
      L.e_meta[at & (QC - 1)] = x.len | (om & 0x01FFF800u) | ((d - 1) << 25);
      atomicMax(&L.s_last[slot], at);   // no return: read at the finish check
      atomicAdd(&L.s_edg[slot], x.len);  // edge budget, likewise
    }
    if (longrow || (fresh && !appended)) atomicOr(&L.s_state[slot], S2_OVER);  // row too long / FIFO full
    tail += min((uint32_t)__popcll(am), room);
    if (hit) atomicOr(&L.s_state[pend_slot], S2_HIT);
    pend = act && (keepc ? appended : true) && sig_maybe(x.sig, ssig);
    pend_node = x.node;
    pend_slot = slot;
    pend_gen = g;
    const uint32_t pslots = wave_or(pend ? 1u << slot : 0u);
    __builtin_amdgcn_wave_barrier();
    // ---- finished queries
    bool done = false;
    if (lane < 32 && ((active >> lane) & 1u)) {
      const uint32_t st = L.s_state[lane];
      const uint32_t last = L.s_last[lane], edg = L.s_edg[lane];
      const uint32_t qi = L.s_qi[lane];
      if (st & S2_HIT) {
        done = true;
        out[qi] = KG_IS_MEMBER;  // NotMember was pre-written by k_resolve
        st_done++;
      } else if ((st & S2_OVER) || (ecap != 0xFFFFFFFFu && edg > ecap) ||
                   (tail_ecap && exhausted && pf == 0 && c_left == 0 && edg > tail_ecap)) {
        // (the list is drained and this wave holds only its last queries: one past the tail budget
        // goes to the next tier now instead of keeping the launch open -- the tail waves set the
        // launch's length, kg_snapshot_tune "stream_tail_ecap")
        done = true;
        // the next tiers read the query by index
        rq[qi] = RQuery{L.s_node[lane], L.s_subj[lane], (int32_t)L.s_depth[lane], ROUTE_LIGHT, L.s_beg[lane],
                        L.s_len[lane]};
        next_list[atomicAdd(next_count, 1u)] = qi;
      } else if ((int32_t)(last - head) < 0 && !((pslots >> lane) & 1u)) {
        done = true;  // every entry consumed, no probe pending: NotMember (pre-written)
        st_done++;
      }
      if (done) L.s_state[lane] = ((st & S2_GEN) + 1u) & S2_GEN;  // stale: its FIFO entries and probes
    }
    const uint32_t freed = (uint32_t)__ballot(done);
    active &= ~freed;
    if (pend && ((freed >> pend_slot) & 1u)) pend = false;
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t_end = wall_clock64(), life = lane == 0 ? t_end - t_start : 0ull;
  block_max3(ctl, ~(unsigned long long)t_start, t_end, t_end - t_start);
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ k_stream5 (variant 16)
// k_stream4 with two independent FIFO engines per wave, interleaved: engine e owns slots
// [16e, 16e + 16) and its own ring of QE entries.  Each half-iteration refills and windows one
// engine and issues its gathers and probes, then processes the OTHER engine's step, whose loads were
// issued a half-iteration earlier -- so one engine's LDS / VALU bookkeeping runs under the other's
// memory round trip, and a wave has up to two steps' loads in flight instead of one.  Per engine the
// step is k_stream4's exactly (window of up to 64 edges from the ring head, children appended in
// order, probes one step after discovery, blind-write visited cache keyed by slot + generation --
// shared by both engines, slot ids are distinct), so per query the FIFO is BFS order.
template <int VLOG2, int QE>
struct Stream5Lds {
  unsigned long long vt[1 << VLOG2];
  uint32_t e_beg[2][QE], e_meta[2][QE];
  uint32_t pref[65];
  uint32_t s_state[32], s_qi[32], s_subj[32], s_sig[32], s_last[32], s_edg[32];
  uint32_t s_node[32], s_depth[32], s_beg[32], s_len[32];
};

template <int VLOG2, int QE>
__global__ __launch_bounds__(256) void k_stream5(DevSnap s, LqList wl, uint32_t* heads, uint8_t* __restrict__ out,
                                                 RQuery* __restrict__ rq, uint32_t* next_list, uint32_t* next_count,
                                                 Ctl* ctl, uint32_t ecap, uint32_t chunk, uint32_t ranges) {
  using Lds = Stream5Lds<VLOG2, QE>;
  constexpr uint32_t WIN = 64u;
  constexpr uint32_t VT = 1u << VLOG2;
  static_assert(QE <= 256 && (QE & (QE - 1)) == 0, "ring of <= 256 entries (9-bit generations stay unique)");
  const uint64_t t_start = wall_clock64();
  __shared__ Lds lds_all[4];
  Lds& L = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint32_t head0 = blockIdx.x & 7;  // XCD label (the launch keeps grid >= 8)
  uint32_t head_sel = head0;
  for (uint32_t i = lane; i < VT; i += 64) L.vt[i] = 0ull;
  if (lane < 32) {
    L.s_state[lane] = 0;
    L.s_last[lane] = 0;
    L.s_edg[lane] = 0;
  }
  if (lane == 0) L.pref[WIN] = 0;
  const uint32_t shard_b = lane < 8 ? wl.counts[lane * 32] : 0u;  // front run (all of it without an order)
  const uint32_t shard_n = lane < 8 ? shard_b + wl.counts[lane * 32 + 16] : 0u;
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;  // wave-uniform: slots holding a query (engine e: bits [16e, 16e + 16))
  uint32_t pf = 0, tk = 0, st_got = 0;
  bool exhausted = false;
  LQuery sq{};
  uint32_t c_left = 0, c_pos = 0;
  LQuery cq{};
  // per engine (index a compile-time constant after unrolling: registers)
  uint32_t head[2] = {0, 0}, tail[2] = {0, 0}, head_off[2] = {0, 0};
  bool pend[2] = {false, false};
  uint32_t pend_node[2] = {0, 0}, pend_slot[2] = {0, 0}, pend_gen[2] = {0, 0};
  // a step's issued loads and what processing them needs
  AdjX xs[2];
  ulonglong2 pbs[2];
  bool act_s[2] = {false, false}, pvalid_s[2] = {false, false};
  uint32_t om_s[2] = {0, 0}, ssig_s[2] = {0, 0}, pnode_s[2] = {0, 0}, pslot_s[2] = {0, 0};
  uint64_t pkey_s[2] = {0, 0};
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
  for (;;) {
    // ---- the staged chunk becomes the current one; the dequeue pipeline advances (as k_stream4)
    if (c_left == 0 && pf == 2) {
      cq = sq;
      c_left = st_got;
      c_pos = 0;
      pf = 0;
    }
    if (pf == 1) {
      const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
      const uint32_t h = head_sel & 7;
      const uint32_t lo = h * wl.cap, hi = lo + (uint32_t)__builtin_amdgcn_readlane((int)shard_n, (int)h);
      if (lo + k < hi) {
        st_got = min(chunk, hi - (lo + k));
        // position p of the shard's order: the front run, then the back run at the shard's end
        const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)shard_b, (int)h), p = k + (uint32_t)lane;
        if ((uint32_t)lane < st_got) sq = wl.list[lo + (p < nb ? p : p + (wl.cap - (hi - lo)))];
        pf = 2;
      } else {
        pf = 0;
        if (++head_sel >= head0 + ranges) exhausted = true;
      }
    }
    if (pf == 0 && !exhausted) {
      if (lane == 0) tk = atomicAdd(&heads[(head_sel & 7) * 32], chunk);
      pf = 1;
    }
    if (active == 0 && exhausted && pf == 0 && c_left == 0 &&
        !__ballot(act_s[0] || act_s[1] || pvalid_s[0] || pvalid_s[1] || pend[0] || pend[1]))
      break;  // every wave reaches this: no slot, no step in flight, nothing left to dequeue
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const uint32_t emask = 0xFFFFu << (16 * e);
      // ---- refill engine e's free slots (their root entries need ring room)
      {
        const uint32_t freem = ~active & emask;
        const uint32_t got = min((uint32_t)__popc(freem), c_left);
        if (got && (tail[e] - head[e]) + got <= QE) {
          const uint32_t r = __popc(freem & (lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu));
          const bool mine = lane < 32 && ((freem >> (lane & 31)) & 1u) && r < got;
          const int src = mine ? (int)(c_pos + r) : lane;
          const uint32_t qi = __shfl(cq.qi, src, 64), qnode = __shfl(cq.node, src, 64),
                         qsubj = __shfl(cq.subj, src, 64), qbeg = __shfl(cq.beg, src, 64),
                         qlen = __shfl(cq.len, src, 64);
          const int32_t qdepth = __shfl(cq.depth, src, 64);
          c_pos += got;
          c_left -= got;
          if (mine) {
            const uint32_t slot = lane, gen = L.s_state[slot] & S2_GEN;
            const bool over = qdepth > (int32_t)S2_DMAX || qlen > S2_LONG || qlen > ecap;
            const uint32_t at = tail[e] + r;
            L.s_qi[slot] = qi;
            L.s_subj[slot] = qsubj;
            L.s_sig[slot] = subj_sig(qsubj);
            L.s_node[slot] = qnode;
            L.s_depth[slot] = (uint32_t)qdepth;
            L.s_beg[slot] = qbeg;
            L.s_len[slot] = qlen;
            L.s_edg[slot] = qlen;
            L.s_last[slot] = at;
            L.s_state[slot] = over ? (gen | S2_OVER) : gen;
            const unsigned long long key =
                (1ull << 63) | ((unsigned long long)gen << 37) | ((unsigned long long)slot << 32) | qnode;
            L.vt[((qnode * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (gen * 0xC2B2AE3Du)) >> (32 - VLOG2)] = key;
            L.e_beg[e][at & (QE - 1)] = qbeg;
            L.e_meta[e][at & (QE - 1)] = s2_meta(over ? 0u : qlen, slot, gen, over ? 2u : (uint32_t)qdepth);
          }
          active |= (uint32_t)__ballot(mine);
          tail[e] += got;
        }
      }
      if ((active & emask) == 0) {  // nothing holds engine e's ring: whatever is left in it is stale
        head[e] = tail[e];
        head_off[e] = 0;
      }
      __builtin_amdgcn_wave_barrier();
      // ---- engine e: window from its ring head, then this step's gathers and the previous step's
      // probes, issued (not waited for: engine e^1's processing below runs under them)
      {
        const uint32_t avail = tail[e] - head[e];
        const uint32_t at0 = (head[e] + lane) & (QE - 1);
        uint32_t emeta = L.e_meta[e][at0], ebeg = L.e_beg[e][at0];
        const uint32_t sl0 = (emeta >> 11) & 31u;
        const uint32_t st0 = L.s_state[sl0];
        const uint32_t pst = L.s_state[pend_slot[e]], psubj = L.s_subj[pend_slot[e]];
        const bool inwin = (uint32_t)lane < avail;
        const bool live = inwin && ((active >> sl0) & 1u) && (st0 == ((emeta >> 16) & S2_GEN));
        uint32_t elen = live ? (emeta & 0x7FFu) : 0u;
        if (lane == 0) {
          ebeg += head_off[e];
          elen = live ? elen - head_off[e] : 0u;
        }
        if (!inwin) emeta = 0;
        const bool pvalid = pend[e] && pst == pend_gen[e];
        const uint64_t pkey = dset_key(pend_node[e], psubj);
        uint32_t total;
        const uint32_t excl = wave_excl_scan(elen, &total);
        L.pref[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        const uint32_t taken = min(total, WIN);
        L.pref[(elen > 0 && excl < taken) ? excl : WIN] = (uint32_t)lane + 1;
        const bool consumed = (uint32_t)lane < avail && excl + elen <= taken;
        const uint32_t ncons = __popcll(__ballot(consumed));
        st_rows += (consumed && live) ? 1u : 0u;
        {
          const uint32_t ex_n = (uint32_t)__builtin_amdgcn_readlane((int)excl, ncons & 63);
          if (ncons < avail && ncons < 64 && ex_n < taken) head_off[e] = (ncons == 0 ? head_off[e] : 0u) + (taken - ex_n);
          else if (ncons > 0) head_off[e] = 0;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t m = wave_incl_scan<DppMax>(L.pref[lane]);
        const int own = ((int)m - 1) & 63;
        const uint32_t ob = __shfl(ebeg, own, 64);
        const uint32_t om = __shfl(emeta, own, 64);
        const uint32_t ox = __shfl(excl, own, 64);
        const bool act = (uint32_t)lane < taken;
        xs[e] = s.adjx[act ? ob + ((uint32_t)lane - ox) : 0u];  // adjx[0] exists
        pbs[e] = *reinterpret_cast<const ulonglong2*>(s.dset + (pvalid ? hash_home(pkey, s.dset_nb) : 0ull) * DSET_BUCKET);
        act_s[e] = act;
        pvalid_s[e] = pvalid;
        om_s[e] = om;
        ssig_s[e] = L.s_sig[(om >> 11) & 31u];
        pkey_s[e] = pkey;
        pnode_s[e] = pend_node[e];
        pslot_s[e] = pend_slot[e];
        pend[e] = false;  // the probes now in flight are this step's; processing sets the next ones
        head[e] += ncons;
        st_edges += (lane == 0) ? taken : 0u;
        st_steps += (lane == 0 && total) ? 1u : 0u;
      }
      __builtin_amdgcn_wave_barrier();
      // ---- engine f = e^1: its step's loads (issued a half-iteration ago) are processed
      {
        const int f = 1 - e;
        const AdjX x = xs[f];
        const ulonglong2 pb = pbs[f];
        const bool act = act_s[f], pvalid = pvalid_s[f];
        const uint32_t om = om_s[f], ssig = ssig_s[f];
        const uint64_t pkey = pkey_s[f];
        const uint32_t slot = (om >> 11) & 31u, d = om >> 25, g = (om >> 16) & S2_GEN;
        bool hit = pvalid && (pb.x == pkey || pb.y == pkey);
        {
          const bool more = pvalid && !hit && pb.y != EMPTY64;
          if (__ballot(more)) {
            if (more) hit = dset_probe(s, pnode_s[f], (uint32_t)pkey);
          }
        }
        st_probes += pvalid ? 1u : 0u;
        const bool keepc = act && d >= 3 && x.len > 0;
        const bool longrow = keepc && x.len > S2_LONG;
        const unsigned long long key =
            (1ull << 63) | ((unsigned long long)g << 37) | ((unsigned long long)slot << 32) | x.node;
        const uint32_t hv = ((x.node * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (g * 0xC2B2AE3Du)) >> (32 - VLOG2);
        // (engine f's slots cannot change between its issue and this processing: the other engine's
        // half touches only its own slots, and a refill only free ones)
        const unsigned long long old = keepc ? L.vt[hv] : 0ull;
        const bool fresh = keepc && !longrow && old != key;
        if (fresh) L.vt[hv] = key;
        const uint64_t am = __ballot(fresh);
        const uint32_t room = QE - (tail[f] - head[f]);
        const uint32_t pos = __popcll(am & ((1ull << lane) - 1));
        const bool appended = fresh && pos < room;
        if (appended) {
          const uint32_t at = tail[f] + pos;
          L.e_beg[f][at & (QE - 1)] = x.begin;
          L.e_meta[f][at & (QE - 1)] = x.len | (om & 0x01FFF800u) | ((d - 1) << 25);
          atomicMax(&L.s_last[slot], at);
          atomicAdd(&L.s_edg[slot], x.len);
        }
        if (longrow || (fresh && !appended)) atomicOr(&L.s_state[slot], S2_OVER);
        tail[f] += min((uint32_t)__popcll(am), room);
        if (hit) atomicOr(&L.s_state[pslot_s[f]], S2_HIT);
        pend[f] = act && (keepc ? appended : true) && sig_maybe(x.sig, ssig);
        pend_node[f] = x.node;
        pend_slot[f] = slot;
        pend_gen[f] = g;
        act_s[f] = false;
        pvalid_s[f] = false;
        const uint32_t pslots = wave_or(pend[f] ? 1u << slot : 0u);
        __builtin_amdgcn_wave_barrier();
        // finished queries of engine f
        bool done = false;
        const uint32_t fmask = 0xFFFFu << (16 * f);
        if (lane < 32 && ((fmask >> lane) & 1u) && ((active >> lane) & 1u)) {
          const uint32_t st = L.s_state[lane];
          const uint32_t last = L.s_last[lane], edg = L.s_edg[lane];
          const uint32_t qi = L.s_qi[lane];
          if (st & S2_HIT) {
            done = true;
            out[qi] = KG_IS_MEMBER;  // NotMember was pre-written by k_resolve
            st_done++;
          } else if ((st & S2_OVER) || (ecap != 0xFFFFFFFFu && edg > ecap)) {
            done = true;
            rq[qi] = RQuery{L.s_node[lane], L.s_subj[lane], (int32_t)L.s_depth[lane], ROUTE_LIGHT, L.s_beg[lane],
                            L.s_len[lane]};
            next_list[atomicAdd(next_count, 1u)] = qi;
          } else if ((int32_t)(last - head[f]) < 0 && !((pslots >> lane) & 1u)) {
            done = true;  // every entry consumed, no probe pending: NotMember (pre-written)
            st_done++;
          }
          if (done) L.s_state[lane] = ((st & S2_GEN) + 1u) & S2_GEN;
        }
        const uint32_t freed = (uint32_t)__ballot(done);
        active &= ~freed;
        if (pend[f] && ((freed >> pend_slot[f]) & 1u)) pend[f] = false;
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  const unsigned long long t_end = wall_clock64(), life = lane == 0 ? t_end - t_start : 0ull;
  block_max3(ctl, ~(unsigned long long)t_start, t_end, t_end - t_start);
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ k_stream3 (variant 10)
// k_stream2 software-pipelined by one step.  k_stream2's step is: take a window of 64 edges at the
// FIFO head -> gather their adjx records (and probe the previous step's children) -> wait -> process
// the children; the gather latency and the child processing add up.  Here iteration i takes window
// i+1 from the FIFO and issues its gathers (with the probes of window i-1's children) BEFORE
// processing window i, whose records arrived during the previous iteration, so the LDS / DPP work
// of a step runs under the memory latency of the next.  Window i+1 is cut from the FIFO before
// window i's children are appended (so it can be shorter than 64 edges when the FIFO runs low);
// its entries' query counts are released only once their children have been processed, and every
// child is re-checked against its slot's current generation at processing time, so a query that
// finished (hit / overflow) or a slot refilled in between never sees stale appends.
template <int VLOG2, int QC, int CHUNK, int INS_CAP>
__global__ __launch_bounds__(256) void k_stream3(DevSnap s, const RQuery* __restrict__ rq, WorkList wl, uint32_t* heads,
                                                 uint8_t* __restrict__ out, uint32_t* next_list, uint32_t* next_count,
                                                 Ctl* ctl, uint32_t ecap) {
  using Lds = Stream2Lds<VLOG2, QC, 1>;
  constexpr uint32_t VT = 1u << VLOG2;
  static_assert(QC <= 256 && (QC & (QC - 1)) == 0, "FIFO ring of <= 256 entries (9-bit generations stay unique)");
  static_assert(CHUNK <= 64, "one chunk entry per lane");
  const uint64_t t_start = wall_clock64();
  __shared__ Lds lds_all[4];
  Lds& L = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint32_t head0 = blockIdx.x & 7;
  uint32_t head_sel = head0;
  for (uint32_t i = lane; i < VT; i += 64) L.vt[i] = 0ull;
  if (lane < 32) {
    L.s_state[lane] = 0;
    L.s_cnt[lane] = 0;
    L.s_ins[lane] = 0;
  }
  if (lane == 0) L.pref[64] = 0;
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;
  bool drained = false;
  uint32_t c_left = 0, c_pos = 0;
  uint32_t cq_qi = 0, cq_node = 0, cq_subj = 0, cq_beg = 0, cq_len = 0;
  int32_t cq_depth = 0;
  uint32_t head = 0, tail = 0, head_off = 0;
  bool pend = false;
  uint32_t pend_node = 0, pend_slot = 0, pend_gen = 0;
  // the probes issued last iteration, applied this one (their bucket lands during this step)
  bool q_valid = false;
  uint64_t q_key = 0;
  ulonglong2 q_a = make_ulonglong2(EMPTY64, EMPTY64);
  uint32_t q_slot = 0, q_gen = 0, q_node = 0, q_subj = 0;
  // the window gathered last iteration, processed this one: per edge lane its record and owner meta,
  // per entry lane the slot | generation whose count it releases (NONE = nothing)
  bool cur_act = false;
  AdjX cur_x{NONE, 0, 0, 0};
  uint32_t cur_om = 0, cur_dec = NONE, cur_taken = 0;
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
  for (;;) {
    // ---- refill free slots (their root entries need FIFO room)
    const uint32_t freem = ~active;
    const uint32_t want = __popc(freem);
    if (want && !drained && (tail - head) + want <= QC) {
      if (c_left == 0) {
        uint32_t got = 0, first = 0;
        if (lane == 0) first = dequeue_n(wl, heads, head_sel, head0, CHUNK, got);
        first = __shfl(first, 0, 64);
        c_left = __shfl(got, 0, 64);
        c_pos = 0;
        if (first == NONE) {
          drained = true;
        } else if ((uint32_t)lane < c_left) {
          cq_qi = wl.list[first + lane];
          const RQuery q = rq[cq_qi];
          cq_node = q.node;
          cq_subj = q.subj;
          cq_depth = q.depth;
          cq_beg = q.beg;
          cq_len = q.len;
        }
      }
      const uint32_t got = min(want, c_left);
      if (got) {
        const uint32_t r = __popc(freem & (lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu));
        const bool mine = lane < 32 && ((freem >> (lane & 31)) & 1u) && r < got;
        const int src = mine ? (int)(c_pos + r) : lane;
        const uint32_t qi = __shfl(cq_qi, src, 64), qnode = __shfl(cq_node, src, 64), qsubj = __shfl(cq_subj, src, 64),
                       qbeg = __shfl(cq_beg, src, 64), qlen = __shfl(cq_len, src, 64);
        const int32_t qdepth = __shfl(cq_depth, src, 64);
        c_pos += got;
        c_left -= got;
        if (mine) {
          const uint32_t slot = lane, gen = L.s_state[slot] & S2_GEN;
          const bool over = qdepth > (int32_t)S2_DMAX || qlen > S2_LONG || qlen > ecap;
          L.s_qi[slot] = qi;
          L.s_subj[slot] = qsubj;
          L.s_sig[slot] = subj_sig(qsubj);
          L.s_cnt[slot] = 1;
          L.s_ins[slot] = 0;
          L.s_edg[slot] = qlen;
          L.s_state[slot] = over ? (gen | S2_OVER) : gen;
          const unsigned long long key =
              (1ull << 63) | ((unsigned long long)gen << 37) | ((unsigned long long)slot << 32) | qnode;
          L.vt[((qnode * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (gen * 0xC2B2AE3Du)) >> (32 - VLOG2)] = key;
          const uint32_t at = (tail + r) & (QC - 1);
          L.e_beg[at] = qbeg;
          L.e_meta[at] = s2_meta(over ? 0u : qlen, slot, gen, over ? 2u : (uint32_t)qdepth);
        }
        active |= (uint32_t)__ballot(mine);
        tail += got;
      }
    }
    if (active == 0 && ((drained && c_left == 0) || tail == head)) {
      if (drained && c_left == 0) break;
      cur_act = false;  // nothing live: a gathered window and probes in flight can only be stale
      cur_dec = NONE;
      cur_taken = 0;
      q_valid = false;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- next window (up to 64 edges from the FIFO head): consume, then issue its gathers.  Taken
    // before the current window is processed when the FIFO already holds a full window (the gathers
    // then fly under this step's processing), else after it, so that the children appended this
    // step fill the window (k_stream2's order for that step)
    bool nxt_act = false;
    AdjX nxt_x{NONE, 0, 0, 0};
    uint32_t nxt_om = 0, nxt_dec = NONE, taken = 0;
    auto take_window = [&]() {
      const uint32_t avail = tail - head;
      uint32_t ebeg = 0, elen = 0, emeta = 0;
      bool live = false;
      if ((uint32_t)lane < avail) {
        const uint32_t at = (head + lane) & (QC - 1);
        emeta = L.e_meta[at];
        ebeg = L.e_beg[at];
        const uint32_t sl = (emeta >> 11) & 31u;
        const uint32_t st = L.s_state[sl];
        live = ((active >> sl) & 1u) && (st == ((emeta >> 16) & S2_GEN));
        elen = live ? (emeta & 0x7FFu) : 0u;
        if (lane == 0) {
          ebeg += head_off;
          elen = live ? elen - head_off : 0u;
        }
      }
      uint32_t total;
      const uint32_t excl = wave_excl_scan(elen, &total);
      L.pref[lane] = 0;
      __builtin_amdgcn_wave_barrier();
      taken = min(total, 64u);
      L.pref[(elen > 0 && excl < taken) ? excl : 64u] = (uint32_t)lane + 1;
      const bool consumed = (uint32_t)lane < avail && excl + elen <= taken;
      const uint32_t ncons = __popcll(__ballot(consumed));
      // released after processing: slot | generation << 5 (NONE = nothing)
      nxt_dec = (consumed && live) ? (((emeta >> 11) & 31u) | (((emeta >> 16) & S2_GEN) << 5)) : NONE;
      st_rows += (consumed && live) ? 1u : 0u;
      {
        const uint32_t ex_n = (uint32_t)__builtin_amdgcn_readlane((int)excl, ncons & 63);
        if (ncons < avail && ncons < 64 && ex_n < taken) head_off = (ncons == 0 ? head_off : 0u) + (taken - ex_n);
        else if (ncons > 0) head_off = 0;
      }
      __builtin_amdgcn_wave_barrier();
      nxt_act = (uint32_t)lane < taken;
      const int own = ((int)wave_incl_scan<DppMax>(L.pref[lane]) - 1) & 63;
      const uint32_t ob = __shfl(ebeg, own, 64);
      nxt_om = __shfl(emeta, own, 64);
      const uint32_t ox = __shfl(excl, own, 64);
      if (nxt_act) nxt_x = s.adjx[ob + ((uint32_t)lane - ox)];  // waited on where it is processed
      head += ncons;
      st_edges += (lane == 0) ? taken : 0u;
    };
    // a full window is waiting in the FIFO (cheap test: at least 64 entries, or the live edge count)
    bool early = (tail - head) >= 64u || cur_taken == 0;
    if (!early) {
      uint32_t el = 0;
      if ((uint32_t)lane < tail - head) {
        const uint32_t em = L.e_meta[(head + lane) & (QC - 1)];
        el = (L.s_state[(em >> 11) & 31u] == ((em >> 16) & S2_GEN)) ? (em & 0x7FFu) : 0u;
      }
      uint32_t tot;
      (void)wave_excl_scan(el, &tot);
      early = tot >= 64u + head_off;
    }
    if (early) take_window();
    st_steps += (lane == 0) ? 1u : 0u;
    // ---- the previous window's children: their first probe bucket is loaded now and evaluated next
    // iteration (in flight with the gathers above and the whole of this step)
    const bool pvalid = pend && L.s_state[pend_slot] == pend_gen;
    const uint32_t psubj = L.s_subj[pend_slot];
    const uint32_t pend_gen_issued = pend_gen, pnode_issued = pend_node, probe_slot = pend_slot;
    const uint64_t pkey = dset_key(pend_node, psubj);
    ulonglong2 pa = make_ulonglong2(EMPTY64, EMPTY64);
    if (pvalid) pa = *reinterpret_cast<const ulonglong2*>(s.dset + hash_home(pkey, s.dset_nb) * DSET_BUCKET);
    st_probes += pvalid ? 1u : 0u;
    // ---- process the current window (gathered last iteration)
    const uint32_t slot = (cur_om >> 11) & 31u, d = cur_om >> 25, g = (cur_om >> 16) & S2_GEN;
    const bool clive = cur_act && L.s_state[slot] == g;  // the query still runs in this slot
    const bool keepc = clive && d >= 3 && cur_x.len > 0;
    const bool longrow = keepc && cur_x.len > S2_LONG;
    const unsigned long long key =
        (1ull << 63) | ((unsigned long long)g << 37) | ((unsigned long long)slot << 32) | cur_x.node;
    const uint32_t hv = ((cur_x.node * 0x9E3779B1u) ^ (slot * 0x85EBCA77u) ^ (g * 0xC2B2AE3Du)) >> (32 - VLOG2);
    const unsigned long long old = keepc ? L.vt[hv] : 0ull;
    const bool fresh = keepc && !longrow && old != key;
    if (fresh) L.vt[hv] = key;
    // INS_CAP 0: the edge budget ecap bounds a query instead (as k_stream2 variant 12)
    const uint32_t k = (INS_CAP && fresh) ? atomicAdd(&L.s_ins[slot], 1u) : 0u;
    const bool ok = fresh && (INS_CAP == 0 || k < (uint32_t)INS_CAP);
    const uint64_t am = __ballot(ok);
    const uint32_t room = QC - (tail - head);
    const uint32_t pos = __popcll(am & ((1ull << lane) - 1));
    const bool appended = ok && pos < room;
    const bool overbudget =
        appended && ecap != 0xFFFFFFFFu && atomicAdd(&L.s_edg[slot], cur_x.len) + cur_x.len > ecap;
    if (appended) {
      const uint32_t at = (tail + pos) & (QC - 1);
      L.e_beg[at] = cur_x.begin;
      L.e_meta[at] = cur_x.len | (cur_om & 0x01FFF800u) | ((d - 1) << 25);
      atomicAdd(&L.s_cnt[slot], 1u);
    }
    if (longrow || (fresh && !appended) || overbudget) atomicOr(&L.s_state[slot], S2_OVER);
    tail += min((uint32_t)__popcll(am), room);
    {  // last iteration's probes: a chain past a full first bucket (rare) is walked here
      bool h = false, more = false;
      if (q_valid) {
        h = q_a.x == q_key || q_a.y == q_key;
        more = !h && q_a.y != EMPTY64;
      }
      if (__ballot(more)) {
        if (more) h = dset_probe(s, q_node, q_subj);
      }
      if (h && L.s_state[q_slot] == q_gen) atomicOr(&L.s_state[q_slot], S2_HIT);  // same query still there
    }
    // its consumed entries release their query's count now that their children are accounted for
    // (a finished / refilled slot's count is not touched: its generation moved on)
    if (cur_dec != NONE && L.s_state[cur_dec & 31u] == (cur_dec >> 5)) atomicSub(&L.s_cnt[cur_dec & 31u], 1u);
    pend = clive && (keepc ? appended : true) && sig_maybe(cur_x.sig, L.s_sig[slot]);
    pend_node = cur_x.node;
    pend_slot = slot;
    pend_gen = g;
    if (!early) take_window();  // deferred: the children appended above join this window
    // ---- finished queries
    const uint32_t pslots = wave_or((pend ? 1u << slot : 0u) | (pvalid ? 1u << probe_slot : 0u));
    __builtin_amdgcn_wave_barrier();
    bool done = false;
    if (lane < 32 && ((active >> lane) & 1u)) {
      const uint32_t st = L.s_state[lane];
      if (st & S2_HIT) {
        done = true;
        out[L.s_qi[lane]] = KG_IS_MEMBER;
        st_done++;
      } else if (st & S2_OVER) {
        done = true;
        next_list[atomicAdd(next_count, 1u)] = L.s_qi[lane];
      } else if (L.s_cnt[lane] == 0 && !((pslots >> lane) & 1u)) {
        done = true;
        st_done++;
      }
      if (done) L.s_state[lane] = ((st & S2_GEN) + 1u) & S2_GEN;
    }
    const uint32_t freed = (uint32_t)__ballot(done);
    active &= ~freed;
    if (pend && ((freed >> pend_slot) & 1u)) pend = false;
    // ---- rotate: the next window becomes the current one, this step's probes the ones to apply
    q_valid = pvalid && !((freed >> probe_slot) & 1u);
    q_key = pkey;
    q_a = pa;
    q_slot = probe_slot;
    q_gen = pend_gen_issued;
    q_node = pnode_issued;
    q_subj = psubj;
    cur_act = nxt_act;
    cur_x = nxt_x;
    cur_om = nxt_om;
    cur_dec = nxt_dec;
    cur_taken = taken;
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long life = lane == 0 ? wall_clock64() - t_start : 0ull;
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ workgroup tiers
// Queries whose visited set outgrew one wave's LDS: one 256-lane workgroup per query, same BFS.
//   k_wg<WgLds>  visited hash (8192 slots) + BFS list (4096) in LDS          ("medium")
//   k_wg<WgHbm>  visited bitmap (n_nodes bits) + BFS list in HBM per slot     ("heavy", "giant")
// Overflow forwards the query to the next tier's list.
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

struct WgLds {
  static constexpr int VLOG2 = 13;
  static constexpr uint32_t VSLOTS = 1u << VLOG2;
  static constexpr uint32_t CAP = 4096;  // hash load <= 0.5
  uint32_t* vis;
  uint32_t* lst;
  __device__ uint32_t* list() const { return lst; }
  __device__ uint64_t cap() const { return CAP; }
  __device__ void reset() {
    for (uint32_t i = threadIdx.x * 4; i < VSLOTS; i += 1024)
      *reinterpret_cast<uint4*>(&vis[i]) = make_uint4(NONE, NONE, NONE, NONE);
    __syncthreads();
  }
  // 1 = inserted, 0 = already present, -1 = table full (bounded: never spins)
  __device__ int insert(uint32_t key) {
    uint32_t h = (key * 2654435761u) >> (32 - VLOG2);
    for (uint32_t p = 0; p < VSLOTS; p++) {
      uint32_t old = atomicCAS(&vis[h], NONE, key);
      if (old == NONE) return 1;
      if (old == key) return 0;
      h = (h + 1) & (VSLOTS - 1);
    }
    return -1;
  }
  __device__ void finish(uint32_t, bool) {}
};

struct WgHbm {
  uint32_t* bm;
  uint32_t* lst;
  uint64_t capacity, words;
  __device__ uint32_t* list() const { return lst; }
  __device__ uint64_t cap() const { return capacity; }
  __device__ void reset() {}
  __device__ int insert(uint32_t key) {
    uint32_t bit = 1u << (key & 31);
    return (atomicOr(&bm[key >> 5], bit) & bit) ? 0 : 1;
  }
  // every set bit in a touched word belongs to this query; after an overflow some set bits have no
  // list entry, so the whole slot bitmap is cleared instead
  __device__ void finish(uint32_t n, bool overflow) {
    if (overflow) {
      for (uint64_t w = threadIdx.x; w < words; w += 256) bm[w] = 0u;
    } else {
      for (uint32_t i = threadIdx.x; i < n; i += 256) atomicAnd(&bm[lst[i] >> 5], 0u);
    }
    __syncthreads();
  }
};

struct WgShared {
  uint32_t qi, n, hit, over;
  uint32_t pref[256];
  uint32_t wsum[4];
};

template <class St>
__device__ void wg_run(const DevSnap& s, St& st, WgShared& sh, const RQuery* __restrict__ rq, const uint32_t* qlist,
                       uint32_t qcount, uint32_t* qhead, uint8_t* __restrict__ out, uint32_t* __restrict__ err,
                       uint32_t* next_list, uint32_t* next_count, Ctl* ctl, int st_idx) {
  const int tid = threadIdx.x;
  uint32_t* list = st.list();
  unsigned long long st_rows = 0, st_edges = 0, st_probes = 0, st_fh = 0, st_done = 0;
  for (;;) {
    if (tid == 0) sh.qi = atomicAdd(qhead, 1u);
    __syncthreads();
    const uint32_t hi = sh.qi;
    if (hi >= qcount) break;
    const uint32_t qi = qlist[hi];
    const RQuery q = rq[qi];
    st.reset();
    if (tid == 0) {
      (void)st.insert(q.node);
      list[0] = q.node;
      sh.n = 1;
      sh.over = 0;
      sh.hit = dset_probe(s, q.node, q.subj) ? 1u : 0u;  // root: checkDirect(D-1)
      st_probes++;
    }
    __syncthreads();
    // The list holds nodes to EXPAND (rest depth >= 2); children are probed when discovered and
    // kept only if they will be expanded themselves (same scheme as k_light).
    uint32_t lvl_b = 0, lvl_e = (q.depth >= 2 && !sh.hit) ? 1u : 0u;
    for (int k = 0; lvl_b < lvl_e; k++) {
      const int d = q.depth - k;     // >= 2
      const bool keep = d - 1 >= 2;
      for (uint32_t base = lvl_b; base < lvl_e; base += 256) {
        const uint32_t i = base + tid;
        const bool valid = i < lvl_e;
        const uint32_t node = valid ? list[i] : 0;
        uint64_t rb = 0, re = 0;
        if (valid) {
          rb = s.adj_off[node];
          re = s.adj_off[node + 1];
          st_rows++;
          st_fh++;
        }
        uint32_t total;
        const uint32_t excl = block_excl_scan((uint32_t)(re - rb), sh.wsum, &total);
        sh.pref[tid] = excl;
        __syncthreads();
        if (tid == 0) st_edges += total;
        for (uint32_t eb = 0; eb < total; eb += 256) {
          if (*(volatile uint32_t*)&sh.over || *(volatile uint32_t*)&sh.hit) break;  // decided: stop early
          const uint32_t e = eb + tid;
          if (e < total) {
            const int own = owner_search(sh.pref, 256, e);
            const uint32_t onode = list[base + own];  // the owner's row start lives in another wave
            const uint32_t child = s.adj[s.adj_off[onode] + (e - sh.pref[own])];
            if (keep) {
              // capacity first: once the list is full nothing more is inserted (a full LDS hash
              // would otherwise make the insert probe forever)
              const int ins = (*(volatile uint32_t*)&sh.n < st.cap()) ? st.insert(child) : -1;
              if (ins < 0) {
                sh.over = 1;
              } else if (ins > 0) {
                st_probes++;
                if (dset_probe(s, child, q.subj)) sh.hit = 1;
                const uint32_t pos = atomicAdd(&sh.n, 1u);
                if (pos < st.cap()) list[pos] = child;
                else sh.over = 1;
              }
            } else {
              st_probes++;
              if (dset_probe(s, child, q.subj)) sh.hit = 1;
            }
          }
        }
        __syncthreads();
        if (sh.hit || sh.over) break;
      }
      __syncthreads();
      if (sh.hit || sh.over || !keep) break;
      lvl_b = lvl_e;
      lvl_e = sh.n;
    }
    __syncthreads();
    const bool overflow = sh.over && !sh.hit;
    if (tid == 0) {
      if (overflow) {
        next_list[atomicAdd(next_count, 1u)] = qi;
      } else {
        out[qi] = sh.hit ? KG_IS_MEMBER : KG_NOT_MEMBER;
        if (err) err[qi] = KG_ERR_NONE;
        st_done++;
      }
    }
    st.finish((uint32_t)min((uint64_t)sh.n, st.cap()), sh.over != 0);
  }
  const int idx[5] = {ST_ROWS, ST_PROBES, ST_FHBM, ST_EDGES, st_idx};
  const unsigned long long v[5] = {st_rows, st_probes, st_idx == ST_HEAVY ? st_fh : 0ull, st_edges, st_done};
  block_stats<5>(ctl, idx, v);
}

__global__ __launch_bounds__(256) void k_medium(DevSnap s, const RQuery* __restrict__ rq, const uint32_t* qlist,
                                                const uint32_t* qcount_p, uint32_t* qhead, uint8_t* __restrict__ out,
                                                uint32_t* __restrict__ err, uint32_t* next_list, uint32_t* next_count,
                                                Ctl* ctl) {
  __shared__ uint32_t vis[WgLds::VSLOTS];
  __shared__ uint32_t lst[WgLds::CAP];
  __shared__ WgShared sh;
  WgLds st{vis, lst};
  wg_run(s, st, sh, rq, qlist, *qcount_p, qhead, out, err, next_list, next_count, ctl, ST_MEDIUM);
}

__global__ __launch_bounds__(256) void k_heavy(DevSnap s, const RQuery* __restrict__ rq, const uint32_t* qlist,
                                               const uint32_t* qcount_p, uint32_t* qhead, uint8_t* __restrict__ out,
                                               uint32_t* __restrict__ err, uint32_t* bitmaps, uint64_t words_per_slot,
                                               uint32_t* lists, uint64_t cap, uint32_t* next_list,
                                               uint32_t* next_count, Ctl* ctl) {
  __shared__ WgShared sh;
  WgHbm st{bitmaps + (uint64_t)blockIdx.x * words_per_slot, lists + (uint64_t)blockIdx.x * cap, cap, words_per_slot};
  wg_run(s, st, sh, rq, qlist, *qcount_p, qhead, out, err, next_list, next_count, ctl, ST_HEAVY);
}

// ------------------------------------------------------------------ k_back: the backward tier
// Queries that outgrew the wave tiers are first tried BACKWARDS, one workgroup per query: the
// reachability question of the rewrite-free path ("a path of <= D-1 subject-set hops from the
// root to a node whose row holds the subject") is symmetric, and in a power-law
// graph the set of nodes that can reach a rarely used subject is usually tiny while the set the
// root reaches is huge.  Level 0 = the subject's holders (hold[] via the subject hash), level j =
// their parents through reverse set-adjacency, j <= D-1; the root found at any level is a hit
// (IsMember), an exhausted search is NotMember.  A visited set that outgrows LDS hands the query
// on to the forward grid tier, which redoes it from scratch (results never depend on the tier).
// Paths from a LIGHT root only cross rewrite-free nodes (k_resolve's routing), so any backward
// path that reaches the root is a forward path of the same length.
// Two widths: k_back<64> runs one query per WAVE (visited hash 512 / list 256 in LDS, 12 queries
// in flight per CU), its overflow goes to k_back<256>, one query per WORKGROUP (8192 / 4096).
template <int W>
struct BackCfg;
// EDGES: reverse edges one query may read here.  A level that reaches hub groups reads their whole
// parent lists (up to 1e5 each) on one wave -- 28 ms for one query at 1 B tuples before this bound
// (profiles/r2o_*): such a query goes to the grid tier, which spreads its edges over the whole GPU.
template <>
struct BackCfg<64> {
  static constexpr uint32_t VLOG2 = 9, CAP = 256;  // larger caps only lengthen the tail (1024: -9 % checks/s)
  static constexpr uint32_t EDGES = 1u << 14;
};
template <>
struct BackCfg<256> {
  static constexpr uint32_t VLOG2 = 13, CAP = 4096;
  static constexpr uint32_t EDGES = 1u << 17;
};

template <int W>
struct BackLds {
  static constexpr uint32_t VSLOTS = 1u << BackCfg<W>::VLOG2, CAP = BackCfg<W>::CAP;  // hash load <= 0.5
  uint32_t vis[VSLOTS];
  uint32_t lst[CAP];
  uint32_t pref[W];
  uint64_t rb[W];
  uint32_t wsum[4];
  uint32_t qi, n, hit, over;
};

template <int W>
__device__ __forceinline__ void bk_sync() {
  if (W == 64) __builtin_amdgcn_wave_barrier();
  else __syncthreads();
}

template <int W>
__device__ __forceinline__ int bk_insert(BackLds<W>& L, uint32_t key) {
  constexpr uint32_t VSLOTS = BackLds<W>::VSLOTS;
  uint32_t h = (key * 2654435761u) >> (32 - BackCfg<W>::VLOG2);
  for (uint32_t p = 0; p < VSLOTS; p++) {
    const uint32_t old = atomicCAS(&L.vis[h], NONE, key);
    if (old == NONE) return 1;
    if (old == key) return 0;
    h = (h + 1) & (VSLOTS - 1);
  }
  return -1;
}

// Appends a newly seen node to the level list (capacity first, so the hash never fills).
template <int W>
__device__ __forceinline__ void bk_add(BackLds<W>& L, uint32_t v) {
  if (*(volatile uint32_t*)&L.n >= BackLds<W>::CAP) {
    L.over = 1;
    return;
  }
  const int ins = bk_insert(L, v);
  if (ins < 0) {
    L.over = 1;
  } else if (ins > 0) {
    const uint32_t pos = atomicAdd(&L.n, 1u);
    if (pos < BackLds<W>::CAP) L.lst[pos] = v;
    else L.over = 1;
  }
}

template <int W>
__global__ __launch_bounds__(256) void k_back(DevSnap s, const RQuery* __restrict__ rq, const uint32_t* qlist,
                                              const uint32_t* qcount_p, uint32_t* qhead, uint8_t* __restrict__ out,
                                              uint32_t* __restrict__ err, uint32_t* next_list, uint32_t* next_count,
                                              Ctl* ctl) {
  constexpr uint32_t VSLOTS = BackLds<W>::VSLOTS, CAP = BackLds<W>::CAP;
  constexpr int BU = 4;
  __shared__ BackLds<W> lds_all[256 / W];
  BackLds<W>& L = lds_all[threadIdx.x / W];
  const int t = threadIdx.x % W;  // thread within the query group
  const uint32_t qcount = *qcount_p;
  unsigned long long st_rows = 0, st_edges = 0, st_done = 0;
  // the first query of every group is static (group g takes g); later ones are dequeued past the
  // groups' count, so groups beyond the list and the list's end cost no atomic on the one hot word
  const uint32_t n_groups = gridDim.x * (256 / W), g0 = blockIdx.x * (256 / W) + threadIdx.x / W;
  for (bool first = true;; first = false) {
    if (first) {
      if (t == 0) L.qi = g0;
    } else {
      if (n_groups >= qcount) break;  // the static round took every query
      if (t == 0) L.qi = n_groups + atomicAdd(qhead, 1u);
    }
    bk_sync<W>();
    const uint32_t hi = L.qi;
    if (hi >= qcount) break;
    const uint32_t qi = qlist[hi];
    const RQuery q = rq[qi];
    const uint2 hr = holders_find(s, q.subj);
    for (uint32_t i = t * 4; i < VSLOTS; i += W * 4)
      *reinterpret_cast<uint4*>(&L.vis[i]) = make_uint4(NONE, NONE, NONE, NONE);
    if (t == 0) {
      L.n = 0;
      L.hit = 0;
      L.over = hr.y > CAP ? 1u : 0u;
    }
    bk_sync<W>();
    if (!L.over) {  // level 0: the holders (the root itself was probed by k_resolve)
      for (uint32_t i = t; i < hr.y; i += W) {
        const uint32_t v = s.hold[hr.x + i];
        if (v == q.node) L.hit = 1;
        else bk_add(L, v);
      }
    }
    bk_sync<W>();
    uint32_t lvl_b = 0, lvl_e = L.n;
    uint32_t budget = BackCfg<W>::EDGES;  // wave-uniform
    for (int j = 1; j <= q.depth - 1 && lvl_b < lvl_e && !L.hit && !L.over; j++) {
      const bool keep = j < q.depth - 1;  // parents found here can still be expanded
      for (uint32_t base = lvl_b; base < lvl_e; base += W) {
        const uint32_t i = base + t;
        uint64_t rb = 0, re = 0;
        if (i < lvl_e) {
          const uint32_t v = L.lst[i];
          rb = s.radj_off[v];
          re = s.radj_off[v + 1];
          st_rows++;
        }
        L.rb[t] = rb;
        uint32_t total;
        const uint32_t excl = W == 64 ? wave_excl_scan((uint32_t)(re - rb), &total)
                                      : block_excl_scan((uint32_t)(re - rb), L.wsum, &total);
        L.pref[t] = excl;
        if (total > budget && t == 0) L.over = 1;  // too much for one wave: the grid tier takes it
        bk_sync<W>();
        if (L.over) break;
        budget -= total;
        if (t == 0) st_edges += total;
        // BU edges per thread and step: the BU parent loads of a thread are independent, so a long
        // reverse row costs 1/BU of the dependent round trips
        for (uint32_t eb = 0; eb < total; eb += W * BU) {
          if (*(volatile uint32_t*)&L.over || *(volatile uint32_t*)&L.hit) break;
          uint32_t p[BU];
#pragma unroll
          for (int u = 0; u < BU; u++) {
            const uint32_t e = eb + u * W + t;
            p[u] = NONE;
            if (e < total) {
              const int own = owner_search(L.pref, W, e);
              p[u] = s.radj[L.rb[own] + (e - L.pref[own])];
            }
          }
#pragma unroll
          for (int u = 0; u < BU; u++) {
            if (p[u] == NONE) continue;
            if (p[u] == q.node) L.hit = 1;
            else if (keep) bk_add(L, p[u]);
          }
        }
        bk_sync<W>();
        if (L.hit || L.over) break;
      }
      bk_sync<W>();
      lvl_b = lvl_e;
      lvl_e = L.n;
    }
    bk_sync<W>();
    if (t == 0) {
      if (L.hit || !L.over) {
        out[qi] = L.hit ? KG_IS_MEMBER : KG_NOT_MEMBER;
        if (err) err[qi] = KG_ERR_NONE;
        st_done++;
      } else {
        next_list[atomicAdd(next_count, 1u)] = qi;
      }
    }
    bk_sync<W>();
  }
  __syncthreads();  // the groups of a workgroup finish at different times
  const int idx[3] = {ST_BROWS, ST_BEDGES, ST_BACK};
  const unsigned long long v[3] = {st_rows, st_edges, st_done};
  block_stats<3>(ctl, idx, v);
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
    // rows come from the generator itself (row e of node v == synth_subject(v, e)), so a shard of
    // the graph (hash-sharded mode) draws exactly the queries the whole graph does
    uint32_t cur = start;
    for (int step = 0; step < 16; step++) {
      const uint32_t deg = synth_degree(L, cur);
      if (deg == 0) break;
      uint32_t sub = synth_subject(L, cur, (uint32_t)(shash(seed, ((uint64_t)i << 8) | step, 9) % deg));
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

// A batch in two phases, so one host thread can keep batches in flight on several devices (the
// multi-replica kg_check_batch): check_batch_begin enqueues every kernel on the workspace's stream
// and returns without waiting; check_batch_end waits for the stream, finishes the grid tier if its
// first round overflowed (rare: a rerun with fewer slots) and fills the statistics.
int check_batch_begin(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t global_max_depth,
                      uint8_t* d_out, uint32_t* d_err, kg_stats* stats, BatchPending* bp) {
  *bp = BatchPending{};
  bp->stats = stats;
  bp->d_out = d_out;
  bp->d_err = d_err;
  if (global_max_depth < 1) global_max_depth = 5;  // config.schema.json:308-315 default
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  HIPC(hipSetDevice(s->device));
  hipStream_t stream = w->stream;
  // boolean rewrites over rewrite-free leaves (kg_formula.hip): the batch runs as the originals plus
  // their leaf sub-checks; check_batch_end combines the leaves into the requested results
  const uint32_t* n_extra = nullptr;
  const size_t n_base = n;
  if (s->n_fplans && n) {
    const kg_query* q2;
    size_t n2;
    uint8_t* out2;
    uint32_t* err2;
    const uint2* ref;
    if (int rc = formula_split(s, w, d_q, n, global_max_depth, &q2, &n2, &n_extra, &out2, &err2, &ref)) return rc;
    bp->split = true;
    bp->f_n = n;
    bp->f_out = d_out;
    bp->f_err = d_err;
    bp->f_ref = ref;
    d_q = q2;
    n = n2;
    d_out = out2;
    d_err = err2;
    bp->d_out = d_out;
    bp->d_err = d_err;
  }
  // scratch: rq[n] | light[8n] (8 shards) | light2[n] | gen[n] | medium[n] | heavy[n] | giant[n] | p2[n] |
  //          back2[n] | Ctl
  auto layout = [](size_t m, size_t* off) {  // rq | light[8m] | light2 | gen | medium | heavy | giant | p2 | back2 | Ctl
    off[0] = 0;
    off[1] = align_up(off[0] + m * sizeof(RQuery));
    off[2] = align_up(off[1] + 8 * m * 4);
    for (int k = 3; k <= 9; k++) off[k] = align_up(off[k - 1] + m * 4);
    return align_up(off[9] + sizeof(Ctl));
  };
  size_t off[10];
  const size_t total = layout(n, off);
  if (total > w->scratch_bytes) {  // sized for >= 64 Ki queries, grown geometrically (hipFree stalls the device)
    const size_t m = std::max<size_t>(65536, std::max<size_t>(2 * w->scratch_n, n));
    size_t tmp[10];
    const size_t want = layout(m, tmp);
    if (w->scratch) hipFree(w->scratch);
    w->scratch = nullptr;
    w->scratch_bytes = 0;
    HIPC(hipMalloc(&w->scratch, want));
    w->scratch_bytes = want;
    w->scratch_n = m;
  }
  const size_t off_rq = off[0], off_light = off[1], off_light2 = off[2], off_gen = off[3], off_med = off[4],
               off_heavy = off[5], off_giant = off[6], off_p2 = off[7], off_back2 = off[8], off_ctl = off[9];
  char* base = (char*)w->scratch;
  RQuery* rq = (RQuery*)(base + off_rq);
  uint32_t* light = (uint32_t*)(base + off_light);
  uint32_t* light2 = (uint32_t*)(base + off_light2);
  uint32_t* gen = (uint32_t*)(base + off_gen);
  uint32_t* medium = (uint32_t*)(base + off_med);
  uint32_t* heavy = (uint32_t*)(base + off_heavy);
  uint32_t* giant = (uint32_t*)(base + off_giant);
  uint32_t* p2 = (uint32_t*)(base + off_p2);
  uint32_t* back2 = (uint32_t*)(base + off_back2);
  Ctl* ctl = (Ctl*)(base + off_ctl);
  // tiers after k_light<64> (kg_snapshot_tune "tiers"): 0 grid; 1 LDS workgroup tier, then grid;
  // 2 LDS workgroup tier, then HBM workgroup tier (one workgroup per query)
  const bool use_medium = s->tiers >= 1, wg_heavy = s->tiers == 2;
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  const uint64_t words = (nn + 31) / 32 + 1;
  const uint64_t cap_h = std::min<uint64_t>(nn, 4u << 20);
  uint32_t H = 0, *hb = nullptr, *hl = nullptr, *gb = nullptr, *gl = nullptr;
  if (wg_heavy) {  // H slots of (bitmap + cap list) + one giant slot (bitmap + n_nodes list)
    H = (uint32_t)std::min<uint64_t>(2 * (uint64_t)s->n_cu,
                                     std::max<uint64_t>(1, (8ull << 30) / ((words + cap_h) * 4)));
    const size_t pool = ((size_t)H * (words + cap_h) + (words + nn)) * 4;
    if (pool > w->heavy_pool_bytes) {
      if (w->heavy_pool) hipFree(w->heavy_pool);
      w->heavy_pool = nullptr;
      w->heavy_pool_bytes = 0;
      HIPC(hipMalloc(&w->heavy_pool, pool));
      HIPC(hipMemsetAsync(w->heavy_pool, 0, pool, stream));  // bitmaps start clear and are left clear
      w->heavy_pool_bytes = pool;
    }
    hb = (uint32_t*)w->heavy_pool;
    hl = hb + (size_t)H * words;
    gb = hl + (size_t)H * cap_h;
    gl = gb + words;
  }
  bool grid_pending = false;
  const uint32_t *grid_list = nullptr, *grid_count = nullptr;

  if (stats && !w->ev[0])
    for (auto& e : w->ev) HIPC(hipEventCreate(&e));
  hipEvent_t e0 = w->ev[0], e1 = w->ev[1], l0 = w->ev[2], l1 = w->ev[3];
  if (stats) HIPC(hipEventRecord(e0, stream));
  HIPC(hipMemsetAsync(ctl, 0, sizeof(Ctl), stream));
  if (n) {
    const bool use_back = s->back_tier && s->ds.radj;
    // k_stream4 (variant 15) takes its work as LQuery records in 8 shards; shard h receives the
    // appends of k_resolve's blocks h, h + 8, ... (<= 256 each).  They live in the light list's
    // space (8 n u32 >= (n + 2048) LQuery for the >= 64 Ki queries the scratch is sized for).
    const uint32_t nblk = (uint32_t)((n + 255) / 256);
    const bool compact = s->light_tier != 1 && (s->stream_variant == 15 || s->stream_variant == 16);
    const uint32_t lq_cap = (nblk + 7) / 8 * 256;
    LQuery* lq = compact ? reinterpret_cast<LQuery*>(light) : nullptr;
    if (compact && (size_t)8 * lq_cap * sizeof(LQuery) > (size_t)8 * w->scratch_n * 4)
      return set_error(-5, "stream work list does not fit the scratch");
    hipLaunchKernelGGL(k_resolve, dim3(nblk), dim3(256), 0, stream, s->ds, d_q, (uint32_t)n,
                       (uint32_t)n_base, n_extra, global_max_depth, rq, d_out, d_err, light, gen,
                       use_back ? (s->resolve_unheld ? 2 : 1) : 0, ctl, lq, lq_cap, compact ? s->stream_big_len : 0u,
                       s->stream_big_depth);
    HIPC(hipGetLastError());
    uint32_t* const after_list = use_medium ? medium : heavy;
    uint32_t* const after_count = use_medium ? &ctl->medium_count : &ctl->heavy_count;
    // overflow of the first wave tier: k_light<64> (wide tier) or straight to the tiers after it
    uint32_t* const ovf_list = s->wide_tier ? light2 : after_list;
    uint32_t* const ovf_count = s->wide_tier ? &ctl->light2_count : after_count;
    if (stats) HIPC(hipEventRecord(l0, stream));
    if (s->light_tier == 1) {
      // 7 workgroups of 4 waves per CU: ~21 KiB of LDS per workgroup allows 28 waves/CU
      const uint32_t light_grid = (uint32_t)std::min<uint64_t>((uint64_t)s->n_cu * 7, (n + 15) / 16 + 8);
      hipLaunchKernelGGL((k_light<16, 7, 64>), dim3(light_grid), dim3(256), 0, stream, s->ds, rq,
                         WorkList{light, ctl->light8, (uint32_t)n, 1u}, ctl->heads, d_out, d_err, ovf_list,
                         ovf_count, ctl);
    } else {
      // ~30 KiB of LDS per workgroup (variant 0: 8 slots x 512 B visited + 256-entry FIFO per wave;
      // 1: 16 slots x 256 B; 2: 16 slots x 512 B + 512-entry FIFO): 5 (2: 3) workgroups per CU
      const WorkList wl{light, ctl->light8, (uint32_t)n, 1u};
      // k_stream variants (slots, visited layout, FIFO, chunk); LDS per workgroup sets the WGs per CU:
      //   0: 8 x 512 B per slot, 256-entry FIFO (~30 KiB, 5/CU)   1: 16 x 256 B (~31 KiB, 5/CU)
      //   2: 16 x 512 B, 512 FIFO (~46 KiB, 3/CU)                  3: 32 x 128 B, 192 FIFO (~30 KiB, 5/CU)
      //   4: 32 x 256 B (~49 KiB, 3/CU)
      //   5: 32 slots sharing one 1024-key table (8 KiB), <= 128 expanded nodes per query (~49 KiB, 3/CU)
      //   6: the same with <= 256 per query and a 320-entry FIFO (~53 KiB, 3/CU)
      //   7: as 5 with <= 64 per query   8: as 7 with a 512-key table (~45 KiB)
      const int sv = s->stream_variant;
      const uint32_t per_cu =
          s->stream_wgs ? (uint32_t)s->stream_wgs : ((sv == 0 || sv == 1 || sv == 3 || sv >= 9) ? 5u : 3u);
      const uint32_t ecap = s->stream_ecap ? s->stream_ecap : 0xFFFFFFFFu;
      // >= 8 workgroups: with stream_steal < 8 a wave drains only `ranges` of the 8 per-XCD ranges
      // starting at its label blockIdx & 7, so every label must occur for every range to be drained
      const uint32_t grid =
          std::max<uint32_t>(8u, (uint32_t)std::min<uint64_t>((uint64_t)s->n_cu * per_cu, (n + 31) / 32 + 8));
      using V0 = SlotVis<8, 7>;
      using V1 = SlotVis<16, 6>;
      using V2 = SlotVis<16, 7>;
      using V3 = SlotVis<32, 5>;
      using V4 = SlotVis<32, 6>;
      using V5 = WaveVis<10, 128>;
      using V6 = WaveVis<10, 256>;
      using V7 = WaveVis<10, 64>;
      using V8 = WaveVis<9, 64>;
#define KG_STREAM(Q, V, QC, CH)                                                                                   \
  hipLaunchKernelGGL((k_stream<Q, V, QC, CH>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads, d_out, \
                     d_err, ovf_list, ovf_count, ctl, ecap)
      if (sv == 1) KG_STREAM(16, V1, 256, 32);
      else if (sv == 2) KG_STREAM(16, V2, 512, 32);
      else if (sv == 3) KG_STREAM(32, V3, 192, 64);
      else if (sv == 4) KG_STREAM(32, V4, 256, 64);
      else if (sv == 5) KG_STREAM(32, V5, 256, 64);
      else if (sv == 6) KG_STREAM(32, V6, 320, 64);
      else if (sv == 7) KG_STREAM(32, V7, 256, 64);
      else if (sv == 8) KG_STREAM(32, V8, 256, 64);
      else if (sv == 9)
        hipLaunchKernelGGL((k_stream2<9, 256, 64, 64, 1>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, ecap, std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, 64u)), s->stream_steal);
      else if (sv == 11)  // 128-edge windows (two edges per lane)
        hipLaunchKernelGGL((k_stream2<9, 256, 64, 64, 2>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, ecap, std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, 64u)), s->stream_steal);
      else if (sv == 12)  // no expanded-node cap per query (edge budget only)
        hipLaunchKernelGGL((k_stream2<9, 256, 64, 0, 1>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, ecap, std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, 64u)), s->stream_steal);
      else if (sv == 14)  // 128-edge windows, no node cap
        hipLaunchKernelGGL((k_stream2<9, 256, 64, 0, 2>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, ecap, std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, 64u)), s->stream_steal);
      else if (sv == 15)  // pipelined dequeue of LQuery records, no returning LDS atomics
        hipLaunchKernelGGL((k_stream4<9, 256>), dim3(grid), dim3(256), 0, stream, s->ds, LqList{lq, ctl->light8, lq_cap},
                           ctl->heads, d_out, rq, ovf_list, ovf_count, ctl, ecap,
                           std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, S4_CHUNK)), s->stream_steal,
                           s->stream_tail_ecap, s->stream_big_len ? std::min<uint32_t>(s->stream_big_chunk, S4_CHUNK) : 0u);
      else if (sv == 16)  // two interleaved FIFO engines per wave
        hipLaunchKernelGGL((k_stream5<9, 128>), dim3(grid), dim3(256), 0, stream, s->ds, LqList{lq, ctl->light8, lq_cap},
                           ctl->heads, d_out, rq, ovf_list, ovf_count, ctl, ecap,
                           std::max<uint32_t>(1u, std::min<uint32_t>(s->stream_chunk, S4_CHUNK)), s->stream_steal);
      else if (sv == 10)
        hipLaunchKernelGGL((k_stream3<9, 256, 64, 64>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, 0xFFFFFFFFu);
      else if (sv == 13)  // k_stream3 without the node cap, bounded by the edge budget
        hipLaunchKernelGGL((k_stream3<9, 256, 64, 0>), dim3(grid), dim3(256), 0, stream, s->ds, rq, wl, ctl->heads,
                           d_out, ovf_list, ovf_count, ctl, ecap);
      else KG_STREAM(8, V0, 256, 16);
#undef KG_STREAM
    }
    HIPC(hipGetLastError());
    if (stats) HIPC(hipEventRecord(l1, stream));
    if (s->wide_tier) {
      hipLaunchKernelGGL((k_light<64, 9, 256>), dim3((uint32_t)s->n_cu * 4), dim3(256), 0, stream, s->ds, rq,
                         WorkList{light2, &ctl->light2_count, 0u, 0u}, ctl->heads2, d_out, d_err, after_list,
                         after_count, ctl);
      HIPC(hipGetLastError());
    }
    if (use_medium) {
      hipLaunchKernelGGL(k_medium, dim3((uint32_t)s->n_cu * 3), dim3(256), 0, stream, s->ds, rq, medium,
                         &ctl->medium_count, &ctl->medium_head, d_out, d_err, heavy, &ctl->heavy_count, ctl);
      HIPC(hipGetLastError());
    }
    if (wg_heavy) {
      hipLaunchKernelGGL(k_heavy, dim3(H), dim3(256), 0, stream, s->ds, rq, heavy, &ctl->heavy_count,
                         &ctl->heavy_head, d_out, d_err, hb, words, hl, cap_h, giant, &ctl->giant_count, ctl);
      HIPC(hipGetLastError());
      hipLaunchKernelGGL(k_heavy, dim3(1), dim3(256), 0, stream, s->ds, rq, giant, &ctl->giant_count,
                         &ctl->giant_head, d_out, d_err, gb, words, gl, nn, giant /*never overflows*/, &ctl->pad0,
                         ctl);
      HIPC(hipGetLastError());
    } else {
      // backward tier first (k_back), its overflow -> forward grid tier
      const uint32_t* fwd_list = heavy;
      const uint32_t* fwd_count = &ctl->heavy_count;
      if (use_back) {
        // wave per query (~48 KiB LDS per workgroup: 3 per CU), its overflow to the workgroup-per-query
        // width (~52 KiB: 3 per CU), whose overflow goes to the grid tier
        hipLaunchKernelGGL(k_back<64>, dim3((uint32_t)s->n_cu * s->back_wgs), dim3(256), 0, stream, s->ds, rq, heavy,
                           &ctl->heavy_count, &ctl->back_head, d_out, d_err, back2, &ctl->back2_count, ctl);
        HIPC(hipGetLastError());
        if (s->back_tier == 2) {  // wave width only: its overflow goes straight to the grid tier
          fwd_list = back2;
          fwd_count = &ctl->back2_count;
        } else {
          hipLaunchKernelGGL(k_back<256>, dim3((uint32_t)s->n_cu * s->back_wgs), dim3(256), 0, stream, s->ds, rq, back2,
                             &ctl->back2_count, &ctl->back2_head, d_out, d_err, giant, &ctl->fwd_count, ctl);
          HIPC(hipGetLastError());
          fwd_list = giant;
          fwd_count = &ctl->fwd_count;
        }
      }
      // first grid round enqueued without waiting; its readback is checked after the batch's one sync
      const int rc = grid_tier(s, w, rq, fwd_list, fwd_count, global_max_depth, d_out, d_err, stream, &bp->gs, 1);
      if (rc < 0) return rc;
      grid_pending = rc == 1;
      grid_list = fwd_list;
      grid_count = fwd_count;
    }
    if (s->has_program) {
      InterpCtl ic{};
      ic.gen_count = &ctl->gen_count;
      ic.p2_list = p2;
      ic.st_general = &ctl->st[ST_GENERAL];
      ic.st_rows = &ctl->st[ST_ROWS];
      ic.st_edges = &ctl->st[ST_EDGES];
      ic.st_probes = &ctl->st[ST_PROBES];
      HIPC(hipMemcpyAsync(&ctl->ic, &ic, sizeof ic, hipMemcpyHostToDevice, stream));
      if (launch_general(s, w, d_q, rq, gen, &ctl->gen_count, &ctl->ic, d_out, d_err, (uint32_t)n, stream)) return -1;
    }
    // the requested results, stream-ordered before anything the caller enqueues after this call
    if (bp->split && formula_combine(s, w, bp->f_n, bp->f_ref, d_out, d_err, bp->f_out, bp->f_err)) return -1;
  }
  // one synchronisation per batch: the grid round's readback and the counters come back together
  static_assert(sizeof(Ctl) <= 32768, "Ctl readback fits the lower half of the pinned buffer");
  void* hbuf = w->host_buf(65536);
  if (!hbuf) return set_error(-1, "pinned host buffer");
  if (stats) {
    HIPC(hipEventRecord(e1, stream));
    HIPC(hipMemcpyAsync(hbuf, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, stream));
  }
  bp->grid_pending = grid_pending;
  bp->grid_list = grid_list;
  bp->grid_count = grid_count;
  bp->rq = rq;
  bp->gdepth = global_max_depth;
  bp->n = n;
  bp->wg_heavy = wg_heavy;
  bp->ctl_host = hbuf;
  return 0;
}

int check_batch_end(Snapshot* s, Workspace* w, BatchPending* bp, bool* reran, bool blocking) {
  if (reran) *reran = false;
  kg_stats* stats = bp->stats;
  hipStream_t stream = w->stream;
  GridStats& gs = bp->gs;
  if (stats || bp->grid_pending)
    if (int rc = w->wait(stream, blocking)) return rc;
  if (bp->grid_pending) {  // a round that overflowed its log reruns here with fewer slots (synchronously)
    if (int rc = grid_tier(s, w, bp->rq, bp->grid_list, bp->grid_count, bp->gdepth, bp->d_out, bp->d_err, stream, &gs, 2))
      return rc;
    if (reran) *reran = w->grid_reran;
    // the rerun rewrote leaf results after check_batch_begin's combine: combine again
    if (bp->split && w->grid_reran &&
        formula_combine(s, w, bp->f_n, bp->f_ref, bp->d_out, bp->d_err, bp->f_out, bp->f_err))
      return -1;
  }
  if (stats) {
    float ms = 0, lms = 0;
    HIPC(hipEventElapsedTime(&ms, w->ev[0], w->ev[1]));
    if (bp->n) HIPC(hipEventElapsedTime(&lms, w->ev[2], w->ev[3]));
    Ctl h;
    memcpy(&h, bp->ctl_host, sizeof(Ctl));
    for (int x = 0; x < 8; x++)
      for (int k = 0; k < ST_N; k++) h.st[k] += h.st8[x][k];
    stats->rows_opened = h.st[ST_ROWS] + h.st[ST_LROWS];
    stats->edges_read = h.st[ST_EDGES] + h.st[ST_LEDGES];
    stats->direct_probes = h.st[ST_PROBES] + h.st[ST_LPROBES];
    stats->light_rows_opened = h.st[ST_LROWS];
    stats->light_edges_read = h.st[ST_LEDGES];
    stats->light_probes = h.st[ST_LPROBES];
    stats->light_ms = lms;
    stats->frontier_hbm = h.st[ST_FHBM];
    stats->n_light = h.st[ST_LIGHT];
    stats->n_medium = h.st[ST_MEDIUM];
    stats->n_heavy = bp->wg_heavy ? h.st[ST_HEAVY] : gs.done;
    stats->n_wide = h.light2_count;
    stats->n_grid = gs.done;
    stats->rows_opened += gs.rows;
    stats->edges_read += gs.edges;
    stats->direct_probes += gs.probes;
    stats->frontier_hbm += gs.logged;
    stats->n_general = h.st[ST_GENERAL];
    stats->n_back = h.st[ST_BACK];
    stats->n_no_holder = h.st[ST_NOHOLD];
    stats->back_rows = h.st[ST_BROWS];
    stats->back_edges = h.st[ST_BEDGES];
    stats->light_steps = h.st[ST_LSTEPS];
    stats->light_waves = h.st[ST_LWAVES];
    stats->light_wave_ticks = h.st[ST_LTICKS];
    unsigned long long t_ns = 0, t_e = 0, l_m = 0;
    for (int x = 0; x < 8; x++) {
      t_ns = std::max(t_ns, h.tmax8[x][0]);
      t_e = std::max(t_e, h.tmax8[x][1]);
      l_m = std::max(l_m, h.tmax8[x][2]);
    }
    stats->light_span_ticks = t_e ? t_e - ~t_ns : 0;
    stats->light_wave_max_ticks = l_m;
    stats->kernel_ms = ms;
  }
  return 0;
}

int check_batch_device(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t global_max_depth,
                       uint8_t* d_out, uint32_t* d_err, kg_stats* stats) {
  BatchPending bp;
  if (int rc = check_batch_begin(s, w, d_q, n, global_max_depth, d_out, d_err, stats, &bp)) return rc;
  return check_batch_end(s, w, &bp, nullptr, s->device_sync != 0);
}

}  // namespace kg
