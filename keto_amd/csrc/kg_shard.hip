// kg_shard.hip -- the hash-sharded check mode: graphs larger than one GPU.
//
// Rank r holds the rows of the nodes with shard_owner(ns, obj) == r.  A batch is a level-
// synchronous BFS across ranks over frontier records kg_frec (query, node, subject, rest depth):
//   kg_shard_seed   maps the home rank's queries (node map, depth clamp engine.go:68-70) and
//                   sends one record per query to the owner of its root
//   kg_shard_level  per received record: a hit report sets the home query's result; otherwise
//                   the owner deduplicates (query, node) in its visited table (first arrival =
//                   shallowest level, as in the single-GPU tiers), probes checkDirect
//                   (engine.go:148-177) on its local dset, reports a hit to the query's home, or
//                   expands the node's local set row (checkExpandSubject engine.go:87-145) into
//                   records (query, child, subject, depth - 1) for the children's owners
// Between levels the driver (keto_amd/sharded.py) exchanges the per-destination buckets with an
// all-to-all (RCCL over xGMI) and stops when no rank sends anything.  Semantics: bounded
// reachability over rewrite-free nodes, exactly the single-GPU engine's.  A query
// that reaches a node whose relation has a rewrite or is undeclared (relflag != 0: the
// interpreter's territory, rewrites.go:30-260 / engine.go:228) is answered KG_ERROR with
// KG_ERR_NOT_IMPLEMENTED, whatever else it reaches: the owner reports it to the home rank, which
// records it in err[] (errors win over hits; kg_shard_finish folds err into res).
// Pruning (the single-GPU tiers' early exits, made rank-independent): a query whose subject id no
// row of any rank holds is NotMember at seed (no program only: with rewrites it may still reach an
// error); a query answered IsMember by the end of level k drops its records from level k+1 on --
// every rank reads the same per-level done bitmap (packed from the home ranks' results, all-gathered
// by the driver), so the answer does not depend on the number of ranks.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kg_bfs.h"
#include "kg_formula.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

constexpr uint32_t Q_BITS = 26, Q_MASK = (1u << Q_BITS) - 1;
// kg_frec.depth bit 30: the sender's Bloom signature of the node's row rules the subject out, so the
// owner skips the checkDirect probe (a certain miss); the rest depth sits in the low bits
constexpr int32_t D_NOPROBE = 1 << 30;
// bit 29: the record checks the own part of a split formula query's node (its rows as a plain node,
// the node's rewrite evaluated by the formula instead)
constexpr int32_t D_OWN = 1 << 29, D_MASK = D_OWN - 1;
// (Round 5's packed local records -- the child's set-row begin in place of its node id, knob
// "shard_pack" -- measured neutral and were removed in round 6, profiles/r5k_level_occupancy_pack_ab.jsonl.)

// Rewrite materialisation runs in this mode too (union nodes are plain; kg_augment.hip), so a node
// needs the interpreter -- unavailable across shards: an error -- when its own relation has a
// rewrite that was not materialised or is undeclared.  The node flags say so for every node on
// every rank alike (relflag for snapshots without them).
__device__ __forceinline__ bool node_bad(const DevSnap& s, uint32_t node) {
  if (s.nflags) return (s.nflags[node] & (NF_REWRITE | NF_ERR)) != 0;
  // no namespace program: nothing is bad, and the node's (ns, rel) -- two random loads -- is not read
  if (!s.relflags) return false;
  return relflag(s, s.nd_ns[node], s.nd_rel[node]) != 0;
}

// Formula split in this mode: a query whose relation has a formula plan (kg_formula.hip) becomes
// its own part and its leaves as records of their own, in result slots n + i * (1 + leaves) + k;
// kg_shard_finish evaluates the formula.
struct ShardFormula {
  const int32_t* fidx;   // (ns, rel) -> plan or -1; null: no plans
  const FPlan* plans;
  uint32_t k;            // slots per split query: 1 (own part) + most leaves
  const uint8_t* virt;   // (ns, rel) -> union relation (no node: NotMember)
  uint32_t* ref;         // [n] plan of query i, or NONE
};
constexpr int SV_PROBES = 64;
// Escalation (kg_snapshot_tune "shard_budget", snapshots without a namespace program): a query whose
// forward records have expanded more set edges than the budget on one rank -- a hub-heavy walk, the
// stream tier's edge budget in the single-GPU engine -- stops walking forward and is answered by the
// backward phase (reverse search from its subject's holders, kg_shard_back_*).  The home rank marks
// it with ESC_BIT in err[] while the batch runs (kg_shard_finish clears it).  The reverse search has
// a budget of its own (shard_back_budget reverse edges per query and rank, the backward tier's); a
// query past both (ESC2_BIT) is walked forward once more without any budget (kg_shard_refwd_seed) --
// the single-GPU engine's stream -> backward -> grid tier chain.
constexpr uint32_t ESC_BIT = 0x40000000u, ESC2_BIT = 0x20000000u;
constexpr int QCNT_LOG2 = 22;  // per-rank edge counters, hashed by query (a collision only escalates early:
                               // every query whose row a full counter drops is marked escalated)
// A received record whose set row is longer than this is expanded by the whole grid (k_shard_heavy).
constexpr uint32_t SHARD_HEAVY = 4096, SHARD_HEAVY_CAP = 1u << 20;
constexpr uint32_t HEAVY_TILE = 256;              // edges per k_shard_heavy tile
constexpr uint64_t HEAVY_TF_CAP = 1ull << 22;     // tiles with a first-row entry (beyond: binary search)
constexpr int HEAVY_EDGE_BITS = 40;               // packed counter: rows << 40 | edges
struct HeavyRow {
  kg_frec r;  // depth without flag bits
  uint64_t rb;
  uint64_t e0;  // first edge of the row in the level's heavy-edge space
  uint32_t len, pad;
};
// The hub rows a level queues for k_shard_heavy: one packed 64-bit atomic per row gives its slot
// and its edge offset together (rows in slot order = edge order, no gaps but past `cap`), and every
// HEAVY_TILE-edge tile that starts inside a row records the row (tile -> first row), so the heavy
// kernel walks the level's hub edges flat, edge-parallel over the whole grid.
struct HeavyList {
  HeavyRow* rows;
  unsigned long long* pk;
  uint32_t* tf;
  uint32_t cap;
};
// Workgroup-aggregated append (every thread of the 256-thread workgroup calls it): one packed atomic
// per workgroup gives the workgroup's first slot and edge offset.  Returns whether this thread's row
// was queued (false past the cap: the caller expands it itself).
__device__ __forceinline__ bool heavy_append(const HeavyList& H, bool app, const HeavyRow& row) {
  __shared__ uint32_t s_hc[4];
  __shared__ uint64_t s_he[4];
  __shared__ unsigned long long s_hold;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(app);
  const uint64_t len = app ? row.len : 0ull;
  uint64_t x = len;  // inclusive scan of the lengths within the wave
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = shfl_up64(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) {
    s_hc[wave] = (uint32_t)__popcll(m);
    s_he[wave] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t tc = s_hc[0] + s_hc[1] + s_hc[2] + s_hc[3], te = s_he[0] + s_he[1] + s_he[2] + s_he[3];
    s_hold = tc ? atomicAdd(H.pk, (unsigned long long)((tc << HEAVY_EDGE_BITS) | te)) : 0ull;
  }
  __syncthreads();
  bool ok = false;
  if (app) {
    uint64_t at = s_hold >> HEAVY_EDGE_BITS, e0 = s_hold & ((1ull << HEAVY_EDGE_BITS) - 1);
    for (int w = 0; w < wave; w++) {
      at += s_hc[w];
      e0 += s_he[w];
    }
    at += (uint64_t)__popcll(m & ((1ull << lane) - 1));
    e0 += x - len;
    if (at < H.cap) {
      HeavyRow y = row;
      y.e0 = e0;
      H.rows[at] = y;
      for (uint64_t t = (e0 + HEAVY_TILE - 1) / HEAVY_TILE; t * HEAVY_TILE < e0 + len && t < HEAVY_TF_CAP; t++)
        H.tf[t] = (uint32_t)at;
      ok = true;
    }
  }
  __syncthreads();
  return ok;
}

// (query, node) visited table: open addressing, cleared per batch.  1 fresh, 0 seen, -1 full.
__device__ __forceinline__ int sv_insert(uint64_t* T, uint64_t mask, uint64_t key) {
  uint64_t h = mix64(key) & mask;
  for (int p = 0; p < SV_PROBES; p++) {
    const uint64_t old = atomicCAS((unsigned long long*)&T[h], (unsigned long long)EMPTY64, (unsigned long long)key);
    if (old == EMPTY64) return 1;
    if (old == key) return 0;
    h = (h + 1) & mask;
  }
  return -1;
}

// (Round 5's lossy direct-mapped variant of this table, knob "shard_vis_mode", measured flat and was
// removed in round 6, profiles/r5e_visited_table_size_ab.jsonl.)

// Workgroup-aggregated append of one record per active thread to the bucket of its destination
// rank: ballots per wave into LDS counters, then ONE device atomic per (workgroup, destination) --
// at world 1 every record goes to one counter, so per-wave atomics serialised on it.  Every thread
// of the workgroup must call it (256 threads).
// sub > 1 (one rank, kg_shard_levels): the single bucket is `sub` segments of `cap` records with a
// counter each, picked by the workgroup's XCD label (blockIdx & (sub - 1)), flags word counts[sub]:
// a level's thousands of workgroup appends no longer queue on one counter word (~11 ns each at the
// memory side, ~90 M/s per word: MI355X_MICROARCH.md); the next level reads the segments.
__device__ __forceinline__ void emit(bool act, uint32_t dest, const kg_frec& r, kg_frec* out, uint64_t cap,
                                     uint32_t* counts, uint32_t nranks, uint32_t sub = 1) {
  __shared__ uint32_t s_cnt[KG_SHARD_MAX_RANKS], s_base[KG_SHARD_MAX_RANKS];
  const int tid = threadIdx.x, lane = lane_id();
  if (sub > 1) {
    dest = blockIdx.x & (sub - 1);
    nranks = sub;
  }
  if (tid < (int)nranks) s_cnt[tid] = 0;
  __syncthreads();
  uint64_t pending = __ballot(act);
  uint32_t my = 0;
  while (pending) {
    const int lead = __ffsll((unsigned long long)pending) - 1;
    const uint32_t d = __shfl(dest, lead, 64);
    const uint64_t m = __ballot(act && dest == d);
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(&s_cnt[d], (uint32_t)__popcll(m));
    base = __shfl(base, lead, 64);
    if (act && dest == d) my = base + __popcll(m & ((1ull << lane) - 1));
    pending &= ~m;
  }
  __syncthreads();
  if (tid < (int)nranks) s_base[tid] = s_cnt[tid] ? atomicAdd(&counts[tid], s_cnt[tid]) : 0u;
  __syncthreads();
  if (act) {
    const uint32_t at = s_base[dest] + my;
    if (at < cap) out[(uint64_t)dest * cap + at] = r;
    else atomicOr(&counts[nranks], 1u);
  }
  __syncthreads();
}

// emit() for Q records per thread (one ballot pass per record slot, still ONE device atomic per
// (workgroup, destination)): the seed handles Q queries per thread, so a batch takes Q times fewer
// workgroup appends on the bucket counters.  Every thread of the workgroup must call it.
template <int Q>
__device__ __forceinline__ void emit_q(const bool (&act)[Q], const uint32_t (&dest)[Q], const kg_frec (&r)[Q],
                                       kg_frec* out, uint64_t cap, uint32_t* counts, uint32_t nranks) {
  __shared__ uint32_t s_cnt[KG_SHARD_MAX_RANKS], s_base[KG_SHARD_MAX_RANKS];
  const int tid = threadIdx.x, lane = lane_id();
  if (tid < (int)nranks) s_cnt[tid] = 0;
  __syncthreads();
  uint32_t my[Q];
#pragma unroll
  for (int j = 0; j < Q; j++) {
    my[j] = 0;
    uint64_t pending = __ballot(act[j]);
    while (pending) {
      const int lead = __ffsll((unsigned long long)pending) - 1;
      const uint32_t d = __shfl(dest[j], lead, 64);
      const uint64_t m = __ballot(act[j] && dest[j] == d);
      uint32_t base = 0;
      if (lane == lead) base = atomicAdd(&s_cnt[d], (uint32_t)__popcll(m));
      base = __shfl(base, lead, 64);
      if (act[j] && dest[j] == d) my[j] = base + __popcll(m & ((1ull << lane) - 1));
      pending &= ~m;
    }
  }
  __syncthreads();
  if (tid < (int)nranks) s_base[tid] = s_cnt[tid] ? atomicAdd(&counts[tid], s_cnt[tid]) : 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < Q; j++) {
    if (act[j]) {
      const uint32_t at = s_base[dest[j]] + my[j];
      if (at < cap) out[(uint64_t)dest[j] * cap + at] = r[j];
      else atomicOr(&counts[nranks], 1u);
    }
  }
  __syncthreads();
}

// One query of the seed: mapping, depth clamp, the root's record (or an answer at once), and what the
// formula split's parts need.
struct SeedQ {
  bool act, split;
  uint32_t dest, ssubj;
  int32_t dsplit;
  kg_frec r;
  kg_query x;
};

__device__ __forceinline__ SeedQ seed_query(const DevSnap& s, const kg_query* __restrict__ q, uint32_t i, uint32_t n,
                                           int32_t global, uint8_t* res, uint32_t* err,
                                           const uint32_t* __restrict__ held, uint32_t held_n, const ShardFormula& F,
                                           uint4* qinfo) {
  SeedQ o{};
  o.ssubj = NONE;
  if (i >= n) return o;
  if (F.ref) F.ref[i] = NONE;
  const kg_query x = q[i];
  o.x = x;
  uint32_t subj = NONE;
  const bool sid = x.t.sns == KG_SUBJECT_ID;
  if (sid) subj = x.t.sobj < 0x7FFFFFFFu ? x.t.sobj : NONE;
  // without a namespace program a subject id that no rank's row holds is NotMember whatever the root:
  // the holder bit (a small, cache-resident bitmap) is read first and such a query never touches the
  // node map (k_resolve's resolve_unheld order)
  const bool unheld = held && !s.relflags && sid &&
                      (subj == NONE || subj >= held_n || !((held[subj >> 5] >> (subj & 31)) & 1u));
  uint32_t node = NONE, rsig_lo = 0xFFFFFFFFu, rsig = 0xFFFFFFFFu, rlen = 0, rbeg = 0;
  const NSlot* rsl = nullptr;  // the root's slot: its inline check-row subjects (a local root's probe)
  if (!unheld && nmap_key_ok(x.t.ns, x.t.rel, x.t.obj)) {
    const uint64_t key = nmap_key(x.t.ns, x.t.rel, x.t.obj);
    const NSlot* sl = nmap_slot(s, key, hash_home(key, s.nmap_n));
    if (sl) {
      node = sl->node;
      rsig = sl->sig;
      rsig_lo = (uint32_t)sl->pad1;  // signature bits 0-11 in bits 20-31
      rlen = sl->len;
      rbeg = sl->beg;
      rsl = sl;
    }
  }
  if (!sid) {
    const uint32_t sn = nmap_find(s, x.t.sns, x.t.srel, x.t.sobj);
    subj = sn == NONE ? NONE : (SET_BIT | sn);
  }
  int32_t d = x.max_depth;
  if (d <= 0 || global < d) d = global;  // engine.go:68-70
  res[i] = KG_NOT_MEMBER;
  err[i] = KG_ERR_NONE;
  const uint8_t rf = relflag(s, x.t.ns, x.t.rel);
  const uint32_t pr = (x.t.ns < s.n_ns && x.t.rel < s.n_rel) ? x.t.ns * s.n_rel + x.t.rel : NONE;
  const bool virt = F.virt && pr != NONE && F.virt[pr];
  bool bad = node != NONE ? node_bad(s, node) : (rf != 0 && !virt);  // a union without a node: NotMember
  if (bad && F.fidx && pr != NONE && F.fidx[pr] >= 0) {  // a formula over plain / union leaves: split
    const FPlan& P = F.plans[F.fidx[pr]];
    bool ok = true;
    for (uint32_t j = 0; j < P.n_leaves; j++) {
      const uint32_t ln = nmap_find(s, x.t.ns, P.leaf[j], x.t.obj);
      if (ln != NONE && node_bad(s, ln)) ok = false;
    }
    if (ok) {
      F.ref[i] = (uint32_t)F.fidx[pr];
      o.split = true;
      bad = false;
    }
  }
  if (bad) {  // the interpreter's territory: the driver's general phase (keto_amd/sharded.py)
    err[i] = KG_ERR_NOT_IMPLEMENTED;
  } else if (o.split) {
    // records by the caller, one per part
  } else if (unheld) {
    // no row of any rank holds the subject: checkDirect can never hit (NotMember)
  } else if (node != NONE && (subj != NONE || s.relflags)) {
    // an unknown subject can never be held, but with a namespace program the query can still
    // reach a rewrite (an error), so it is seeded all the same (its probes are skipped)
    o.act = true;
    // remote_meta: the slot of a root another rank owns carries the owner and the owner's row length and
    // signature (k_shard_nmap_remote), so it is judged like a local one: a record only if the owner's
    // checkDirect can hit or the root can expand
    const bool rmeta = s.remote_meta && (rbeg & ADJX_REMOTE) && !s.relflags;
    o.dest = s.remote_meta ? ((rbeg & ADJX_REMOTE) ? (rbeg & 0xFFu) : s.shard_rank) : (s.nowner ? s.nowner[node] : 0u);
    // otherwise signatures are built from this rank's rows: only a locally owned node's rules a probe out
    // an inlined slot (a short local check row) holds the row itself instead of its signature: exact
    const uint32_t icnt = rsl ? nslot_inline(rsl->pad1) : 0u;
    const bool sigm = icnt ? (subj != NONE && nslot_inline_has(icnt, rsl->pad1, rsl->sig, subj))
                           : sig_maybe(rsig_lo, rsig, subj_sig(subj));
    const bool may = subj == NONE || (o.dest != s.shard_rank && !rmeta) || sigm;
    if (rmeta && subj != NONE && !may && (rlen == 0 || d < 2)) o.act = false;
    o.r = kg_frec{(s.shard_rank << Q_BITS) | i, node, subj, d | (may ? 0 : D_NOPROBE)};
    if (o.dest == s.shard_rank && !s.relflags) {
      // a locally owned root without a namespace program (as shard_child): checkDirect here, a
      // record only if the root can expand
      if (may && d >= 1 && subj != NONE && nslot_probe(s, rsl, node, subj)) {
        res[i] = KG_IS_MEMBER;
        o.act = false;
      } else if (rlen == 0 || d < 2) {
        o.act = false;
      } else {
        o.r.depth = d | D_NOPROBE;
      }
    }
  }
  o.dsplit = d;
  o.ssubj = subj;
  // what the backward phase needs of a query that escalates: root, subject, depth
  if (qinfo) qinfo[i] = make_uint4(node, subj, (uint32_t)d, o.act ? 1u : 0u);
  return o;
}

// SEED_Q queries per thread: query (blockIdx * SEED_Q + j) * 256 + threadIdx (coalesced per j).
constexpr int SEED_Q = 4;
__global__ __launch_bounds__(256) void k_shard_seed(DevSnap s, const kg_query* __restrict__ q, uint32_t n,
                                                    int32_t global, kg_frec* out, uint64_t cap, uint32_t* counts,
                                                    uint8_t* res, uint32_t* err, const uint32_t* __restrict__ held,
                                                    uint32_t held_n, ShardFormula F, uint4* qinfo) {
  bool act[SEED_Q];
  uint32_t dest[SEED_Q];
  kg_frec rec[SEED_Q];
  SeedQ sq[SEED_Q];
#pragma unroll
  for (int j = 0; j < SEED_Q; j++) {
    const uint32_t i = (blockIdx.x * SEED_Q + j) * blockDim.x + threadIdx.x;
    sq[j] = seed_query(s, q, i, n, global, res, err, held, held_n, F, qinfo);
    act[j] = sq[j].act;
    dest[j] = sq[j].dest;
    rec[j] = sq[j].r;
  }
  emit_q<SEED_Q>(act, dest, rec, out, cap, counts, s.shard_n);
  // split queries: the own part (slot 0, the node's rows as a plain node) and every leaf (slot 1 + j),
  // each the checkIsAllowed of its node at the query's depth; a part without a node is NotMember
  if (!F.fidx) return;  // uniform over the grid
  for (int j = 0; j < SEED_Q; j++) {
    const uint32_t i = (blockIdx.x * SEED_Q + j) * blockDim.x + threadIdx.x;
    const SeedQ& o = sq[j];
    for (uint32_t k = 0; k < F.k; k++) {  // uniform trip count: emit needs every thread
      bool pa = false;
      uint32_t pd = 0;
      kg_frec pr{};
      if (o.split && (o.ssubj != NONE || s.relflags)) {
        const FPlan& P = F.plans[F.ref[i]];
        uint32_t pn = NONE;
        if (k == 0) pn = nmap_find(s, o.x.t.ns, o.x.t.rel, o.x.t.obj);
        else if (k - 1 < P.n_leaves) pn = nmap_find(s, o.x.t.ns, P.leaf[k - 1], o.x.t.obj);
        if (pn != NONE) {
          pa = true;
          pd = s.nowner ? s.nowner[pn] : 0u;
          const uint32_t slot = n + i * F.k + k;
          pr = kg_frec{(s.shard_rank << Q_BITS) | slot, pn, o.ssubj, o.dsplit | (k == 0 ? D_OWN : 0)};
        }
      }
      emit(pa, pd, pr, out, cap, counts, s.shard_n);
    }
  }
}

// One set-adjacency edge (parent record pr -> child ax) of an expansion: the child's record for its
// owner, a hit / error report for the query's home, or nothing.
__device__ __forceinline__ void shard_child(const DevSnap& s, const kg_frec& pr, const AdjX& ax, uint32_t me,
                                            uint8_t* res, uint32_t* err, kg_frec& c, uint32_t& dest, bool& send) {
  const uint32_t child = ax.node;
  if (pr.depth >= 2) {
    if (s.remote_meta) {
      dest = (ax.begin & ADJX_REMOTE) ? (ax.begin & 0xFFu) : me;
      if (dest != me && !s.relflags) {
        // a remote child with its owner's row length and signature (remote_meta): the same decision
        // as for a local one, taken here -- a record goes out only if the owner's checkDirect can hit
        // (it probes) or the child can still expand; the rest never travel.  With a namespace
        // program every child travels (the owner checks its relation for errors)
        const bool may = pr.subj != NONE && sig_maybe(ax.lsig, ax.sig, subj_sig(pr.subj));
        if (may || (adjx_len16(ax) && pr.depth >= 3)) {
          c = kg_frec{pr.q, child, pr.subj, (pr.depth - 1) | (may ? 0 : D_NOPROBE)};
          send = true;
        }
        return;
      }
    } else {
      dest = s.nowner ? s.nowner[child] : 0u;
    }
    if (dest == me && !s.relflags) {
      // a locally owned child without a namespace program: its checkDirect (depth - 2 >= 0) is
      // probed here, and a record goes out only if the child can still expand (a set row and
      // depth - 1 >= 2) -- leaves never travel or touch the visited table.  Results are
      // unchanged (membership is monotone and nothing can end as an error without a program);
      // a hit only lands one level earlier.
      const bool hit =
          pr.subj != NONE && sig_maybe(ax.lsig, ax.sig, subj_sig(pr.subj)) && dset_probe(s, child, pr.subj);
      const uint32_t alen = adjx_len16(ax);  // exact below ADJX_LEN_SAT
      if (hit && (pr.q >> Q_BITS) == me) {
        res[pr.q & Q_MASK] = KG_IS_MEMBER;
      } else if (hit) {
        c = kg_frec{pr.q, KG_FREC_HIT, 0u, 0};
        dest = pr.q >> Q_BITS;
        send = true;
      } else if (alen && pr.depth >= 3) {
        c = kg_frec{pr.q, child, pr.subj, (pr.depth - 1) | D_NOPROBE};
        send = true;
      }
    } else {
      // signatures are built from this rank's rows: only a locally owned child's rules a probe out
      const bool may = pr.subj == NONE || dest != me || sig_maybe(ax.lsig, ax.sig, subj_sig(pr.subj));
      c = kg_frec{pr.q, child, pr.subj, (pr.depth - 1) | (may ? 0 : D_NOPROBE)};
      send = true;
    }
  } else if (node_bad(s, child)) {  // a depth-0 child with a rewrite
    if ((pr.q >> Q_BITS) == me) {
      atomicMax(&err[pr.q & Q_MASK], (uint32_t)KG_ERR_NOT_IMPLEMENTED);
    } else {
      c = kg_frec{pr.q, KG_FREC_ERR, (uint32_t)KG_ERR_NOT_IMPLEMENTED, 0};
      dest = pr.q >> Q_BITS;
      send = true;
    }
  }
}

// ---- backward phase (escalated queries, snapshots without a namespace program)
// The reverse search of the single-GPU backward tier (kg_check.hip k_back) across ranks: a path
// root -> ... -> N of k <= D - 1 set hops ending in a holder N of the subject (a row of N holds it)
// exists iff the root is met within D - 1 reverse hops from the holders.  Backward records are
// (q, node, root, rem): node lies `D - 1 - rem` reverse hops from a holder.  A node's parents sit in
// the rows of their owners, so every rank keeps the reverse set-adjacency of ITS rows (radj: the
// local parents of any node) and every rank sees every backward record -- the driver all-gathers a
// level's records instead of exchanging buckets.  Each (q, node) is emitted by the owner of the
// parent row only, the root test is a compare at the sender, and the first arrival of (q, node) is
// at its smallest distance (level order), as in the forward phase.

// One reverse edge (record pr at node N -> parent P of N held in this rank's rows).
__device__ __forceinline__ void back_child(const DevSnap& s, const kg_frec& pr, uint32_t parent, uint32_t me,
                                           uint8_t* res, kg_frec& c, bool& send) {
  if (parent == pr.subj) {  // the root: a path of D - 1 - (rem - 1) <= D - 1 hops
    if ((pr.q >> Q_BITS) == me) res[pr.q & Q_MASK] = KG_IS_MEMBER;
    else {
      c = kg_frec{pr.q, KG_FREC_HIT, 0u, 0};
      send = true;
    }
  } else if (pr.depth >= 2) {  // the parent's own parents are still within D - 1 hops
    c = kg_frec{pr.q, parent, pr.subj, pr.depth - 1};
    send = true;
  }
}

// Segmented input (n_seg > 1: the receive buffer of a fixed-split all-to-all or all-gather -- segment k
// holds min(d_n_in[k], seg_cap) records from in[k * seg_cap]): every thread of the workgroup calls
// seg_total once (it stages the segments' prefix sums in LDS) and seg_src per record.
__device__ __forceinline__ uint64_t seg_total(uint64_t* s_segpre, uint32_t n_seg, const uint32_t* d_n_in,
                                              uint64_t seg_cap) {
  if (threadIdx.x == 0) {
    uint64_t a = 0;
    for (uint32_t k = 0; k < n_seg; k++) {
      s_segpre[k] = a;
      a += min((uint64_t)d_n_in[k], seg_cap);
    }
    s_segpre[n_seg] = a;
  }
  __syncthreads();
  return s_segpre[n_seg];
}

__device__ __forceinline__ uint64_t seg_src(const uint64_t* s_segpre, uint32_t n_seg, uint64_t seg_cap, uint64_t i) {
  uint32_t k = 0;
  while (k + 1 < n_seg && s_segpre[k + 1] <= i) k++;
  return (uint64_t)k * seg_cap + (i - s_segpre[k]);
}

// One workgroup handles 256 received records per iteration; their set rows are expanded
// edge-parallel (block scan of the row lengths, LDS owner search).  A row longer than SHARD_HEAVY
// (a hub) is not expanded by its workgroup -- one workgroup would hold the level for the whole row --
// but queued for k_shard_heavy, which spreads its edges over the grid.  (Expanding every row that
// way instead -- an expansion list walked edge-parallel by a second kernel -- measured slower: the
// in-workgroup expansion overlaps other workgroups' record processing, profiles/r2s8_*.)
// Segmented input (n_seg > 1): the receive buffer of a fixed-split all-to-all -- segment k holds
// d_n_in[k] records (clamped to seg_cap) from in[k * seg_cap]; the level walks their concatenation.
// (The compiler's choice of registers: forcing 6 or 8 waves per SIMD -- round 5's "shard_level_occ"
// knob -- measured no better, profiles/r5k_level_occupancy_pack_ab.jsonl.)
__global__ __launch_bounds__(256) void k_shard_level(DevSnap s, const kg_frec* __restrict__ in, uint64_t n_bound,
                                                     const uint32_t* d_n_in, kg_frec* out, uint64_t cap, uint32_t* counts, uint8_t* res,
                                                     uint32_t* err, uint64_t* vis, uint64_t vmask,
                                                     const uint32_t* __restrict__ done, uint32_t done_wpr,
                                                     HeavyList heavy,
                                                     uint32_t* qcnt, uint32_t budget, uint32_t n_seg,
                                                     uint64_t seg_cap, uint32_t heavy_min, uint32_t out_sub,
                                                     uint32_t res_done) {
  __shared__ uint32_t s_pref[256], s_wsum[4];
  __shared__ uint64_t s_rb[256];
  __shared__ kg_frec s_rec[256];
  __shared__ uint64_t s_segpre[KG_SHARD_MAX_RANKS + 1];
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t me = s.shard_rank;
  // record count: from the previous level's counter on the device (clamped to the bucket: a count
  // past it means dropped records, which the caller's overflow check turns into a rerun)
  const uint64_t n_in =
      n_seg > 1 ? seg_total(s_segpre, n_seg, d_n_in, seg_cap) : (d_n_in ? min((uint64_t)*d_n_in, n_bound) : n_bound);
  for (uint64_t base = (uint64_t)blockIdx.x * 256; base < n_in; base += (uint64_t)gridDim.x * 256) {
    const uint64_t i = base + tid;
    kg_frec r{0, NONE, 0, 0};
    bool hit_out = false, err_out = false, esc_out = false;
    uint64_t rb = 0, len = 0;
    if (i < n_in) {
      r = in[n_seg > 1 ? seg_src(s_segpre, n_seg, seg_cap, i) : i];
      const bool probe = !(r.depth & D_NOPROBE), own = (r.depth & D_OWN) != 0;
      r.depth &= D_MASK;
      if (r.node == KG_FREC_HIT) {
        if ((r.q >> Q_BITS) == me) res[r.q & Q_MASK] = KG_IS_MEMBER;
      } else if (r.node == KG_FREC_ESC) {
        if ((r.q >> Q_BITS) == me) atomicOr(&err[r.q & Q_MASK], ESC_BIT);
      } else if (r.node == KG_FREC_ERR) {
        if ((r.q >> Q_BITS) == me) atomicMax(&err[r.q & Q_MASK], r.subj);
      } else if (done && ((r.q & Q_MASK) >> 5) < done_wpr &&
                 ((done[(size_t)(r.q >> Q_BITS) * done_wpr + ((r.q & Q_MASK) >> 5)] >> (r.q & 31)) & 1u)) {
        // answered IsMember by an earlier level: nothing more to do for this query
      } else if (res_done && (r.q >> Q_BITS) == me && res[r.q & Q_MASK] == KG_IS_MEMBER) {
        // the same read from the results themselves (one rank: every query is this rank's; a result
        // set by this very level only prunes earlier)
      } else {
        // the probe's first dset bucket and the node's set-row bounds are loaded before the visited
        // insert returns (all three in one round trip; a node already visited just ignores them)
        const bool want_p = probe && r.depth >= 1 && r.subj != NONE;
        const uint64_t dkey = dset_key(r.node, r.subj);
        const ulonglong2 pb = *reinterpret_cast<const ulonglong2*>(
            s.dset + (want_p ? dset_home(dkey, s.dset_nb) : 0ull) * DSET_BUCKET);
        const uint64_t a0 = s.adj_off[r.node], a1 = s.adj_off[r.node + 1];
        const uint64_t xb = s.adjx_off ? (uint64_t)s.adjx_off[r.node] : a0;  // the row's begin in adjx
        const uint64_t vkey = ((uint64_t)r.q << 32) | r.node;
        const int ins = sv_insert(vis, vmask, vkey);
        // the flags word follows the (sub-)bucket counters: counts[out_sub] in the one-rank sub mode
        if (ins < 0) atomicOr(&counts[out_sub > 1 ? out_sub : s.shard_n], 2u);
        if (ins > 0 && !own && node_bad(s, r.node)) {  // a rewrite / undeclared relation
          if ((r.q >> Q_BITS) == me) atomicMax(&err[r.q & Q_MASK], (uint32_t)KG_ERR_NOT_IMPLEMENTED);
          else err_out = true;
        } else if (ins > 0) {
          // checkDirect(depth - 1): the first bucket, then (rarely, load <= 0.25) the rest of the chain
          bool direct = want_p && (pb.x == dkey || pb.y == dkey);
          if (want_p && !direct && pb.y != EMPTY64) direct = dset_probe(s, r.node, r.subj);
          if (direct) {
            if ((r.q >> Q_BITS) == me) res[r.q & Q_MASK] = KG_IS_MEMBER;
            else hit_out = true;
          } else if (r.depth >= 2 || (r.depth == 1 && s.relflags)) {
            // children at depth - 1 >= 1 can still be probed; children at depth 0 cannot, but
            // checkIsAllowed(child, 0) still evaluates astRelationFor (engine.go:199-206), so with a
            // namespace program their relation flags are checked (shard_child) for the error report
            rb = xb;
            len = a1 - a0;
            if (len && budget) {  // escalation: this rank's set-edge count of the query passes the budget
              const uint32_t add = (uint32_t)min(len, (uint64_t)budget);
              const uint32_t old = atomicAdd(&qcnt[mix64(r.q) & ((1u << QCNT_LOG2) - 1)], add);
              if (old + add >= budget) {
                // escalated: the backward phase answers it.  Counters are hashed by query, so a slot can
                // be past the budget because of ANOTHER query: every record whose row is dropped marks its
                // own query (not only the one that crossed the threshold) -- a dropped row of an unmarked
                // query would end its walk as NotMember (round 5: 2-4 missed members in 20 k C4 checks at
                // budget 2)
                if ((r.q >> Q_BITS) == me) atomicOr(&err[r.q & Q_MASK], ESC_BIT);
                else esc_out = true;
                len = 0;
              }
            }
          }
        }
      }
    }
    // set rows longer than heavy_min go to the level's hub list (k_shard_heavy walks them flat over the
    // grid); with heavy_min 0 every expansion does, and this workgroup only handles its records
    if (heavy_append(heavy, len > heavy_min, HeavyRow{r, rb, 0ull, (uint32_t)len, 0u})) len = 0;
    // hit and error reports go to the query's home
    kg_frec hr{r.q, err_out ? KG_FREC_ERR : (esc_out ? KG_FREC_ESC : KG_FREC_HIT),
               err_out ? (uint32_t)KG_ERR_NOT_IMPLEMENTED : 0u, 0};
    emit(hit_out || err_out || esc_out, r.q >> Q_BITS, hr, out, cap, counts, s.shard_n, out_sub);
    // expansion
    s_rb[tid] = rb;
    s_rec[tid] = r;
    uint32_t total;
    uint32_t v = (uint32_t)len, x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) s_wsum[wave] = v;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) before += s_wsum[w];
      total += s_wsum[w];
    }
    s_pref[tid] = before + v - x;
    __syncthreads();
    for (uint32_t eb = 0; eb < total; eb += 256) {
      const uint32_t e = eb + tid;
      kg_frec c{};
      uint32_t dest = 0;
      bool send = false;
      if (e < total) {
        const int own = owner_search(s_pref, 256, e);
        shard_child(s, s_rec[own], s.adjx[s_rb[own] + (e - s_pref[own])], me, res, err, c, dest, send);
      }
      emit(send, dest, c, out, cap, counts, s.shard_n, out_sub);
    }
    __syncthreads();
  }
}

// Escalated queries of this rank still open after the forward phase, as backward list entries
// (q, root, subject, depth); they go to every rank.  The (query, node) table is cleared for the
// backward keys.
__global__ __launch_bounds__(256) void k_shard_back_list(uint32_t n, const uint8_t* __restrict__ res,
                                                         const uint32_t* __restrict__ err, const uint4* __restrict__ qinfo,
                                                         uint32_t me, kg_frec* out, uint64_t cap, uint32_t* counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool act = false;
  kg_frec r{};
  if (i < n && (err[i] & ESC_BIT) && res[i] != KG_IS_MEMBER) {
    const uint4 qi = qinfo[i];
    // an escalated query was seeded (qi.w), has a root, a subject and depth >= 2 (it expanded)
    act = qi.w != 0 && qi.y != NONE;
    r = kg_frec{(me << Q_BITS) | i, qi.x, qi.y, (int32_t)qi.z};
  }
  emit(act, 0u, r, out, cap, counts, 1u);
}

// The final forward phase: this rank's queries that escalated out of both the forward and the
// backward budget, re-seeded at their roots (their owners probe the root again).
__global__ __launch_bounds__(256) void k_shard_refwd_seed(DevSnap s, uint32_t n, const uint8_t* __restrict__ res,
                                                          const uint32_t* __restrict__ err,
                                                          const uint4* __restrict__ qinfo, kg_frec* out, uint64_t cap,
                                                          uint32_t* counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool act = false;
  kg_frec r{};
  uint32_t dest = 0;
  if (i < n && (err[i] & ESC2_BIT) && res[i] != KG_IS_MEMBER) {
    const uint4 qi = qinfo[i];
    act = qi.w != 0;
    r = kg_frec{(s.shard_rank << Q_BITS) | i, qi.x, qi.y, (int32_t)qi.z};
    dest = act && s.nowner ? s.nowner[qi.x] : 0u;
  }
  emit(act, dest, r, out, cap, counts, s.shard_n);
}

// Level 0 of the backward phase: for every listed query, this rank's holders N of its subject
// (rows of N hold it) at distance 0, as records (q, N, root, D - 1).  The holder lists are walked
// edge-parallel like set rows.  A holder that is the root would be a direct tuple, answered by the
// forward phase's root probe.
__global__ __launch_bounds__(256) void k_shard_back_seed(DevSnap s, const kg_frec* __restrict__ list, uint64_t m_bound,
                                                         const uint32_t* d_m, kg_frec* out, uint64_t cap,
                                                         uint32_t* counts, uint32_t n_seg, uint64_t seg_cap,
                                                         uint32_t budget) {
  __shared__ uint32_t s_pref[256], s_wsum[4], s_first[256];
  __shared__ kg_frec s_rec[256];
  __shared__ uint64_t s_segpre[KG_SHARD_MAX_RANKS + 1];
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t m = n_seg > 1 ? seg_total(s_segpre, n_seg, d_m, seg_cap) : (d_m ? min((uint64_t)*d_m, m_bound) : m_bound);
  for (uint64_t base = (uint64_t)blockIdx.x * 256; base < m; base += (uint64_t)gridDim.x * 256) {
    const uint64_t i = base + tid;
    uint32_t cnt = 0, first = 0;
    bool esc = false;
    kg_frec r{0, NONE, NONE, 0};
    if (i < m) {
      const kg_frec e = list[n_seg > 1 ? seg_src(s_segpre, n_seg, seg_cap, i) : i];
      if (e.depth >= 2) {  // holders at distance 0 lead to the root within D - 1 hops only if D - 1 >= 1
        const uint2 h = holders_find(s, e.subj);
        first = h.x;
        cnt = h.y;
        r = kg_frec{e.q, NONE, e.node, e.depth - 1};  // subj carries the root from here on
        // a subject held by more rows on this rank than the reverse-edge budget allows (a popular
        // subject: its reverse search would start wider than the forward walk it replaces) goes
        // straight to the final forward phase -- an ESC report to its home, through the all-gather
        if (budget && cnt > budget) {
          cnt = 0;
          esc = true;
        }
      }
    }
    emit(esc, 0u, kg_frec{r.q, KG_FREC_ESC, 0u, 0}, out, cap, counts, 1u);
    s_first[tid] = first;
    s_rec[tid] = r;
    uint32_t v = cnt, x = v, total = 0, before = 0;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) s_wsum[wave] = v;
    __syncthreads();
    for (int w = 0; w < 4; w++) {
      if (w < wave) before += s_wsum[w];
      total += s_wsum[w];
    }
    s_pref[tid] = before + v - x;
    __syncthreads();
    for (uint32_t eb = 0; eb < total; eb += 256) {
      const uint32_t e = eb + tid;
      kg_frec c{};
      bool send = false;
      if (e < total) {
        const int own = owner_search(s_pref, 256, e);
        const kg_frec& pr = s_rec[own];
        c = kg_frec{pr.q, s.hold[s_first[own] + (e - s_pref[own])], pr.subj, pr.depth};
        send = c.node != pr.subj;
      }
      emit(send, 0u, c, out, cap, counts, 1u);
    }
    __syncthreads();
  }
}

// One backward level over the all-gathered records: hit reports for this rank's queries, else
// dedup (query, node) and expand this rank's parents of the node (reverse rows longer than
// SHARD_HEAVY go to k_shard_heavy).  Records go to one bucket (the next level's all-gather).
__global__ __launch_bounds__(256) void k_shard_back_level(DevSnap s, const kg_frec* __restrict__ in, uint64_t n_bound,
                                                          const uint32_t* d_n_in, kg_frec* out, uint64_t cap,
                                                          uint32_t* counts, uint8_t* res, uint32_t* err, uint64_t* vis,
                                                          uint64_t vmask, const uint32_t* __restrict__ done,
                                                          uint32_t done_wpr, HeavyList heavy, uint32_t* qcnt,
                                                          uint32_t budget,
                                                          uint32_t n_seg, uint64_t seg_cap) {
  __shared__ uint32_t s_pref[256], s_wsum[4];
  __shared__ uint64_t s_rb[256];
  __shared__ kg_frec s_rec[256];
  __shared__ uint64_t s_segpre[KG_SHARD_MAX_RANKS + 1];
  const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t me = s.shard_rank;
  const uint64_t n_in =
      n_seg > 1 ? seg_total(s_segpre, n_seg, d_n_in, seg_cap) : (d_n_in ? min((uint64_t)*d_n_in, n_bound) : n_bound);
  for (uint64_t base = (uint64_t)blockIdx.x * 256; base < n_in; base += (uint64_t)gridDim.x * 256) {
    const uint64_t i = base + tid;
    kg_frec r{0, NONE, 0, 0};
    uint64_t rb = 0, len = 0;
    bool esc_out = false;
    if (i < n_in) {
      r = in[n_seg > 1 ? seg_src(s_segpre, n_seg, seg_cap, i) : i];
      if (r.node == KG_FREC_HIT) {
        if ((r.q >> Q_BITS) == me) res[r.q & Q_MASK] = KG_IS_MEMBER;
      } else if (r.node == KG_FREC_ESC) {
        if ((r.q >> Q_BITS) == me) atomicOr(&err[r.q & Q_MASK], ESC2_BIT);
      } else if (done && ((r.q & Q_MASK) >> 5) < done_wpr &&
                 ((done[(size_t)(r.q >> Q_BITS) * done_wpr + ((r.q & Q_MASK) >> 5)] >> (r.q & 31)) & 1u)) {
        // answered IsMember by an earlier level
      } else {
        const uint64_t vkey = ((uint64_t)r.q << 32) | r.node;
        const int ins = sv_insert(vis, vmask, vkey);
        if (ins < 0) atomicOr(&counts[1], 2u);
        if (ins > 0 && r.depth >= 1) {
          rb = s.radj_off[r.node];
          len = s.radj_off[r.node + 1] - rb;
          if (len && budget) {  // the reverse search's own budget: past it, the final forward phase
            const uint32_t add = (uint32_t)min(len, (uint64_t)budget);
            const uint32_t old = atomicAdd(&qcnt[mix64(r.q) & ((1u << QCNT_LOG2) - 1)], add);
            if (old + add >= budget) {  // (every query whose row is dropped is marked: see k_shard_level)
              if ((r.q >> Q_BITS) == me) atomicOr(&err[r.q & Q_MASK], ESC2_BIT);
              else esc_out = true;
              len = 0;
            }
          }
        }
      }
    }
    if (heavy_append(heavy, len > SHARD_HEAVY, HeavyRow{r, rb, 0ull, (uint32_t)len, 1u})) len = 0;
    emit(esc_out, 0u, kg_frec{r.q, KG_FREC_ESC, 0u, 0}, out, cap, counts, 1u);  // to the home, via the all-gather
    s_rb[tid] = rb;
    s_rec[tid] = r;
    uint32_t v = (uint32_t)len, x = v, total = 0, before = 0;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) s_wsum[wave] = v;
    __syncthreads();
    for (int w = 0; w < 4; w++) {
      if (w < wave) before += s_wsum[w];
      total += s_wsum[w];
    }
    s_pref[tid] = before + v - x;
    __syncthreads();
    for (uint32_t eb = 0; eb < total; eb += 256) {
      const uint32_t e = eb + tid;
      kg_frec c{};
      bool send = false;
      if (e < total) {
        const int own = owner_search(s_pref, 256, e);
        back_child(s, s_rec[own], s.radj[s_rb[own] + (e - s_pref[own])], me, res, c, send);
      }
      emit(send, 0u, c, out, cap, counts, 1u);
    }
    __syncthreads();
  }
}

// The hub rows a level queued, walked flat: HEAVY_TILE-edge tiles of the level's hub-edge space over
// the whole grid, each tile's first row from the tile map, the row of each edge by a search over the
// tile's rows staged in LDS.
__global__ __launch_bounds__(256) void k_shard_heavy(DevSnap s, HeavyList heavy, kg_frec* out, uint64_t cap,
                                                     uint32_t* counts, uint8_t* res, uint32_t* err, uint32_t nranks,
                                                     uint32_t out_sub, uint32_t* zero_counts,
                                                     uint32_t zero_n, unsigned long long* zero_pk,
                                                     uint32_t* maxacc) {
  static_assert(HEAVY_TILE == 256, "one edge per thread");
  __shared__ uint32_t s_r0;
  __shared__ uint64_t s_e0[HEAVY_TILE + 1];
  // kg_shard_levels: the next level's bucket counters and hub-list counter, free since the level
  // before this one read them (what a separate k_shard_prep launch per level did); the largest
  // sub-bucket count goes to *maxacc first (the counters count past the cap: what a rerun needs)
  if (blockIdx.x == 0) {
    if (zero_counts && threadIdx.x < zero_n) {
      if (maxacc) atomicMax(maxacc, zero_counts[threadIdx.x]);
      zero_counts[threadIdx.x] = 0;
    }
    if (zero_pk && threadIdx.x == 0) *zero_pk = 0;
  }
  const uint32_t nh = (uint32_t)min((unsigned long long)heavy.cap, *heavy.pk >> HEAVY_EDGE_BITS), me = s.shard_rank;
  if (nh == 0) return;
  const HeavyRow last = heavy.rows[nh - 1];
  const uint64_t total = last.e0 + last.len;  // rows past the cap were expanded by their workgroup
  for (uint64_t t0 = (uint64_t)blockIdx.x * HEAVY_TILE; t0 < total; t0 += (uint64_t)gridDim.x * HEAVY_TILE) {
    if (threadIdx.x == 0) {
      const uint64_t t = t0 / HEAVY_TILE;
      uint32_t r0 = 0;
      if (t < HEAVY_TF_CAP) {
        r0 = heavy.tf[t];
      } else {  // past the tile map: the last row starting at or before t0
        uint32_t lo = 0, hi = nh;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (heavy.rows[mid].e0 <= t0) lo = mid;
          else hi = mid;
        }
        r0 = lo;
      }
      s_r0 = r0;
    }
    __syncthreads();
    // the tile's rows (every queued row has >= 1 edge, so at most HEAVY_TILE + 1 of them): their first
    // edges staged in LDS, each thread's row by binary search there
    const uint32_t r0 = s_r0, nr = min(nh - r0, HEAVY_TILE + 1u);
    for (uint32_t k = threadIdx.x; k < nr; k += HEAVY_TILE) s_e0[k] = heavy.rows[r0 + k].e0;
    __syncthreads();
    const uint64_t e = t0 + threadIdx.x;
    kg_frec c{};
    uint32_t dest = 0;
    bool send = false;
    if (e < total) {
      uint32_t lo = 0, hi = nr;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_e0[mid] <= e) lo = mid;
        else hi = mid;
      }
      const HeavyRow H = heavy.rows[r0 + lo];
      const uint64_t k = e - H.e0;
      if (H.pad) back_child(s, H.r, s.radj[H.rb + k], me, res, c, send);  // a reverse row (backward phase)
      else shard_child(s, H.r, s.adjx[H.rb + k], me, res, err, c, dest, send);
    }
    emit(send, dest, c, out, cap, counts, nranks, out_sub);  // ends with a barrier: s_r0 is free again
  }
}

// Done bitmap of this rank's queries (IsMember so far, or an err bit of esc_mask: escalated out of
// the current phase), one word per thread.
__global__ void k_shard_done(uint32_t n, const uint8_t* __restrict__ res, const uint32_t* __restrict__ err,
                             uint32_t esc_mask, uint32_t words, uint32_t* __restrict__ bits) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  uint32_t b = 0;
  for (uint32_t k = 0; k < 32; k++) {
    const uint32_t i = w * 32 + k;
    if (i < n && (res[i] == KG_IS_MEMBER || (esc_mask && (err[i] & esc_mask)))) b |= 1u << k;
  }
  bits[w] = b;
}

// One launch before each exchange of the N > 1 protocol (kg_shard_comm.hip), replacing four: block 0's
// first wave folds the outgoing bucket counts into the batch accumulators (acc: flags | largest | sent
// | sent to peers; lvl: this exchange's largest bucket), block 0 zeroes the level's output counters and
// the hub-row head, and every thread packs one word of the done bitmap (words = 0: none).
__global__ void k_shard_pre(const uint32_t* __restrict__ cc, uint32_t N, uint32_t B, uint32_t me,
                            unsigned long long* acc, unsigned long long* lvl, uint32_t* zero_counts,
                            unsigned long long* heavy_pk, uint32_t n, const uint8_t* __restrict__ res,
                            const uint32_t* __restrict__ err, uint32_t esc_mask, uint32_t words, uint32_t* bits) {
  if (blockIdx.x == 0) {
    if (threadIdx.x < 64) {
      const uint32_t i = threadIdx.x;
      const uint32_t v = i < N ? cc[i] : 0u;
      unsigned long long fl = (i < N && v > B) ? 1ull : 0ull, mx = v, sum = v, wire = i != me ? v : 0u;
      for (int off = 32; off; off >>= 1) {
        fl |= __shfl_xor(fl, off, 64);
        mx = max(mx, __shfl_xor(mx, off, 64));
        sum += __shfl_xor(sum, off, 64);
        wire += __shfl_xor(wire, off, 64);
      }
      if (i == 0) {
        acc[0] |= fl | cc[N];
        acc[1] = max(acc[1], mx);
        acc[2] += sum;
        acc[3] += wire;
        *lvl = max(*lvl, mx);
      }
    }
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) zero_counts[i] = 0;
    if (threadIdx.x == 0 && heavy_pk) *heavy_pk = 0;
  }
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w < words) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < 32; k++) {
      const uint32_t i = w * 32 + k;
      if (i < n && (res[i] == KG_IS_MEMBER || (esc_mask && (err[i] & esc_mask)))) b |= 1u << k;
    }
    bits[w] = b;
  }
}

int shard_pre_level(Snapshot* s, hipStream_t stream, const uint32_t* d_cur, uint32_t N, uint32_t B, uint32_t me,
                    unsigned long long* acc, unsigned long long* lvl, uint32_t* d_next_counts, size_t n,
                    const uint8_t* d_res, const uint32_t* d_err, int with_esc, uint32_t* d_bits, uint32_t words) {
  HIPC(hipSetDevice(s->device));
  if (N > 64) return set_error(-2, "shard_pre_level: at most 64 ranks");
  if (words && words < (n + 31) / 32) return set_error(-2, "done bitmap too small (%u words for %zu queries)", words, n);
  const uint32_t blocks = std::max<uint32_t>(1, (words + 255) / 256);
  hipLaunchKernelGGL(k_shard_pre, dim3(blocks), dim3(256), 0, stream, d_cur, N, B, me, acc, lvl, d_next_counts,
                     shard_heavy_head(s, stream), (uint32_t)n, d_res, d_err, with_esc ? ESC_BIT : 0u, words, d_bits);
  HIPC(hipGetLastError());
  return 0;
}

// One launch before each level of kg_shard_levels: the done bitmap from the results so far
// (k_shard_done's packing; words = 0 at the first level) and the level's zeroed bucket counter and
// hub-row count -- what the per-level driver did with a kernel and two fills.
__global__ void k_shard_prep(uint32_t n, const uint8_t* __restrict__ res, const uint32_t* __restrict__ err,
                             uint32_t esc_mask, uint32_t words, uint32_t* __restrict__ bits, uint32_t* counts,
                             uint32_t n_sub, unsigned long long* heavy_pk, uint32_t* maxacc) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w < n_sub) {  // the level's (sub-)bucket counters; the flags word after them accumulates
    atomicMax(maxacc, counts[w]);
    counts[w] = 0;
  }
  if (w == 0) *heavy_pk = 0;
  if (w >= words) return;
  uint32_t b = 0;
  for (uint32_t k = 0; k < 32; k++) {
    const uint32_t i = w * 32 + k;
    if (i < n && (res[i] == KG_IS_MEMBER || (esc_mask && (err[i] & esc_mask)))) b |= 1u << k;
  }
  bits[w] = b;
}

// After kg_shard_levels: the caller's view of the two level buffers -- records left in the last one
// (the sum of its sub-bucket counters) and the flags accumulated in both.
// *need (if given) = the bucket size every level's sub-buckets would have fit in: n_sub x the largest
// sub-bucket count of the loop (the counters keep counting past a full segment), and at least the
// seed's record count (*seed, the loop's first input; read before counts_end is written).
__global__ void k_shard_fold(const uint32_t* __restrict__ sub_end, const uint32_t* __restrict__ sub_other,
                             uint32_t n_sub, uint32_t* counts_end, uint32_t* counts0, const uint32_t* maxacc,
                             const uint32_t* seed, unsigned long long* need) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const unsigned long long seeded = *seed;
  uint32_t left = 0, mx = *maxacc;
  for (uint32_t k = 0; k < n_sub; k++) {
    left += sub_end[k];
    mx = max(mx, max(sub_end[k], sub_other[k]));
  }
  counts_end[0] = left;
  counts0[1] |= sub_end[n_sub] | sub_other[n_sub];
  if (need) *need = max(*need, max((unsigned long long)mx * n_sub, seeded));
}

__global__ void k_shard_finish(uint32_t n, uint8_t* res, uint32_t* err, ShardFormula F) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  err[i] &= ~(ESC_BIT | ESC2_BIT);  // the escalation markers are batch-internal
  if (F.ref && F.ref[i] != NONE) {  // own part | formula over the leaves (kg_formula.hip)
    const FPlan& P = F.plans[F.ref[i]];
    const uint32_t base = n + i * F.k;
    uint32_t e = KG_ERR_NONE, bits = 0;
    for (uint32_t k = 0; k < 1 + P.n_leaves; k++)
      if (e == KG_ERR_NONE) e = err[base + k];
    for (uint32_t j = 0; j < P.n_leaves; j++) bits |= (res[base + 1 + j] == KG_IS_MEMBER ? 1u : 0u) << j;
    err[i] = e;
    res[i] = (res[base] == KG_IS_MEMBER || fplan_eval(P, bits)) ? KG_IS_MEMBER : KG_NOT_MEMBER;
  }
  if (err[i] != KG_ERR_NONE) res[i] = KG_ERROR;
}

// The formula split's tables for a batch of n queries (plans only when the snapshot has them).
static int shard_formula(Snapshot* s, ShardCtx* c, size_t n, ShardFormula* F) {
  *F = ShardFormula{nullptr, nullptr, 0, s->d_virt, nullptr};
  if (!s->n_fplans) return 0;
  if (n > c->ref_n) {
    if (c->ref) HIPC(hipFree(c->ref));
    c->ref = nullptr;
    c->ref_n = 0;
    HIPC(hipMalloc((void**)&c->ref, std::max<size_t>(n, 1024) * 4));
    c->ref_n = std::max<size_t>(n, 1024);
  }
  *F = ShardFormula{s->d_fidx, (const FPlan*)s->d_fplans, 1 + s->fp_leaves, s->d_virt, c->ref};
  return 0;
}

// A node that can end a check in an error, counted where a record could reach it: a set edge leads
// to it from this rank's rows (its local parents; roots are judged by the seed itself), or -- a union
// the owner found impure from its own TTU rows, a flag only the owner holds -- at its owner.  Without
// the reverse index every bad node counts.
__global__ void k_shard_bad_nodes(DevSnap s, unsigned long long* count) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = v < s.n_nodes && node_bad(s, v);
  if (bad && s.radj_off) {
    const bool reached = s.radj_off[v + 1] > s.radj_off[v];
    const uint32_t ns = s.nd_ns[v], rel = s.nd_rel[v];
    const bool vunion = s.virt && ns < s.n_ns && rel < s.n_rel && s.virt[(size_t)ns * s.n_rel + rel];
    const bool owned = !s.nowner || s.nowner[v] == s.shard_rank;
    bad = reached || (vunion && owned && s.shard_n > 1);
  }
  const uint64_t m = __ballot(bad);
  if (lane_id() == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

int shard_bad_nodes(Snapshot* s, uint64_t* count) {
  HIPC(hipSetDevice(s->device));
  *count = 0;
  if (!s->ds.n_nodes) return 0;
  unsigned long long* d = nullptr;
  HIPC(hipMalloc((void**)&d, 8));
  HIPC(hipMemsetAsync(d, 0, 8, s->stream));
  hipLaunchKernelGGL(k_shard_bad_nodes, dim3((s->ds.n_nodes + 255) / 256), dim3(256), 0, s->stream, s->ds, d);
  HIPC(hipGetLastError());
  unsigned long long h = 0;
  HIPC(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, s->stream));
  HIPC(hipStreamSynchronize(s->stream));
  HIPC(hipFree(d));
  *count = h;
  return 0;
}

// Remote child metadata (DevSnap::remote_meta).  Per node, this rank's set-row length and check-row
// signature in AdjX's lsig / sig layout: non-zero only for nodes this rank owns (a node's rows all sit
// on its owner), so a max all-reduce over the ranks leaves every rank the owners' values.
__global__ void k_shard_meta(DevSnap s, const uint64_t* __restrict__ coff, const uint32_t* __restrict__ csub,
                             uint64_t* meta) {
  for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < s.n_nodes;
       v += (uint64_t)gridDim.x * blockDim.x) {
    uint2 m = make_uint2(0u, 0u);
    for (uint64_t i = coff[v], e = coff[v + 1]; i < e && (m.x != SIG_LO || m.y != 0xFFFFFFFFu); i++) {
      const uint2 b = subj_sig(csub[i]);
      m.x |= b.x;
      m.y |= b.y;
    }
    const uint64_t len = s.adj_off[v + 1] - s.adj_off[v];
    const uint32_t lsig = (uint32_t)min(len, (uint64_t)ADJX_LEN_SAT) | (m.x & SIG_LO);
    meta[v] = (uint64_t)lsig | ((uint64_t)m.y << 32);
  }
}

// Every local set edge to a child another rank owns: the owner in `begin` (ADJX_REMOTE | rank) and the
// owner's row length and signature (all-reduced meta).  Local children keep their records.
__global__ void k_shard_adjx_remote(DevSnap s, AdjX* adjx, uint64_t n_edges, const uint64_t* __restrict__ meta) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_edges;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = adjx[e].node;
    const uint32_t o = s.nowner[c];
    if (o != s.shard_rank) {
      const uint64_t m = meta[c];
      adjx[e] = AdjX{c, ADJX_REMOTE | o, (uint32_t)m, (uint32_t)(m >> 32)};
    }
  }
}

// The node-map slot of a node another rank owns, likewise (the seed's root): beg = ADJX_REMOTE | owner,
// len and the signature words the owner's.  The slot's flags byte stays.
__global__ void k_shard_nmap_remote(DevSnap s, NSlot* nm, uint64_t slots, const uint64_t* __restrict__ meta) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * blockDim.x) {
    if (nm[i].key == EMPTY64) continue;
    const uint32_t v = nm[i].node;
    const uint32_t o = s.nowner[v];
    if (o == s.shard_rank) continue;
    const uint64_t m = meta[v];
    const uint32_t lsig = (uint32_t)m;
    nm[i].beg = ADJX_REMOTE | o;
    nm[i].len = lsig & ADJX_LEN_SAT;
    nm[i].sig = (uint32_t)(m >> 32);
    nm[i].pad1 = (nm[i].pad1 & 0xFFull) | (lsig & SIG_LO);
  }
}

int shard_meta_local(Snapshot* s, uint64_t* d_meta, hipStream_t st) {
  HIPC(hipSetDevice(s->device));
  if (!s->ds.n_nodes) return 0;
  const uint64_t* coff = s->ds.crow_off ? s->ds.crow_off : s->ds.row_off;
  const uint32_t* csub = s->ds.crow_off ? s->ds.crow_subj : s->ds.row_subj;
  hipLaunchKernelGGL(k_shard_meta, dim3((uint32_t)std::min<uint64_t>((s->ds.n_nodes + 255) / 256, 65536)), dim3(256),
                     0, st, s->ds, coff, csub, d_meta);
  HIPC(hipGetLastError());
  return 0;
}

int shard_meta_apply(Snapshot* s, const uint64_t* d_meta, hipStream_t st) {
  HIPC(hipSetDevice(s->device));
  if (s->shard_n < 2 || !s->ds.nowner) return set_error(-2, "remote child metadata: not a hash-sharded snapshot");
  if (s->n_set_edges >= ADJX_REMOTE) return 0;  // row begins need bit 31: keep the nowner reads
  if (s->n_set_edges) {
    hipLaunchKernelGGL(k_shard_adjx_remote, dim3(4096), dim3(256), 0, st, s->ds, const_cast<AdjX*>(s->ds.adjx),
                       s->n_set_edges, d_meta);
    HIPC(hipGetLastError());
  }
  if (s->ds.nmap_n) {
    hipLaunchKernelGGL(k_shard_nmap_remote, dim3(4096), dim3(256), 0, st, s->ds, const_cast<NSlot*>(s->ds.nmap),
                       s->ds.nmap_n, d_meta);
    HIPC(hipGetLastError());
  }
  HIPC(hipStreamSynchronize(st));
  s->ds.remote_meta = 1;
  return 0;
}

size_t shard_slot_limit() { return Q_MASK; }

size_t shard_result_slots(const Snapshot* s, size_t n) { return s->n_fplans ? n * (2 + (size_t)s->fp_leaves) : n; }

static int shard_vis_prepare(Snapshot* s, ShardCtx* c, hipStream_t stream, size_t n) {
  // per-batch (query, node) table of 2^shard_vis_log2 slots (kg_snapshot_tune "shard_vis",
  // default 2^23 = 64 MiB); an overflow is reported in the flags and the driver grows it
  (void)n;
  const uint64_t slots = 1ull << s->shard_vis_log2;
  if (c->vis && c->vis_slots != slots) {
    HIPC(hipFree(c->vis));
    c->vis = nullptr;
  }
  if (!c->vis) {
    HIPC(hipMalloc(&c->vis, slots * 8));
    c->vis_slots = slots;
  }
  HIPC(hipMemsetAsync(c->vis, 0xFF, c->vis_slots * 8, stream));
  if (!c->heavy) {
    HIPC(hipMalloc(&c->heavy, (size_t)SHARD_HEAVY_CAP * sizeof(HeavyRow) + 256 + HEAVY_TF_CAP * 4));
  }
  return 0;
}

// The stream's hub-row list: rows, then the packed counter, then the tile map.
static HeavyList heavy_list(ShardCtx* c) {
  HeavyRow* rows = (HeavyRow*)c->heavy;
  unsigned long long* pk = (unsigned long long*)(rows + SHARD_HEAVY_CAP);
  uint32_t* tf = (uint32_t*)((char*)pk + 256);
  return HeavyList{rows, pk, tf, SHARD_HEAVY_CAP};
}

// Escalation is on for snapshots without a namespace program (errors below the root cannot occur)
// whose reverse indexes exist, with a non-zero budget.
bool shard_escalates(const Snapshot* s) { return s->shard_budget && !s->ds.relflags && s->ds.radj; }

int shard_seed(Snapshot* s, const kg_query* d_q, size_t n, int32_t gdepth, kg_frec* d_out, size_t cap,
               uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, hipStream_t stream) {
  if (gdepth < 1) gdepth = 5;  // config.schema.json:308-315 default
  const size_t slots = shard_result_slots(s, n);
  if (slots > Q_MASK) return set_error(-2, "sharded batch too large (%zu result slots > %u)", slots, Q_MASK);
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  if (int rc = shard_vis_prepare(s, c, stream, n)) return rc;
  HIPC(hipMemsetAsync(d_counts, 0, (s->shard_n + 1) * 4, stream));
  c->final = false;
  c->gdepth = gdepth;
  uint4* qinfo = nullptr;
  if (shard_escalates(s)) {
    if (!c->qcnt) HIPC(hipMalloc(&c->qcnt, (4ull << QCNT_LOG2)));
    HIPC(hipMemsetAsync(c->qcnt, 0, (4ull << QCNT_LOG2), stream));
    if (slots > c->qinfo_n) {
      if (c->qinfo) HIPC(hipFree(c->qinfo));
      c->qinfo = nullptr;
      c->qinfo_n = 0;
      HIPC(hipMalloc(&c->qinfo, std::max<size_t>(slots, 1024) * sizeof(uint4)));
      c->qinfo_n = std::max<size_t>(slots, 1024);
    }
    qinfo = (uint4*)c->qinfo;
    if (slots > n) HIPC(hipMemsetAsync(qinfo + n, 0, (slots - n) * sizeof(uint4), stream));
  }
  ShardFormula F;
  if (shard_formula(s, c, n, &F)) return -1;
  if (slots > n) {  // the split parts' slots start NotMember / no error
    HIPC(hipMemsetAsync(d_res + n, 0, slots - n, stream));
    HIPC(hipMemsetAsync(d_err + n, 0, (slots - n) * 4, stream));
  }
  if (n) {
    const uint32_t* held = s->shard_held ? s->shard_held : s->ds.hbits;
    const uint32_t held_n = s->shard_held ? s->shard_held_n : s->ds.hbits_n;
    hipLaunchKernelGGL(k_shard_seed, dim3((uint32_t)((n + 256 * SEED_Q - 1) / (256 * SEED_Q))), dim3(256), 0, stream,
                       s->ds, d_q, (uint32_t)n,
                       gdepth, d_out, (uint64_t)cap, d_counts, d_res, d_err,
                       (s->shard_n == 1 || s->shard_held) ? held : nullptr, held_n, F, qinfo);
    HIPC(hipGetLastError());
  }
  return 0;
}

unsigned long long* shard_heavy_head(Snapshot* s, hipStream_t stream) {
  if (hipSetDevice(s->device) != hipSuccess) return nullptr;
  ShardCtx* c = s->shard_ctx(stream ? stream : s->stream);
  return c ? (unsigned long long*)heavy_list(c).pk : nullptr;
}

int shard_level(Snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out, size_t cap,
                uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done, uint32_t done_words,
                hipStream_t stream, uint32_t n_seg, size_t seg_cap, bool prezeroed) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  // the bucket sizes restart; the flags word (counts[shard_n]: dropped records, visited table full)
  // accumulates over the batch's levels, so the caller reads it once at the end.  prezeroed: the
  // caller's kernel before this level already cleared the bucket counters and the hub-row head.
  if (!prezeroed) HIPC(hipMemsetAsync(d_counts, 0, s->shard_n * 4, stream));
  if (n_in) {
    const HeavyList heavy = heavy_list(c);
    if (!prezeroed) HIPC(hipMemsetAsync(heavy.pk, 0, 8, stream));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n_in + 255) / 256, (uint64_t)s->n_cu * s->shard_wgs);
    const uint32_t budget = shard_escalates(s) && c->qcnt && !c->final ? s->shard_budget : 0u;
    hipLaunchKernelGGL(k_shard_level, dim3(grid), dim3(256), 0, stream, s->ds, d_in, (uint64_t)n_in, d_n_in, d_out,
                       (uint64_t)cap, d_counts, d_res, d_err, (uint64_t*)c->vis, c->vis_slots - 1,
                       d_done, d_done ? done_words : 0u, heavy, (uint32_t*)c->qcnt,
                       budget, n_seg, (uint64_t)seg_cap, s->shard_heavy, 1u, 0u);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_shard_heavy, dim3((uint32_t)s->n_cu * 4), dim3(256), 0, stream, s->ds, heavy, d_out,
                       (uint64_t)cap, d_counts, d_res, d_err, s->shard_n, 1u, nullptr, 0u, nullptr, nullptr);
    HIPC(hipGetLastError());
  }
  return 0;
}

// One rank: `levels` forward levels enqueued back to back in ONE call (the Python driver's per-level
// loop cost ~6 host calls and launches per level; with several batches in flight on one process the
// enqueue thread, not the device, set the step time).  Level k reads buffer cur (its record count
// from d_counts[cur][0] on the device) and writes buffer cur ^ 1; from the second level on, queries
// answered IsMember (esc_mode 1: or escalated) drop their records through the done bitmap.
int shard_levels(Snapshot* s, int levels, kg_frec* d_buf[2], size_t cap, uint32_t* d_counts[2], int start,
                 uint8_t* d_res, uint32_t* d_err, size_t slots, int esc_mode, int* end, hipStream_t stream,
                 unsigned long long* need) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  if (s->shard_n != 1) return set_error(-2, "kg_shard_levels runs one-rank batches (shard_n = %u)", s->shard_n);
  ShardCtx* c = s->shard_ctx(stream);
  if (!c || !c->vis) return set_error(-2, "kg_shard_levels before kg_shard_seed (on this stream)");
  const uint32_t words = (uint32_t)((slots + 31) / 32);
  if ((size_t)words + 1 > c->bits_n) {
    if (c->bits) HIPC(hipFree(c->bits));
    c->bits = nullptr;
    c->bits_n = 0;
    HIPC(hipMalloc((void**)&c->bits, ((size_t)words + 1) * 4));
    c->bits_n = (size_t)words + 1;
  }
  const HeavyList heavy = heavy_list(c);
  const uint32_t esc = esc_mode == 1 ? ESC_BIT : (esc_mode == 2 ? ESC2_BIT : 0u);
  const uint32_t budget = shard_escalates(s) && c->qcnt && !c->final ? s->shard_budget : 0u;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((cap + 255) / 256, (uint64_t)s->n_cu * s->shard_wgs);
  // the levels' records go to SUB per-XCD segments of one buffer, each with its own counter (emit's
  // sub mode): level 0 reads the seed's bucket, every later level the SUB segments of the one before
  const uint32_t SUB = cap >= 8 * 256 ? 8u : 1u;
  const uint64_t seg = cap / SUB;
  if (!c->cnt8) HIPC(hipMalloc((void**)&c->cnt8, 32 * 4));
  HIPC(hipMemsetAsync(c->cnt8, 0, 32 * 4, stream));
  uint32_t* sub[2] = {c->cnt8, c->cnt8 + 16};
  uint32_t* maxsub = c->cnt8 + 12;  // the largest sub-bucket count of any level (k_shard_heavy / _prep)
  // Without escalation the levels need no done bitmap -- every query is this rank's, so a level
  // reads its results directly when pruning is on (slots > 0; off when a query can still end in an
  // error an IsMember must not hide) -- and no k_shard_prep launch per level: each level's k_shard_heavy
  // zeroes the next level's bucket counters (read by the level before it) and hub-list counter (two
  // alternating words, 128 B apart).  Two launches per level instead of three.
  const bool direct = esc == 0 && budget == 0;
  unsigned long long* pk2[2] = {heavy.pk, heavy.pk + 16};  // inside the 256-B gap before the tile map
  if (direct) HIPC(hipMemsetAsync(heavy.pk, 0, 256, stream));
  int cur = start & 1;
  for (int k = 0; k < levels; k++) {
    const int nx = cur ^ 1;
    const uint32_t w = k > 0 ? words : 0u;
    HeavyList hk = heavy;
    if (direct) {
      hk.pk = pk2[k & 1];
    } else {
      hipLaunchKernelGGL(k_shard_prep, dim3(std::max<uint32_t>(1, (w + 255) / 256)), dim3(256), 0, stream,
                         (uint32_t)slots, d_res, d_err, esc, w, c->bits, sub[nx], SUB, heavy.pk, maxsub);
      HIPC(hipGetLastError());
    }
    const bool seg_in = k > 0;
    hipLaunchKernelGGL(k_shard_level, dim3(grid), dim3(256), 0, stream, s->ds, d_buf[cur], (uint64_t)cap,
                       seg_in ? sub[cur] : d_counts[cur], d_buf[nx], seg, sub[nx], d_res, d_err, (uint64_t*)c->vis,
                       c->vis_slots - 1, k > 0 && !direct ? (const uint32_t*)c->bits : nullptr, direct ? 0u : w, hk,
                       (uint32_t*)c->qcnt, budget, seg_in ? SUB : 1u, seg_in ? seg : (uint64_t)0, s->shard_heavy, SUB,
                       direct && k > 0 && slots ? 1u : 0u);
    HIPC(hipGetLastError());
    // direct: the level after this one writes sub[cur] (this level's input counters) and pk2[(k+1) & 1]
    hipLaunchKernelGGL(k_shard_heavy, dim3((uint32_t)s->n_cu * 4), dim3(256), 0, stream, s->ds, hk, d_buf[nx], seg,
                       sub[nx], d_res, d_err, s->shard_n, SUB, direct && seg_in ? sub[cur] : nullptr,
                       direct && seg_in ? SUB : 0u, direct ? pk2[(k + 1) & 1] : nullptr, maxsub);
    HIPC(hipGetLastError());
    cur = nx;
  }
  if (levels > 0) {  // the caller's counters: records left in the last buffer, flags of both
    hipLaunchKernelGGL(k_shard_fold, dim3(1), dim3(64), 0, stream, sub[cur], sub[cur ^ 1], SUB, d_counts[cur],
                       d_counts[0], (const uint32_t*)maxsub, (const uint32_t*)d_counts[start & 1], need);
    HIPC(hipGetLastError());
  }
  if (end) *end = cur;
  return 0;
}

int shard_done(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, int with_esc, uint32_t* d_bits,
               uint32_t words, hipStream_t stream) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  if (words < (n + 31) / 32) return set_error(-2, "done bitmap too small (%u words for %zu queries)", words, n);
  if (with_esc && !d_err) return set_error(-2, "kg_shard_done: with_escalated needs d_err");
  if (with_esc < 0 || with_esc > 2) return set_error(-2, "kg_shard_done: with_escalated must be 0, 1 or 2");
  if (words) {
    hipLaunchKernelGGL(k_shard_done, dim3((words + 255) / 256), dim3(256), 0, stream, (uint32_t)n, d_res, d_err,
                       with_esc == 1 ? ESC_BIT : (with_esc == 2 ? ESC2_BIT : 0u), words, d_bits);
    HIPC(hipGetLastError());
  }
  return 0;
}

int shard_back_list(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_list, size_t cap,
                    uint32_t* d_counts, hipStream_t stream) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  HIPC(hipMemsetAsync(d_counts, 0, 8, stream));
  if (!c->vis) return set_error(-2, "kg_shard_back_list before kg_shard_seed");
  HIPC(hipMemsetAsync(c->vis, 0xFF, c->vis_slots * 8, stream));  // backward keys start clear
  if (c->qcnt) HIPC(hipMemsetAsync(c->qcnt, 0, (4ull << QCNT_LOG2), stream));  // reverse-edge counts
  if (n && shard_escalates(s) && c->qinfo && n <= c->qinfo_n) {
    hipLaunchKernelGGL(k_shard_back_list, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, (uint32_t)n, d_res,
                       d_err, (const uint4*)c->qinfo, s->shard_rank, d_list, (uint64_t)cap, d_counts);
    HIPC(hipGetLastError());
  }
  return 0;
}

int shard_refwd_seed(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_out, size_t cap,
                     uint32_t* d_counts, hipStream_t stream) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  HIPC(hipMemsetAsync(d_counts, 0, (s->shard_n + 1) * 4, stream));
  if (!c->vis) return set_error(-2, "kg_shard_refwd_seed before kg_shard_seed");
  HIPC(hipMemsetAsync(c->vis, 0xFF, c->vis_slots * 8, stream));  // forward keys start clear again
  c->final = true;  // kg_shard_level runs without escalation until the next kg_shard_seed
  if (n && shard_escalates(s) && c->qinfo && n <= c->qinfo_n) {
    hipLaunchKernelGGL(k_shard_refwd_seed, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, s->ds, (uint32_t)n,
                       d_res, d_err, (const uint4*)c->qinfo, d_out, (uint64_t)cap, d_counts);
    HIPC(hipGetLastError());
  }
  return 0;
}

int shard_back_seed(Snapshot* s, const kg_frec* d_list, size_t m, const uint32_t* d_m, kg_frec* d_out, size_t cap,
                    uint32_t* d_counts, hipStream_t stream, uint32_t n_seg, size_t seg_cap) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  HIPC(hipMemsetAsync(d_counts, 0, 8, stream));
  if (m && s->ds.radj) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((m + 255) / 256, (uint64_t)s->n_cu * s->shard_wgs);
    hipLaunchKernelGGL(k_shard_back_seed, dim3(grid), dim3(256), 0, stream, s->ds, d_list, (uint64_t)m, d_m, d_out,
                       (uint64_t)cap, d_counts, n_seg, (uint64_t)seg_cap, s->shard_back_budget);
    HIPC(hipGetLastError());
  }
  return 0;
}

int shard_back_level(Snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out, size_t cap,
                     uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done, uint32_t done_words,
                     hipStream_t stream, uint32_t n_seg, size_t seg_cap) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  // the bucket size restarts; the flags word (d_counts[1]) accumulates over the phase
  HIPC(hipMemsetAsync(d_counts, 0, 4, stream));
  if (n_in && s->ds.radj) {
    const HeavyList heavy = heavy_list(c);
    HIPC(hipMemsetAsync(heavy.pk, 0, 8, stream));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n_in + 255) / 256, (uint64_t)s->n_cu * s->shard_wgs);
    hipLaunchKernelGGL(k_shard_back_level, dim3(grid), dim3(256), 0, stream, s->ds, d_in, (uint64_t)n_in, d_n_in, d_out,
                       (uint64_t)cap, d_counts, d_res, d_err, (uint64_t*)c->vis, c->vis_slots - 1, d_done,
                       d_done ? done_words : 0u, heavy, (uint32_t*)c->qcnt,
                       c->qcnt ? s->shard_back_budget : 0u, n_seg, (uint64_t)seg_cap);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_shard_heavy, dim3((uint32_t)s->n_cu * 4), dim3(256), 0, stream, s->ds, heavy, d_out,
                       (uint64_t)cap, d_counts, d_res, d_err, 1u, 1u, nullptr, 0u, nullptr, nullptr);
    HIPC(hipGetLastError());
  }
  return 0;
}

// The holder bitmap across ranks: export this rank's (import 0), or install the OR of all ranks'
// (import 1) so kg_shard_seed's no-holder test sees every rank's rows.
int shard_held(Snapshot* s, uint32_t* d_bits, size_t words, int import, hipStream_t stream) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  if (!import) {
    const size_t have = ((size_t)s->ds.hbits_n + 31) / 32;
    if (words < have) return set_error(-2, "holder bitmap needs %zu words", have);
    HIPC(hipMemsetAsync(d_bits, 0, words * 4, stream));
    if (have) HIPC(hipMemcpyAsync(d_bits, s->ds.hbits, have * 4, hipMemcpyDeviceToDevice, stream));
    return 0;
  }
  if (s->shard_held) s->free_alloc(s->shard_held);
  s->shard_held = nullptr;
  if (s->alloc((void**)&s->shard_held, words * 4 + 4)) return -1;
  if (words) HIPC(hipMemcpyAsync(s->shard_held, d_bits, words * 4, hipMemcpyDeviceToDevice, stream));
  s->shard_held_n = (uint32_t)std::min<size_t>(words * 32, 0xFFFFFFFFull);
  HIPC(hipStreamSynchronize(stream));
  return 0;
}

int shard_finish(Snapshot* s, size_t n, uint8_t* d_res, uint32_t* d_err, hipStream_t stream) {
  HIPC(hipSetDevice(s->device));
  if (!stream) stream = s->stream;
  ShardCtx* c = s->shard_ctx(stream);  // this stream's batch state (batches in flight on other streams)
  if (!c) return set_error(-4, "sharded batch state");
  if (n) {
    ShardFormula F;
    if (shard_formula(s, c, n, &F)) return -1;
    hipLaunchKernelGGL(k_shard_finish, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, (uint32_t)n, d_res,
                       d_err, F);
    HIPC(hipGetLastError());
  }
  return 0;
}

}  // namespace kg
