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
//   k_stream4   the stream tier: 32 queries per wave over one LDS FIFO of row entries, BFS over
//               the set-adjacency CSR.  A node reached at rest depth d is probed for the exact
//               tuple (checkDirect at d-1 >= 0) and, when d >= 2, expanded (checkExpandSubject's
//               children at d-1).  On rewrite-free nodes the reference's group semantics reduce
//               to "a path of <= D-1 subject-set hops to a node holding the tuple" -- SURVEY.md
//               8a; BFS marks every node at its shallowest depth, which is the schedule-free
//               answer.  Early exit on the first hit (group: first IsMember wins,
//               concurrent_checkgroup.go:104-115).
//   k_back      queries the stream tier handed on, backwards from the subject's holders.
//   grid tier   the rest, level-synchronous over the whole GPU (kg_grid.hip, kg_msbfs.hip).
//   general     rewrite interpreter (kg_interp.hip).
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
  uint32_t heavy_head, giant_head, gen_head, pad0;  // heavy: the stream tier's hand-ons (k_back's input)
  uint32_t back_head, fwd_count, back2_head, back2_count;  // (back_head, back2_head, fwd_count unused since round 6)
  uint32_t bheads[1][8 * 32];  // k_back<64>: dequeue heads of the list's 8 ranges, one 128-B line each
  uint32_t heads[8 * 32];   // per-XCD dequeue heads of the stream tier, one 128-B line each
  uint32_t light8[8 * 32];  // per-XCD shard sizes of the stream tier's work list (k_resolve appends)
  unsigned long long st[ST_N];
  unsigned long long st8[8][32];  // per-XCD shards of the hot counters (block-reduced adds)
  // k_stream4 wave span on the device clock, per XCD shard (one 128-B line each): max of ~start
  // (= the earliest start), latest end, longest wave -- workgroup-reduced atomicMax on a zeroed block
  unsigned long long tmax8[8][16];
  InterpCtl ic;
  alignas(256) uint64_t grid_sum[GRID_SUM_WORDS];  // the grid tier's first-round counters + list length (kg_grid.h)
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
// Every thread must call it (256 threads).
__device__ void block_append_lq(bool pred, const LQuery& v, LQuery* list, uint32_t* count) {
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
  uint2* dst = reinterpret_cast<uint2*>(list + bbase);
  for (uint32_t k = threadIdx.x; k < 3 * t; k += 256) dst[k] = src[k];
  __syncthreads();
}

// ------------------------------------------------------------------ k_resolve
// kg_query is 28 B (one record per thread)
__device__ __forceinline__ kg_query ld_once_q(const kg_query* p) { return *p; }

// Light-routed queries go to the stream tier as LQuery records in 8 shards of lq_cap entries (shard
// blockIdx & 7) and skip rq[i]; only queries that later tiers read by index (GENERAL) are written to
// rq (the stream tier writes the RQuery of a query it hands on).
// kg_query_packed (include/ketogpu.h) -> kg_query, in registers
__device__ __forceinline__ kg_query unpack_query(const uint4 v) {
  const uint32_t sns = (v.z >> 24) | ((v.w & 0xFu) << 8);
  kg_query x;
  x.t.ns = v.z & 0xFFFu;
  x.t.obj = v.x;
  x.t.rel = (v.z >> 12) & 0xFFFu;
  x.t.sns = sns == KG_PACK_SUBJECT_ID ? KG_SUBJECT_ID : sns;
  x.t.sobj = v.y;
  x.t.srel = (v.w >> 4) & 0xFFFu;
  x.max_depth = (int32_t)(v.w >> 16);
  return x;
}

// pq != nullptr: the batch's queries are packed (16 B each, kg_check_batch_packed_device) and q is unused
__global__ __launch_bounds__(256) void k_resolve(DevSnap s, const kg_query* __restrict__ q, const uint4* __restrict__ pq,
                                                 uint32_t n,
                                                 uint32_t n_base, const uint32_t* __restrict__ n_extra,
                                                 int32_t global, RQuery* __restrict__ rq, uint8_t* __restrict__ out,
                                                 uint32_t* __restrict__ err, uint32_t* gen_list,
                                                 int no_holder_filter, Ctl* ctl, LQuery* lq_list, uint32_t lq_cap) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // n: capacity (list strides); with a formula split the live count is n_base + *n_extra
  bool valid = i < (n_extra ? n_base + *n_extra : n);
  uint32_t route = ROUTE_DONE;
  bool did_probe = false, no_holder = false;
  LQuery lq{};
  if (valid) {
    kg_query x = pq ? unpack_query(pq[i]) : ld_once_q(q + i);
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
    if (use_bits) hw = subj < s.hbits_n ? ld_once(s.hbits + (subj >> 5)) : 0u;
    else if (want_h && !use_bits) h0 = s.hslots[hi];
    // without a namespace program nothing can end as an error, so a subject that no row holds is
    // NotMember whatever the root: the bit (an Infinity-Cache hit) is read first and such a query
    // never touches the node map (~13 % of the C2 batch; one random HBM line each)
    const bool unheld = no_holder_filter == 2 && use_bits && !s.relflags && !((hw >> (subj & 31)) & 1u);
    NSlot n0{};
    if (key_ok && !unheld) n0 = ld_once(s.nmap + ni);
    uint32_t node = NONE, rb = 0, rl = 0, rsig_lo = 0xFFFFFFFFu, rsig = 0xFFFFFFFFu, nfl = 0, icnt = 0;
    uint64_t rpad = 0;
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
        rsig_lo = (uint32_t)v.pad1;  // signature bits 0-11 in bits 20-31
        nfl = (uint32_t)(v.pad1 & 0xFFu);
        icnt = nslot_inline(v.pad1);
        rpad = v.pad1;
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
      if (icnt) {
        // the whole check row is in the slot: exact, no dset line
        member = subj != NONE && nslot_inline_has(icnt, rpad, rsig, subj);
      } else {
        did_probe = subj != NONE && !nobit && sig_maybe(rsig_lo, rsig, subj_sig(subj));
        member = did_probe && dset_probe(s, node, subj);
      }
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
    if (route == ROUTE_GENERAL) rq[i] = RQuery{node, subj, d, route, rb, rl};
    lq = LQuery{i, node, subj, d, rb, rl};
    // every result starts as NotMember / no error (coalesced here): the tiers after this one store
    // only what differs (k_stream4 writes IsMember bytes only)
    out[i] = member ? KG_IS_MEMBER : KG_NOT_MEMBER;
    if (err) err[i] = KG_ERR_NONE;
  }
  {
    const int idx[2] = {ST_PROBES, ST_NOHOLD};
    const unsigned long long v[2] = {(valid && did_probe) ? 1ull : 0ull, no_holder ? 1ull : 0ull};
    block_stats<2>(ctl, idx, v);
  }
  // stream-tier work list: 8 shards of lq_cap records (shard = blockIdx & 7), dequeued per XCD
  const uint32_t h = blockIdx.x & 7;
  block_append_lq(valid && route == ROUTE_LIGHT, lq, lq_list + (size_t)h * lq_cap, &ctl->light8[h * 32]);
  block_append(valid && route == ROUTE_GENERAL, i, gen_list, &ctl->gen_count);
}

// ------------------------------------------------------------------ stream-tier FIFO entries
// FIFO entries are 8 bytes: row begin | meta = len 11 | slot 5 | generation 9 | rest depth 7; per-slot
// state is one word (generation | HIT | OVER).
constexpr uint32_t S2_LONG = 2047;  // longest row a FIFO entry can hold (11-bit length)
constexpr uint32_t S2_GEN = 0x1FF, S2_DMAX = 127;
constexpr uint32_t S2_HIT = 1u << 30, S2_OVER = 1u << 31;

__device__ __forceinline__ uint32_t s2_meta(uint32_t len, uint32_t slot, uint32_t gen, uint32_t depth) {
  return len | (slot << 11) | ((gen & S2_GEN) << 16) | (depth << 25);
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan<DppOr>(v), 63);
}

// ------------------------------------------------------------------ k_stream4 (variant 15)
// The stream tier: one wave runs up to 32 queries at once over ONE FIFO of row entries (adjx begin,
// length, slot | generation | rest depth).  Every step takes the next 64 edges from the FIFO head --
// whatever queries they belong to -- gathers their adjx records and, in the same round trip, probes
// dset (checkDirect) for the children the previous step found; so lanes stay busy however small the
// queries are, and a finished query's slot is refilled at once.
//   * per query, FIFO order is BFS order (children are appended after every entry of the current
//     level), so first-mark dedup marks each node at its shallowest depth: the canonical answer
//   * the visited set is a DIRECT-MAPPED cache of keys valid | gen | slot | node with blind writes --
//     no probing, no CAS.  A collision can only make a node be expanded again (extra work, same
//     answer: expanding a node again at a smaller rest depth explores a subset of its first
//     expansion); it never reports a node present that this query did not insert
//   * a query ends on a hit (IsMember), when it has no FIFO entry and no pending probe left
//     (NotMember, pre-written by k_resolve), or on overflow (FIFO full, a row longer than S2_LONG,
//     the edge budget "stream_ecap"), which hands it to the backward / grid tiers to be redone there
//   * a finished slot bumps its generation: its FIFO entries and pending probes become stale
//   * the step is straight-line predicated code; every load is issued unconditionally (below)
//   * work comes as LQuery records (k_resolve writes the resolved query into the list itself), and a
//     dequeue is PIPELINED over steps: step t issues the head atomic, step t+1 issues the coalesced
//     record load, the records are used from step t+2 on -- both round trips hide under the steps'
//     gathers, so chunks can be small
//   * per-slot bookkeeping without returning LDS atomics: a query is finished when the FIFO position
//     of its last appended entry (s_last, an atomicMax) lies behind the head -- no decrement per
//     consumed entry and no increment per append; the edge budget is an atomicAdd read once, at the
//     step's finish check (a query past it is retired in the same step)
//   * the range bounds of the 8 per-XCD list shards are read once, into lanes 0..7
//   * queries handed on write their RQuery for the next tiers (k_resolve no longer does)
constexpr uint32_t S4_CHUNK = 64;
// Edges per lane and step (round 6): the step is bound by its chain of dependent LDS and HBM round
// trips, not by issue (~150 VALU per step at 4 waves per SIMD, ~2.5 us per step), and LDS caps the
// waves per CU; two edges per lane double the gathers and probes one round trip carries.
// (-DKG_STREAM_EPL=1 builds the one-edge step for A/Bs.)
#ifndef KG_STREAM_EPL
#define KG_STREAM_EPL 2
#endif
// Visited-cache keys per wave (log2) and FIFO entries per wave.  256 keys (round 6; 512 before): 25.5 KB of
// LDS per workgroup instead of 33.7 KB, so 5 workgroups per CU fit (the VGPR limit, 95 VGPRs) instead of 4 --
// the same work per batch (rows, edges, probes and tiers unchanged) in a 13 % shorter launch; a 128-entry
// FIFO instead measured slower (more queries handed on), profiles/r6z4_stream_lds_ab.jsonl.  -D overrides
// build A/B variants.
#ifndef KG_STREAM_VLOG2
#define KG_STREAM_VLOG2 8
#endif
#ifndef KG_STREAM_QC
#define KG_STREAM_QC 256
#endif

template <int VLOG2, int QC, int EPL>
struct Stream4Lds {
  unsigned long long vt[1 << VLOG2];  // direct-mapped visited cache (0 = empty)
  uint32_t e_beg[QC], e_meta[QC];     // FIFO ring
  uint32_t pref[64 * EPL + 1];        // edge-owner marks (+1 dummy)
  uint32_t s_state[32], s_qi[32], s_subj[32], s_last[32], s_edg[32];
  uint32_t s_node[32], s_depth[32], s_beg[32], s_len[32];
  uint4 s_ss[32];  // per slot: the subject's Bloom mask (2 words), the visited-cache salt of (slot, generation)
};

struct LqList {
  const LQuery* list;
  const uint32_t* counts;  // shard h: counts[32 h] records from list[h * cap] (k_resolve's appends)
  uint32_t cap;
};

template <int VLOG2, int QC, int EPL>
__global__ __launch_bounds__(256) void k_stream4(DevSnap s, LqList wl, uint32_t* heads, uint8_t* __restrict__ out,
                                                 RQuery* __restrict__ rq, uint32_t* next_list, uint32_t* next_count,
                                                 Ctl* ctl, uint32_t ecap, uint32_t chunk, uint32_t ranges) {
  using Lds = Stream4Lds<VLOG2, QC, EPL>;
  static_assert(EPL == 1 || EPL == 2, "one or two edges per lane and step");
  constexpr uint32_t WIN = 64u * EPL;
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
  const uint32_t shard_n = lane < 8 ? wl.counts[lane * 32] : 0u;
  __builtin_amdgcn_wave_barrier();
  uint32_t active = 0;  // wave-uniform: slots holding a query
  // dequeue pipeline (wave-uniform state): 0 idle, 1 head atomic in flight (tk, lane 0), 2 records staged
  uint32_t pf = 0, tk = 0, st_got = 0;
  bool exhausted = false;  // every range this wave drains is empty
  LQuery sq{};             // staged chunk (lane k: record k)
  uint32_t c_left = 0, c_pos = 0;
  LQuery cq{};             // current chunk
  uint32_t head = 0, tail = 0, head_off = 0;
  // the previous step's children awaiting their checkDirect probe: one per edge a lane gathered
  bool pend[EPL];
  uint32_t pend_node[EPL], pend_slot[EPL], pend_gen[EPL];
#pragma unroll
  for (int h = 0; h < EPL; h++) {
    pend[h] = false;
    pend_node[h] = pend_slot[h] = pend_gen[h] = 0;
  }
  // per-lane counters: each grows by at most one per step, and a wave's steps stay far below 2^32
  uint32_t st_rows = 0, st_edges = 0, st_probes = 0, st_done = 0, st_steps = 0;
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
        // visited-cache salt of (slot, generation): one LDS read per step instead of two multiplies
        const uint32_t salt = (slot * 0x85EBCA77u) ^ (gen * 0xC2B2AE3Du);
        L.s_qi[slot] = qi;
        L.s_subj[slot] = qsubj;
        const uint2 qm = subj_sig(qsubj);
        L.s_ss[slot] = make_uint4(qm.x, qm.y, salt, 0u);
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
        L.vt[((qnode * 0x9E3779B1u) ^ salt) >> (32 - VLOG2)] = key;
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
        st_got = min(chunk, hi - (lo + k));
        if ((uint32_t)lane < st_got) sq = wl.list[lo + k + (uint32_t)lane];
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
    if (active == 0) {
      if (exhausted && pf == 0 && c_left == 0) break;
      head = tail;  // no query holds the FIFO: whatever is left in it is stale
      head_off = 0;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- window: up to 64 FIFO entries from the head, up to WIN = 64 * EPL edges of them (edge e on
    // lane e % 64, in the lane's pass e / 64)
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
    bool pvalid[EPL];
    uint64_t pkey[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      const uint32_t pst = L.s_state[pend_slot[h]], psubj = L.s_subj[pend_slot[h]];
      pvalid[h] = pend[h] && pst == pend_gen[h];
      pkey[h] = dset_key(pend_node[h], psubj);
    }
    const bool inwin = (uint32_t)lane < avail;
    const bool live = inwin && ((active >> sl0) & 1u) && (st0 == ((emeta >> 16) & S2_GEN));  // no HIT/OVER
    uint32_t elen = live ? (emeta & 0x7FFu) : 0u;
    if (lane == 0) {
      ebeg += head_off;
      elen = live ? elen - head_off : 0u;
    }
    if (!inwin) emeta = 0;
    uint32_t total;
    const uint32_t excl = wave_excl_scan(elen, &total);
#pragma unroll
    for (int h = 0; h < EPL; h++) L.pref[lane + 64 * h] = 0;
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
    AdjX x[EPL];
    uint32_t om[EPL];
    bool act[EPL];
    uint32_t mcarry = 0;  // owner marks of the earlier passes' edges (a max-scan carried across passes)
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      uint32_t m = wave_incl_scan<DppMax>(L.pref[lane + 64 * h]);
      if (h > 0) m = max(m, mcarry);
      if (h + 1 < EPL) mcarry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
      const int own = ((int)m - 1) & 63;
      const uint32_t ob = __shfl(ebeg, own, 64);
      om[h] = __shfl(emeta, own, 64);
      const uint32_t ox = __shfl(excl, own, 64);
      const uint32_t e = (uint32_t)lane + 64u * h;
      act[h] = e < taken;
      x[h] = s.adjx[act[h] ? ob + (e - ox) : 0u];  // adjx[0] exists (n_set_edges + 1)
    }
    ulonglong2 pb[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++)
      pb[h] = ld_once(
          reinterpret_cast<const ulonglong2*>(s.dset + (pvalid[h] ? dset_home(pkey[h], s.dset_nb) : 0ull) * DSET_BUCKET));
    uint32_t slot[EPL], d[EPL], g[EPL];
    uint4 ss[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      slot[h] = (om[h] >> 11) & 31u;
      d[h] = om[h] >> 25;
      g[h] = (om[h] >> 16) & S2_GEN;
      ss[h] = L.s_ss[slot[h]];  // LDS, under the gathers' latency: Bloom mask, visited-cache salt
    }
    head += ncons;
    st_edges += (lane == 0) ? taken : 0u;
    st_steps += (lane == 0) ? 1u : 0u;
    // checkDirect probe, first bucket; a chain past a full first bucket (rare at load <= 0.25) is
    // walked by the lanes that need it under a wave-uniform branch
    // bitwise, not short-circuit: a branch on pvalid split the bucket's 16-B load in two, one half
    // issued and waited for inside the branch
    bool hit[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      hit[h] = pvalid[h] & ((pb[h].x == pkey[h]) | (pb[h].y == pkey[h]));
      const bool more = pvalid[h] & !hit[h] & (pb[h].y != EMPTY64);
      if (__ballot(more)) {
        if (more) hit[h] = dset_probe(s, pend_node[h], (uint32_t)pkey[h]);
      }
      st_probes += pvalid[h] ? 1u : 0u;
    }
    // ---- children: kept ones (rest >= 2 after the hop, non-empty set row) are marked + appended;
    // every child new to the query is probed next step.  Pass 0's edges precede pass 1's in FIFO
    // order, so marks and appends go pass by pass: a node met twice in one step is kept at its first
    // (shallowest) occurrence and the FIFO stays in BFS order per query.
    bool keepc[EPL], fresh[EPL];
    uint32_t xlen[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      xlen[h] = adjx_len16(x[h]);  // saturated at ADJX_LEN_SAT: any such row is long here
      keepc[h] = act[h] && d[h] >= 3 && xlen[h] > 0;  // x of an inactive lane is adjx[0]: never used
      const bool longrow = keepc[h] && xlen[h] > S2_LONG;
      const unsigned long long key =
          (1ull << 63) | ((unsigned long long)g[h] << 37) | ((unsigned long long)slot[h] << 32) | x[h].node;
      const uint32_t hv = ((x[h].node * 0x9E3779B1u) ^ ss[h].z) >> (32 - VLOG2);
      const unsigned long long old = keepc[h] ? L.vt[hv] : 0ull;
      fresh[h] = keepc[h] && !longrow && old != key;
      if (fresh[h]) L.vt[hv] = key;
      if (longrow) atomicOr(&L.s_state[slot[h]], S2_OVER);  // row too long for a FIFO entry
    }
    const uint32_t room = QC - (tail - head);
    uint32_t nfresh = 0;
    bool appended[EPL];
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      const uint64_t am = __ballot(fresh[h]);
      const uint32_t pos = nfresh + (uint32_t)__popcll(am & ((1ull << lane) - 1));
      nfresh += (uint32_t)__popcll(am);
      appended[h] = fresh[h] && pos < room;
      if (appended[h]) {
        const uint32_t at = tail + pos;
        L.e_beg[at & (QC - 1)] = x[h].begin;
        L.e_meta[at & (QC - 1)] = xlen[h] | (om[h] & 0x01FFF800u) | ((d[h] - 1) << 25);
        atomicMax(&L.s_last[slot[h]], at);   // no return: read at the finish check
        atomicAdd(&L.s_edg[slot[h]], xlen[h]);  // edge budget, likewise
      }
      if (fresh[h] && !appended[h]) atomicOr(&L.s_state[slot[h]], S2_OVER);  // FIFO full
    }
    tail += min(nfresh, room);
    uint32_t pmask = 0;
#pragma unroll
    for (int h = 0; h < EPL; h++) {
      if (hit[h]) atomicOr(&L.s_state[pend_slot[h]], S2_HIT);
      pend[h] = act[h] && (keepc[h] ? appended[h] : true) && sig_maybe(x[h].lsig, x[h].sig, make_uint2(ss[h].x, ss[h].y));
      pend_node[h] = x[h].node;
      pend_slot[h] = slot[h];
      pend_gen[h] = g[h];
      pmask |= pend[h] ? 1u << slot[h] : 0u;
    }
    const uint32_t pslots = wave_or(pmask);
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
      } else if ((st & S2_OVER) || (ecap != 0xFFFFFFFFu && edg > ecap)) {
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
#pragma unroll
    for (int h = 0; h < EPL; h++)
      if (pend[h] && ((freed >> pend_slot[h]) & 1u)) pend[h] = false;
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t_end = wall_clock64(), life = lane == 0 ? t_end - t_start : 0ull;
  block_max3(ctl, ~(unsigned long long)t_start, t_end, t_end - t_start);
  const int idx[7] = {ST_LROWS, ST_LEDGES, ST_LPROBES, ST_LIGHT, ST_LSTEPS, ST_LWAVES, ST_LTICKS};
  const unsigned long long v[7] = {st_rows, st_edges, st_probes, st_done, st_steps, lane == 0 ? 1ull : 0ull, life};
  block_stats<7>(ctl, idx, v);
}

// ------------------------------------------------------------------ workgroup helpers
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
// k_back<64> runs one query per WAVE (visited hash 512 / list 256 in LDS, 12 queries in flight per
// CU); its overflow goes to the grid tier.  (Rounds 2-5 also built a workgroup-per-query width,
// k_back<256>, behind it -- an A/B knob that never beat this chain; the template keeps W generic.)
template <int W>
struct BackCfg;
// EDGES: reverse edges one query may read here.  A level that reaches hub groups reads their whole
// parent lists (up to 1e5 each) on one wave -- 28 ms for one query at 1 B tuples before this bound
// (profiles/r2o_*): such a query goes to the grid tier, which spreads its edges over the whole GPU.
// The launch lasts as long as its longest query and the grid tier runs for the hand-ons anyway, so
// the bound is low: 2^14 -> 2^12 took C2 from 6.8 to 7.0-7.2 x 10^9 checks/s
// (profiles/r4t_back_edges_ecap_sweep.jsonl, r4u_back_edges_sweep.jsonl; 2^10-2^11 and 2^15 slower).
template <>
struct BackCfg<64> {
  static constexpr uint32_t VLOG2 = 9, CAP = 256;  // larger caps only lengthen the tail (1024: -9 % checks/s)
  static constexpr uint32_t EDGES = 1u << 12;
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
                                              Ctl* ctl, uint32_t edges) {
  constexpr uint32_t VSLOTS = BackLds<W>::VSLOTS, CAP = BackLds<W>::CAP;
  constexpr int BU = 4;
  __shared__ BackLds<W> lds_all[256 / W];
  BackLds<W>& L = lds_all[threadIdx.x / W];
  const int t = threadIdx.x % W;  // thread within the query group
  const uint32_t qcount = *qcount_p;
  unsigned long long st_rows = 0, st_edges = 0, st_done = 0;
  // the first query of every group is static (group g takes g); the rest of the list is cut into 8
  // ranges, each dequeued through its own head on a line of its own (qhead[r * 32]): a group starts at
  // its XCD's range and moves on when that one is dry.  One hot word saturates near 90 M dequeues/s
  // (MI355X_MICROARCH.md "dequeue"): ~9 k dequeues per C3 batch on one word were ~100 us of k_back.
  const uint32_t n_groups = gridDim.x * (256 / W), g0 = blockIdx.x * (256 / W) + threadIdx.x / W;
  const uint32_t rest = qcount > n_groups ? qcount - n_groups : 0u, rlen = (rest + 7) / 8;
  uint32_t r_at = blockIdx.x & 7, r_tried = 0;
  for (bool first = true;; first = false) {
    if (first) {
      if (t == 0) L.qi = g0;
    } else {
      if (!rest) break;  // the static round took every query
      if (t == 0) {
        uint32_t qi = NONE;
        for (; r_tried < 8; r_tried++, r_at = (r_at + 1) & 7) {
          const uint32_t k = atomicAdd(&qhead[r_at * 32], 1u);
          if (k < rlen && r_at * rlen + k < rest) {
            qi = n_groups + r_at * rlen + k;
            break;
          }
        }
        L.qi = qi;
      }
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
    uint32_t budget = edges ? edges : BackCfg<W>::EDGES;  // wave-uniform
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

// The rewrite interpreter's control block pointers (its counters live in the batch's zeroed Ctl).
__global__ void k_ic_init(InterpCtl* ic, const uint32_t* gen_count, uint32_t* p2_list, Ctl* ctl) {
  ic->gen_count = gen_count;
  ic->p2_list = p2_list;
  ic->st_general = &ctl->st[ST_GENERAL];
  ic->st_rows = &ctl->st[ST_ROWS];
  ic->st_edges = &ctl->st[ST_EDGES];
  ic->st_probes = &ctl->st[ST_PROBES];
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
                      uint8_t* d_out, uint32_t* d_err, kg_stats* stats, BatchPending* bp,
                      const kg_query_packed* d_pk) {
  *bp = BatchPending{};
  bp->stats = stats;
  bp->d_out = d_out;
  bp->d_err = d_err;
  if (global_max_depth < 1) global_max_depth = 5;  // config.schema.json:308-315 default
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  HIPC(hipSetDevice(s->device));
  hipStream_t stream = w->stream;
  // timing of a batch with stats: the whole batch (ev 0-1), k_stream4 (2-3), the formula split (4-5)
  // and each tail-tier level launch (Workspace::lev_mark)
  if (stats && !w->ev[0])
    for (auto& e : w->ev) HIPC(hipEventCreate(&e));
  // per-launch level events only when asked for (kg_snapshot_tune "level_events"): an event record
  // between back-to-back launches leaves a gap in the stream (round 6: -15 % on the headline with
  // stats on every batch)
  w->lev_on = stats != nullptr && s->level_events != 0;
  w->lev_n = 0;
  w->lev_kind = 0;
  w->lev_launches = 0;
  if (stats) HIPC(hipEventRecord(w->ev[0], stream));
  // packed queries: k_resolve unpacks them in registers when it is the only reader of the queries --
  // without a namespace program there is no formula split and no general route; otherwise they are
  // unpacked into the workspace first
  const uint4* pq = nullptr;
  if (d_pk && n) {
    if (s->n_fplans || s->ds.relflags || s->ds.nflags) {
      if (n > w->unpacked_n) {
        if (w->unpacked) hipFree(w->unpacked);
        w->unpacked = nullptr;
        w->unpacked_n = 0;
        HIPC(hipMalloc(&w->unpacked, n * sizeof(kg_query)));
        w->unpacked_n = n;
      }
      if (int rc = unpack_queries(d_pk, n, w->unpacked, stream)) return rc;
      d_q = w->unpacked;
    } else {
      pq = reinterpret_cast<const uint4*>(d_pk);
      d_q = nullptr;
    }
  }
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
    if (stats) HIPC(hipEventRecord(w->ev[4], stream));
    if (int rc = formula_split(s, w, d_q, n, global_max_depth, &q2, &n2, &n_extra, &out2, &err2, &ref)) return rc;
    if (stats) HIPC(hipEventRecord(w->ev[5], stream));
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
  // scratch: rq[n] | lq (8 shards of lq_cap LQuery records) | gen[n] | heavy[n] | giant[n] | p2[n] | back2[n] | Ctl.
  // Shard h of the stream tier's work list receives the appends of k_resolve's blocks h, h + 8, ...
  // (<= 256 records each), so a shard holds ceil(blocks / 8) * 256 records.
  auto lq_cap_of = [](size_t m) { return (((m + 255) / 256 + 7) / 8) * 256; };
  auto layout = [&](size_t m, size_t* off) {
    off[0] = 0;
    off[1] = align_up(off[0] + m * sizeof(RQuery));
    off[2] = align_up(off[1] + 8 * lq_cap_of(m) * sizeof(LQuery));
    for (int k = 3; k <= 7; k++) off[k] = align_up(off[k - 1] + m * 4);
    return align_up(off[7] + sizeof(Ctl));
  };
  size_t off[8];
  const size_t total = layout(n, off);
  if (total > w->scratch_bytes) {  // sized for >= 64 Ki queries, grown geometrically (hipFree stalls the device)
    const size_t m = std::max<size_t>(65536, std::max<size_t>(2 * w->scratch_n, n));
    size_t tmp[8];
    const size_t want = layout(m, tmp);
    if (w->scratch) hipFree(w->scratch);
    w->scratch = nullptr;
    w->scratch_bytes = 0;
    HIPC(hipMalloc(&w->scratch, want));
    w->scratch_bytes = want;
    w->scratch_n = m;
  }
  char* base = (char*)w->scratch;
  RQuery* rq = (RQuery*)(base + off[0]);
  LQuery* lq = (LQuery*)(base + off[1]);
  uint32_t* gen = (uint32_t*)(base + off[2]);
  uint32_t* heavy = (uint32_t*)(base + off[3]);
  uint32_t* p2 = (uint32_t*)(base + off[5]);
  uint32_t* back2 = (uint32_t*)(base + off[6]);
  Ctl* ctl = (Ctl*)(base + off[7]);
  const uint32_t lq_cap = (uint32_t)lq_cap_of(n);
  bool grid_pending = false;
  const uint32_t *grid_list = nullptr, *grid_count = nullptr;

  hipEvent_t e1 = w->ev[1], l0 = w->ev[2], l1 = w->ev[3];
  HIPC(hipMemsetAsync(ctl, 0, sizeof(Ctl), stream));
  if (n) {
    const bool use_back = s->ds.radj != nullptr;
    const uint32_t nblk = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_resolve, dim3(nblk), dim3(256), 0, stream, s->ds, d_q, pq, (uint32_t)n, (uint32_t)n_base, n_extra,
                       global_max_depth, rq, d_out, d_err, gen, use_back ? 2 : 0, ctl, lq,
                       lq_cap);
    HIPC(hipGetLastError());
    if (stats) HIPC(hipEventRecord(l0, stream));
    {
      // ~25 KiB of LDS per workgroup (4 waves: a 256-key visited cache and a 256-entry FIFO each);
      // stream_wgs per CU (default 2: the rest of the LDS serves the other batches in flight)
      const uint32_t per_cu = s->stream_wgs ? (uint32_t)s->stream_wgs : 2u;
      const uint32_t ecap = s->stream_ecap ? s->stream_ecap : 0xFFFFFFFFu;
      // >= 8 workgroups: with stream_steal < 8 a wave drains only `ranges` of the 8 per-XCD ranges
      // starting at its label blockIdx & 7, so every label must occur for every range to be drained
      const uint32_t grid =
          std::max<uint32_t>(8u, (uint32_t)std::min<uint64_t>((uint64_t)s->n_cu * per_cu, (n + 31) / 32 + 8));
      hipLaunchKernelGGL((k_stream4<KG_STREAM_VLOG2, KG_STREAM_QC, KG_STREAM_EPL>), dim3(grid), dim3(256), 0, stream, s->ds, LqList{lq, ctl->light8, lq_cap},
                         ctl->heads, d_out, rq, heavy, &ctl->heavy_count, ctl, ecap, S4_CHUNK, s->stream_steal);
    }
    HIPC(hipGetLastError());
    if (stats) HIPC(hipEventRecord(l1, stream));
    {
      // backward tier first (k_back), its overflow -> forward grid tier
      const uint32_t* fwd_list = heavy;
      const uint32_t* fwd_count = &ctl->heavy_count;
      if (use_back) {
        // one query per wave (~48 KiB LDS per workgroup: 3 per CU); its overflow goes to the grid tier
        // (the workgroup-per-query width k_back<256> between them measured no better and was removed
        // in round 6 with the "back" knob)
        hipLaunchKernelGGL(k_back<64>, dim3((uint32_t)s->n_cu * s->back_wgs), dim3(256), 0, stream, s->ds, rq, heavy,
                           &ctl->heavy_count, ctl->bheads[0], d_out, d_err, back2, &ctl->back2_count, ctl,
                           (uint32_t)s->back_edges);
        HIPC(hipGetLastError());
        fwd_list = back2;
        fwd_count = &ctl->back2_count;
      }
      // first grid round enqueued without waiting; its readback is checked after the batch's one sync
      const int rc = grid_tier(s, w, rq, fwd_list, fwd_count, global_max_depth, d_out, d_err, stream, &bp->gs, 1, true,
                               ctl->grid_sum);
      if (rc < 0) return rc;
      grid_pending = rc == 1;
      grid_list = fwd_list;
      grid_count = fwd_count;
    }
    if (s->has_program) {
      // the interpreter's control block: its counters and heads were zeroed with the Ctl; the pointers are
      // written by a one-thread kernel (round 6: a hipMemcpyAsync from this stack variable -- pageable
      // memory -- held the host until the stream had drained, a gap before the interpreter passes of
      // every C3 batch)
      hipLaunchKernelGGL(k_ic_init, dim3(1), dim3(1), 0, stream, &ctl->ic, (const uint32_t*)&ctl->gen_count, p2, ctl);
      if (launch_general(s, w, d_q, rq, gen, &ctl->gen_count, &ctl->ic, d_out, d_err, (uint32_t)n, stream)) return -1;
    }
    // the requested results, stream-ordered before anything the caller enqueues after this call
    if (bp->split && formula_combine(s, w, bp->f_n, bp->f_ref, d_out, d_err, bp->f_out, bp->f_err)) return -1;
  }
  // one synchronisation per batch: the grid round's readback and the counters come back together
  static_assert(sizeof(Ctl) <= 32768, "Ctl readback fits the lower half of the pinned buffer");
  void* hbuf = w->host_buf(65536);
  if (!hbuf) return set_error(-1, "pinned host buffer");
  if (stats) HIPC(hipEventRecord(e1, stream));
  // one readback: the counters and, when the grid tier ran a round, its summary (Ctl::grid_sum)
  if (stats || grid_pending) HIPC(hipMemcpyAsync(hbuf, ctl, sizeof(Ctl), hipMemcpyDeviceToHost, stream));
  bp->grid_pending = grid_pending;
  bp->grid_list = grid_list;
  bp->grid_count = grid_count;
  bp->rq = rq;
  bp->gdepth = global_max_depth;
  bp->n = n;
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
    const Ctl* hc = reinterpret_cast<const Ctl*>(bp->ctl_host);
    if (int rc = grid_tier(s, w, bp->rq, bp->grid_list, bp->grid_count, bp->gdepth, bp->d_out, bp->d_err, stream, &gs, 2,
                           true, nullptr, hc->grid_sum))
      return rc;
    if (reran) *reran = w->grid_reran;
    // the rerun rewrote leaf results after check_batch_begin's combine: combine again
    if (bp->split && w->grid_reran &&
        formula_combine(s, w, bp->f_n, bp->f_ref, bp->d_out, bp->d_err, bp->f_out, bp->f_err))
      return -1;
  }
  if (stats) {
    float ms = 0, lms = 0, sms = 0;
    HIPC(hipEventElapsedTime(&ms, w->ev[0], w->ev[1]));
    if (bp->n) HIPC(hipEventElapsedTime(&lms, w->ev[2], w->ev[3]));
    if (bp->split) HIPC(hipEventElapsedTime(&sms, w->ev[4], w->ev[5]));
    double tms = 0;
    for (int k = 0; k < w->lev_n; k++) {
      float x = 0;
      if (w->lev_ev[2 * k] && w->lev_ev[2 * k + 1] &&
          hipEventElapsedTime(&x, w->lev_ev[2 * k], w->lev_ev[2 * k + 1]) == hipSuccess)
        tms += x;
      else
        (void)hipGetLastError();
    }
    w->lev_on = false;
    stats->tail_ms = tms;
    stats->tail_launches = w->lev_launches;
    stats->tail_kind = (uint64_t)w->lev_kind;
    stats->tail_rows = gs.rows;
    stats->tail_edges = gs.edges;
    stats->tail_probes = gs.probes;
    stats->tail_logged = gs.logged;
    stats->ms_edges_loaded = gs.ms_eload;
    stats->ms_words_active = gs.ms_wact;
    stats->split_ms = sms;
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
    stats->n_medium = 0;  // (removed tiers: kept in the ABI struct, always 0)
    stats->n_heavy = gs.done;
    stats->n_wide = 0;
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
                       uint8_t* d_out, uint32_t* d_err, kg_stats* stats, const kg_query_packed* d_pk) {
  BatchPending bp;
  if (int rc = check_batch_begin(s, w, d_q, n, global_max_depth, d_out, d_err, stats, &bp, d_pk)) return rc;
  return check_batch_end(s, w, &bp, nullptr, true);
}

// ---- the narrow host boundary (kg_check_batch_packed): 16-B queries in, sparse error codes out
// One query per thread; a 16-B load and a 28-B store, both coalesced (HBM-streaming, no reuse).
__global__ __launch_bounds__(256) void k_unpack(const uint4* __restrict__ pk, uint32_t n, kg_query* __restrict__ q) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  q[i] = unpack_query(pk[i]);
}

// The checks answered KG_ERROR as (base + index, code) pairs after a count word: list[0] = count,
// pairs from list[2].  One device atomic per wave with an error (errors are rare).
__global__ __launch_bounds__(256) void k_err_list(const uint8_t* __restrict__ out, const uint32_t* __restrict__ err,
                                                  uint32_t n, uint32_t base, uint32_t* list, uint32_t cap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool e = i < n && out[i] == KG_ERROR;
  const uint64_t m = __ballot(e);
  if (!m) return;
  const int lead = __ffsll((unsigned long long)m) - 1;
  uint32_t at = 0;
  if (lane_id() == lead) at = atomicAdd(list, (uint32_t)__popcll(m));
  at = __shfl(at, lead, 64) + lanes_below(m);
  if (e && at < cap) {
    list[2 + 2 * (size_t)at] = base + i;
    list[3 + 2 * (size_t)at] = err[i];
  }
}

// kg_pack_query on the device (kg_pack_queries_device): 28-B load, 16-B store per thread; an id that
// does not fit sets *bad
__global__ __launch_bounds__(256) void k_pack(const kg_query* __restrict__ q, uint32_t n, uint4* __restrict__ pk,
                                              uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const kg_query x = q[i];
  const uint32_t sns = x.t.sns == KG_SUBJECT_ID ? KG_PACK_SUBJECT_ID : x.t.sns;
  const uint32_t srel = x.t.sns == KG_SUBJECT_ID ? 0u : x.t.srel;
  const uint32_t d = x.max_depth <= 0 ? 0u : (x.max_depth > 65535 ? 65535u : (uint32_t)x.max_depth);
  if (x.t.ns > KG_PACK_ID_MAX || x.t.rel > KG_PACK_ID_MAX || (sns != KG_PACK_SUBJECT_ID && sns > KG_PACK_ID_MAX) ||
      srel > KG_PACK_ID_MAX)
    atomicOr(bad, 1u);
  pk[i] = make_uint4(x.t.obj, x.t.sobj, x.t.ns | (x.t.rel << 12) | ((sns & 0xFFu) << 24),
                     (sns >> 8) | (srel << 4) | (d << 16));
}

int pack_queries(const kg_query* d_q, size_t n, kg_query_packed* d_pk, uint32_t* d_bad, hipStream_t stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_pack, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, d_q, (uint32_t)n, (uint4*)d_pk,
                     d_bad);
  HIPC(hipGetLastError());
  return 0;
}

int unpack_queries(const kg_query_packed* d_pk, size_t n, kg_query* d_q, hipStream_t stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_unpack, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, (const uint4*)d_pk,
                     (uint32_t)n, d_q);
  HIPC(hipGetLastError());
  return 0;
}

int error_list(const uint8_t* d_out, const uint32_t* d_err, size_t n, uint32_t base, uint32_t* d_list, size_t cap,
               hipStream_t stream) {
  HIPC(hipMemsetAsync(d_list, 0, 8, stream));
  if (!n) return 0;
  hipLaunchKernelGGL(k_err_list, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, d_out, d_err, (uint32_t)n,
                     base, d_list, (uint32_t)cap);
  HIPC(hipGetLastError());
  return 0;
}

}  // namespace kg
