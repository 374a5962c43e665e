// kg_expand.hip -- batched expand trees (expand.Engine.BuildTree, internal/expand/engine.go:35-104).
//
// BuildTree is a sequential pre-order DFS with ONE visited set per request (created at the root,
// graph_utils.go:35-50): a subject set already visited returns nil, a set without rows returns
// nil, rest depth <= 1 turns a set with rows into a Leaf, otherwise a Union whose children are the
// row subjects in shard order (nil children become Leaf{row subject}).  The depth clamp
// (engine.go:37-39) is re-applied per level but is the identity below the root (children get
// d-1 >= 1).
//
// One wave64 per root.  Every row subject yields exactly one child record, so a Union's child
// count (its row length) is known when it is emitted and the output is a single pre-order stream.
// Order only matters for subject sets that will be EXPANDED (unvisited, rows non-empty, d-1 >= 2):
// everything before the first such candidate in a 64-wide row chunk is emitted in parallel as
// leaves, candidates are visited strictly in row order.  Output streams go to 1024-record chunks
// of an HBM arena (bump allocator), then a compaction kernel lays each root out contiguously.
// Visited sets live in LDS (pass 1); roots that outgrow LDS rerun with an HBM bitmap (pass 2).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "kg_bfs.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

constexpr uint32_t CHUNK = 256;  // records per arena chunk

// A DFS frame carries its node's row range, so neither a push (the candidate's range is known from
// the parent's chunk scan) nor a pop re-reads row_off on the walk's dependent chain.
struct ExpFrame {
  uint64_t rb;
  uint32_t node;
  uint32_t cursor;
  uint32_t len;
  int32_t d;
};

struct ExpCtl {
  uint32_t arena_head;   // next free chunk
  uint32_t overflow;     // arena exhausted
  uint32_t p2_count, p2_head;
  uint32_t head;         // pass-1 dequeue
  uint32_t p3_count, p3_head;  // pass-3 (full bitmap) queue: pass-2 overflows
  uint32_t pad;
  unsigned long long records;
  // gather-walk passes (expand_gw): the small slots take the pass-1 overflows (p2), the large slots
  // what outgrew a small slot (ga), the hash pass what outgrew a large one (gb)
  uint32_t gs_head, ga_count, ga_head, gb_count, gb_head, gw_small_done, pad2[2];
  unsigned long long gw_ticks[4];  // longest gather / walk of one root, small and large slots (wall clock, 100 MHz)
  unsigned long long gw_stat[8];   // diagnostics (sums over roots): chunks, unions at rest depth 2 / 3 / 4 / >= 5, pops, entries gathered
  // round 6: the arena's chunks and pass 1's roots are cut into 8 ranges, each claimed through its own
  // head on a 128-B line of its own.  One word saturates near 90 M atomics/s (MI355X_MICROARCH.md
  // "dequeue"): a C5 call's ~100 k root dequeues and ~100 k chunk claims on two words were a ~1.1 ms
  // floor under k_expand_lds.
  alignas(128) uint32_t ahead[8 * 32];
  uint32_t rhead[8 * 32];
  uint32_t qhead[8 * 32];  // the 64-lane pass's heads over pass 0's overflow list
  uint32_t p0_count, pad3[31];
};

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A free arena chunk (lane 0 only): from the range of this workgroup's XCD label, then the others;
// NONE when all eight are used up.
__device__ __forceinline__ uint32_t claim_chunk(ExpCtl* ctl, uint32_t n_chunks) {
  const uint32_t per = (n_chunks + 7) / 8;
  uint32_t sh = blockIdx.x & 7;
  for (int k = 0; k < 8; k++, sh = (sh + 1) & 7) {
    const uint32_t lo = sh * per, hi = min(n_chunks, lo + per);
    if (lo >= hi) continue;
    if (ld_sc1(&ctl->ahead[sh * 32]) >= hi - lo) continue;  // dry: no atomic
    const uint32_t c = atomicAdd(&ctl->ahead[sh * 32], 1u);
    if (c < hi - lo) return lo + c;
  }
  return NONE;
}

// Per-root result of the DFS: first chunk and record count (0 records = nil tree).
struct RootOut {
  uint32_t first_chunk;
  uint32_t count;
};

struct Stream {
  kg_tree_node* arena;
  uint32_t* next;  // chunk -> next chunk
  uint32_t n_chunks;
  ExpCtl* ctl;
  uint32_t first, cur, pos;  // wave-uniform
  bool ok;
};

__device__ __forceinline__ uint32_t alloc_chunk(Stream& S) {
  uint32_t c = 0;
  if (lane_id() == 0) c = claim_chunk(S.ctl, S.n_chunks);
  c = __shfl(c, 0, 64);
  if (c >= S.n_chunks) {
    if (lane_id() == 0) S.ctl->overflow = 1;
    S.ok = false;
    return NONE;
  }
  if (lane_id() == 0) S.next[c] = NONE;
  return c;
}

// Lanes with `pred` append one record each, in lane order, to the wave's stream.
__device__ __forceinline__ void emit(Stream& S, bool pred, const kg_tree_node& r) {
  const uint64_t m = __ballot(pred);
  if (!m || !S.ok) return;
  const uint32_t cnt = __popcll(m);
  const uint32_t rank = lanes_below(m);
  uint32_t room = CHUNK - S.pos;
  uint32_t nxt = NONE;
  if (cnt > room) {
    nxt = alloc_chunk(S);
    if (!S.ok) return;
    if (lane_id() == 0) S.next[S.cur] = nxt;
  }
  if (pred) {
    if (rank < room) S.arena[(size_t)S.cur * CHUNK + S.pos + rank] = r;
    else S.arena[(size_t)nxt * CHUNK + (rank - room)] = r;
  }
  if (cnt > room) {
    S.cur = nxt;
    S.pos = cnt - room;
  } else {
    S.pos += cnt;
  }
}

__device__ __forceinline__ kg_tree_node rec_set(const DevSnap& s, uint8_t type, uint32_t node, uint32_t nch) {
  kg_tree_node r;
  r.type = type;
  r.is_set = 1;
  r.pad = 0;
  r.ns = s.nd_ns[node];
  r.obj = s.nd_obj[node];
  r.rel = s.nd_rel[node];
  r.n_children = nch;
  return r;
}
__device__ __forceinline__ kg_tree_node rec_subject(const DevSnap& s, uint32_t sub) {
  if (sub & SET_BIT) return rec_set(s, 2, sub & ~SET_BIT, 0);
  kg_tree_node r;
  r.type = 2;
  r.is_set = 0;
  r.pad = 0;
  r.ns = KG_SUBJECT_ID;
  r.obj = sub;
  r.rel = 0;
  r.n_children = 0;
  return r;
}

enum : int { EXP_OK = 0, EXP_OVERFLOW = 1, EXP_ARENA = 2 };

template <class Store>
__device__ int expand_root(const DevSnap& s, Store& st, const kg_set& root, int32_t global, ExpFrame* stack,
                           Stream& S, uint32_t& n_records) {
  const int lane = lane_id();
  S.ok = true;
  S.pos = 0;
  S.first = S.cur = alloc_chunk(S);
  n_records = 0;
  if (!S.ok) return EXP_ARENA;
  int32_t d = root.max_depth;
  if (d <= 0 || global < d) d = global;  // engine.go:37-39
  if (root.sns == KG_SUBJECT_ID) {       // SubjectID -> Leaf
    emit(S, lane == 0, rec_subject(s, root.sobj < 0x7FFFFFFFu ? root.sobj : 0x7FFFFFFFu));
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  const uint32_t rn = nmap_find(s, root.sns, root.srel, root.sobj);
  if (rn == NONE) return EXP_OK;  // no rows anywhere: nil
  st.reset();
  uint32_t n_vis = 0;
  wave_add_roots(st, lane == 0, rn, n_vis);  // marks the root visited
  const uint64_t rb0 = s.row_off[rn], re0 = s.row_off[rn + 1];
  if (rb0 == re0) {
    st.finish(n_vis);
    return EXP_OK;  // no rows: nil
  }
  if (d <= 1) {
    emit(S, lane == 0, rec_set(s, 2, rn, 0));
    st.finish(n_vis);
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  emit(S, lane == 0, rec_set(s, 1, rn, (uint32_t)(re0 - rb0)));
  uint32_t count = 1;
  int sp = 0;
  ExpFrame F{rb0, rn, 0, (uint32_t)(re0 - rb0), d};
  int status = EXP_OK;
  for (;;) {
    const uint64_t rb = F.rb, re = F.rb + F.len;
    const bool can_expand = F.d - 1 >= 2;
    bool pushed = false;
    while (rb + F.cursor < re) {
      const uint64_t i = rb + F.cursor + lane;
      const bool valid = i < re;
      const uint32_t sub = valid ? s.row_subj[i] : 0;
      bool cand = false;
      uint64_t crb = 0, cre = 0;
      if (valid && can_expand && (sub & SET_BIT)) {
        const uint32_t c = sub & ~SET_BIT;
        crb = s.row_off[c];
        cre = s.row_off[c + 1];
        // a set visited before this chunk is a leaf whatever comes first (the visited set only
        // grows): only unvisited sets with rows are order-dependent candidates, taken one by one.
        // The visited lookup does not wait for the row range (both depend on the subject only).
        const bool seen = st.contains(c);
        cand = cre > crb && !seen;
      }
      const uint64_t mc = __ballot(cand);
      const uint32_t p = mc ? (uint32_t)(__ffsll((unsigned long long)mc) - 1) : 64u;
      // everything before the first candidate: leaves (and marks, order-free for non-candidates)
      const bool leaf = valid && (uint32_t)lane < p;
      // d-1 <= 1: child sets become leaves but BuildTree still marks them visited, which a later
      // (shallower) encounter elsewhere in the tree observes.  Sets without rows need no mark:
      // any encounter of them is a leaf.  SubjectIDs are never marked (engine.go:41-45).
      if (!can_expand && !wave_add_roots(st, leaf && (sub & SET_BIT), sub & ~SET_BIT, n_vis)) {
        status = EXP_OVERFLOW;
        break;
      }
      emit(S, leaf, rec_subject(s, sub));
      count += __popcll(__ballot(leaf));
      if (!S.ok) return EXP_ARENA;
      if (p == 64u) {
        F.cursor += (uint32_t)min<uint64_t>(64, re - (rb + F.cursor));
        continue;
      }
      // candidate at lane p, in order
      const uint32_t csub = __shfl(sub, (int)p, 64);
      const uint32_t cnode = csub & ~SET_BIT;
      const uint32_t clen = (uint32_t)(__shfl((uint32_t)(cre - crb), (int)p, 64));
      const uint64_t cbeg = ((uint64_t)(uint32_t)__shfl((uint32_t)(crb >> 32), (int)p, 64) << 32) |
                            (uint32_t)__shfl((uint32_t)crb, (int)p, 64);
      F.cursor += p + 1;
      const uint32_t before = n_vis;
      if (!wave_add_roots(st, lane == 0, cnode, n_vis)) {
        status = EXP_OVERFLOW;
        break;
      }
      if (n_vis == before) {  // already visited: BuildTree -> nil -> Leaf{row subject}
        emit(S, lane == 0, rec_subject(s, csub));
        count++;
        if (!S.ok) return EXP_ARENA;
        continue;
      }
      emit(S, lane == 0, rec_set(s, 1, cnode, clen));
      count++;
      if (!S.ok) return EXP_ARENA;
      if (sp >= 0x7FFF) {
        status = EXP_OVERFLOW;
        break;
      }
      if (lane == 0) stack[sp] = F;
      sp++;
      F = ExpFrame{cbeg, cnode, 0, clen, F.d - 1};
      pushed = true;
      break;
    }
    if (status != EXP_OK) break;
    if (pushed) continue;
    if (sp == 0) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    sp--;
    F = stack[sp];
  }
  st.finish((uint32_t)min<uint64_t>(n_vis, st.cap()));
  n_records = count;
  return status;
}



// Passes 2 and 3 hold the batch's largest roots, whose walks are the batch's tail: one wave doing
// hundreds of thousands of dependent round trips (C5's largest tree: 335 k records, ~135 ms).  This
// variant of expand_root cuts the trips per expanded set:
//   * a chunk scan issues the child's row range, its node triple (for the record) and the visited
//     lookup in ONE round trip after the row_subj load, so leaves are emitted from registers;
//   * the frame stack and each frame's scanned chunk live in LDS (XF frames: C5's depth-5 walk needs
//     7), so a pop resumes the parent's chunk without re-reading row_subj / row_off / nd_* -- only the
//     visited lookups are redone (the set grew during the subtree);
//   * the candidate's insert is a plain store into the empty slot its lookup found (the table belongs
//     to this wave and nothing was inserted in between): no CAS round trip before the push.
// Output is identical to expand_root (same candidates in the same order).
constexpr int XF = 16;
struct ExpLds {
  ExpFrame fr[XF];
  uint64_t cbase[XF];  // row position of lane 0 of the frame's cached chunk
  uint32_t cn[XF];     // cached lanes (0: none)
  uint32_t sub[XF][64], clen[XF][64], ns[XF][64], obj[XF][64], rel[XF][64];
  uint64_t crb[XF][64];
};

template <class Store>
__device__ int expand_root_x(const DevSnap& s, Store& st, const kg_set& root, int32_t global, ExpFrame* gstack,
                             Stream& S, uint32_t& n_records, ExpLds& X) {
  const int lane = lane_id();
  S.ok = true;
  S.pos = 0;
  S.first = S.cur = alloc_chunk(S);
  n_records = 0;
  if (!S.ok) return EXP_ARENA;
  int32_t d = root.max_depth;
  if (d <= 0 || global < d) d = global;  // engine.go:37-39
  if (root.sns == KG_SUBJECT_ID) {       // SubjectID -> Leaf
    emit(S, lane == 0, rec_subject(s, root.sobj < 0x7FFFFFFFu ? root.sobj : 0x7FFFFFFFu));
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  const uint32_t rn = nmap_find(s, root.sns, root.srel, root.sobj);
  if (rn == NONE) return EXP_OK;  // no rows anywhere: nil
  st.reset();
  uint32_t n_vis = 0;
  wave_add_roots(st, lane == 0, rn, n_vis);  // marks the root visited
  const uint64_t rb0 = s.row_off[rn], re0 = s.row_off[rn + 1];
  if (rb0 == re0) {
    st.finish(n_vis);
    return EXP_OK;
  }
  if (d <= 1) {
    emit(S, lane == 0, rec_set(s, 2, rn, 0));
    st.finish(n_vis);
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  emit(S, lane == 0, rec_set(s, 1, rn, (uint32_t)(re0 - rb0)));
  uint32_t count = 1;
  int sp = 0;
  if (lane < XF) X.cn[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  ExpFrame F{rb0, rn, 0, (uint32_t)(re0 - rb0), d};
  int status = EXP_OK;
  for (;;) {
    const uint64_t rb = F.rb, re = F.rb + F.len;
    const bool can_expand = F.d - 1 >= 2;
    bool pushed = false;
    while (rb + F.cursor < re) {
      const uint64_t at0 = rb + F.cursor;
      // the chunk: the rest of this frame's cached chunk if the cursor is inside it, else a fresh one
      const bool cached = sp < XF && X.cn[sp] && at0 >= X.cbase[sp] && at0 < X.cbase[sp] + X.cn[sp];
      uint32_t sub = 0, clen = 0, nns = 0, nobj = 0, nrel = 0;
      uint64_t crb = 0;
      bool valid;
      uint32_t width;
      if (cached) {
        const uint32_t k0 = (uint32_t)(at0 - X.cbase[sp]);
        width = X.cn[sp] - k0;
        valid = (uint32_t)lane < width;
        const uint32_t k = valid ? k0 + lane : 0u;
        sub = X.sub[sp][k];
        clen = X.clen[sp][k];
        crb = X.crb[sp][k];
        nns = X.ns[sp][k];
        nobj = X.obj[sp][k];
        nrel = X.rel[sp][k];
      } else {
        width = (uint32_t)min<uint64_t>(64, re - at0);
        valid = (uint32_t)lane < width;
        sub = s.row_subj[valid ? at0 + lane : at0];
        const bool set = valid && (sub & SET_BIT);
        const uint32_t c = set ? sub & ~SET_BIT : 0u;  // node 0 exists: unconditional loads, no waits in branches
        const uint64_t r0 = s.row_off[c], r1 = s.row_off[c + 1];
        nns = s.nd_ns[c];
        nobj = s.nd_obj[c];
        nrel = s.nd_rel[c];
        crb = set ? r0 : 0;
        clen = set ? (uint32_t)(r1 - r0) : 0u;
        if (sp < XF) {
          X.sub[sp][lane] = sub;
          X.clen[sp][lane] = clen;
          X.crb[sp][lane] = crb;
          X.ns[sp][lane] = nns;
          X.obj[sp][lane] = nobj;
          X.rel[sp][lane] = nrel;
          if (lane == 0) {
            X.cbase[sp] = at0;
            X.cn[sp] = width;
          }
        }
      }
      const bool is_set = valid && (sub & SET_BIT);
      const uint32_t c = sub & ~SET_BIT;
      bool cand = false;
      uint32_t vat = 0;
      if (is_set && can_expand) {
        // a set visited before this chunk is a leaf whatever comes first (the visited set only
        // grows): only unvisited sets with rows are order-dependent candidates, taken one by one
        const bool seen = st.find(c, vat);
        cand = clen > 0 && !seen;
      }
      const uint64_t mc = __ballot(cand);
      const uint32_t p = mc ? (uint32_t)(__ffsll((unsigned long long)mc) - 1) : 64u;
      // everything before the first candidate: leaves (and marks, order-free for non-candidates)
      const bool leaf = valid && (uint32_t)lane < p;
      // d-1 <= 1: child sets become leaves but BuildTree still marks them visited, which a later
      // (shallower) encounter elsewhere in the tree observes.  SubjectIDs are never marked.
      if (!can_expand && !wave_add_roots(st, leaf && is_set, c, n_vis)) {
        status = EXP_OVERFLOW;
        break;
      }
      kg_tree_node r;
      r.type = 2;
      r.pad = 0;
      r.n_children = 0;
      r.is_set = is_set ? 1 : 0;
      r.ns = is_set ? nns : KG_SUBJECT_ID;
      r.obj = is_set ? nobj : sub;
      r.rel = is_set ? nrel : 0u;
      emit(S, leaf, r);
      count += __popcll(__ballot(leaf));
      if (!S.ok) return EXP_ARENA;
      if (p == 64u) {
        F.cursor += width;
        continue;
      }
      // candidate at lane p, in order: unvisited when its lookup ran, and nothing was inserted since
      const uint32_t cnode = __shfl(c, (int)p, 64);
      const uint32_t cl = __shfl(clen, (int)p, 64);
      const uint32_t cat = __shfl(vat, (int)p, 64);
      const uint64_t cbeg = ((uint64_t)(uint32_t)__shfl((uint32_t)(crb >> 32), (int)p, 64) << 32) |
                            (uint32_t)__shfl((uint32_t)crb, (int)p, 64);
      kg_tree_node u;
      u.type = 1;
      u.is_set = 1;
      u.pad = 0;
      u.ns = __shfl(nns, (int)p, 64);
      u.obj = __shfl(nobj, (int)p, 64);
      u.rel = __shfl(nrel, (int)p, 64);
      u.n_children = cl;
      F.cursor += p + 1;
      if (n_vis + 1 > st.cap()) {
        status = EXP_OVERFLOW;
        break;
      }
      if (lane == 0) {
        st.put_new(cnode, cat);
        st.list()[n_vis] = cnode;
      }
      n_vis++;
      emit(S, lane == 0, u);
      count++;
      if (!S.ok) return EXP_ARENA;
      if (sp >= 0x7FFF) {
        status = EXP_OVERFLOW;
        break;
      }
      if (lane == 0) {
        if (sp < XF) X.fr[sp] = F;
        else gstack[sp] = F;
      }
      sp++;
      if (lane == 0 && sp < XF) X.cn[sp] = 0;  // the child frame starts without a cached chunk
      __builtin_amdgcn_wave_barrier();
      F = ExpFrame{cbeg, cnode, 0, cl, F.d - 1};
      pushed = true;
      break;
    }
    if (status != EXP_OK) break;
    if (pushed) continue;
    if (sp == 0) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    sp--;
    F = sp < XF ? X.fr[sp] : gstack[sp];
  }
  st.finish((uint32_t)min<uint64_t>(n_vis, st.cap()));
  n_records = count;
  return status;
}

// ------------------------------------------------------------------ pass 0: 16-lane walkers (round 6)
// C5's ~100 k hot roots average ~45 records (a handful of expanded sets each): one 64-lane wave per
// root left most lanes idle on every row chunk and paid a whole wave's chain of dependent round trips
// per root.  Here a wave runs FOUR roots at once, one per 16-lane group, with expand_root's exact
// pre-order (the same chunk scan, 16 entries at a time, first-candidate rule, one visited set per
// request).  Each walker has its own LDS visited hash and record stream; a root that outgrows the
// small hash or SW_RECS records is given up (its chunks are abandoned) and redone by the 64-lane pass.
constexpr int SW = 16;
constexpr int SW_VL2 = 9;           // visited-hash slots per walker (512)
constexpr uint32_t SW_CAP = 224;    // visited sets per walker (hash load <= ~0.5)
constexpr uint32_t SW_RECS = 2048;  // records per root before it is handed to the 64-lane pass
__device__ __forceinline__ int sw_lane() { return lane_id() & (SW - 1); }
__device__ __forceinline__ int sw_base() { return lane_id() & ~(SW - 1); }
__device__ __forceinline__ uint32_t sw_bits(uint64_t m) { return (uint32_t)(m >> sw_base()) & 0xFFFFu; }
__device__ __forceinline__ uint32_t sw_below(uint32_t m) { return (uint32_t)__popc(m & ((1u << sw_lane()) - 1)); }

struct SubStore {
  uint32_t* vis;  // 1 << SW_VL2 slots
  __device__ void reset() const {
    for (int i = sw_lane() * 4; i < (1 << SW_VL2); i += SW * 4)
      *reinterpret_cast<uint4*>(&vis[i]) = make_uint4(NONE, NONE, NONE, NONE);
    __builtin_amdgcn_wave_barrier();
  }
  __device__ bool insert(uint32_t key) const {
    uint32_t h = (key * 2654435761u) >> (32 - SW_VL2);
    for (int p = 0; p < (1 << SW_VL2); p++) {
      const uint32_t old = atomicCAS(&vis[h], NONE, key);
      if (old == NONE) return true;
      if (old == key) return false;
      h = (h + 1) & ((1u << SW_VL2) - 1);
    }
    return true;
  }
  __device__ bool contains(uint32_t key) const {
    uint32_t h = (key * 2654435761u) >> (32 - SW_VL2);
    for (int p = 0; p < (1 << SW_VL2); p++) {
      const uint32_t k = vis[h];
      if (k == key) return true;
      if (k == NONE) return false;
      h = (h + 1) & ((1u << SW_VL2) - 1);
    }
    return false;
  }
};

// group-uniform values: S.cur / S.pos / S.first / S.ok are the same in the walker's 16 lanes
__device__ __forceinline__ uint32_t sw_alloc_chunk(Stream& S) {
  uint32_t c = 0;
  if (sw_lane() == 0) c = claim_chunk(S.ctl, S.n_chunks);
  c = __shfl(c, sw_base(), 64);
  if (c >= S.n_chunks) {
    if (sw_lane() == 0) S.ctl->overflow = 1;
    S.ok = false;
    return NONE;
  }
  if (sw_lane() == 0) S.next[c] = NONE;
  return c;
}

__device__ __forceinline__ void sw_emit(Stream& S, bool pred, const kg_tree_node& r) {
  const uint32_t m = sw_bits(__ballot(pred));
  if (!m || !S.ok) return;
  const uint32_t cnt = (uint32_t)__popc(m), rank = sw_below(m);
  const uint32_t room = CHUNK - S.pos;
  uint32_t nxt = NONE;
  if (cnt > room) {
    nxt = sw_alloc_chunk(S);
    if (!S.ok) return;
    if (sw_lane() == 0) S.next[S.cur] = nxt;
  }
  if (pred) {
    if (rank < room) S.arena[(size_t)S.cur * CHUNK + S.pos + rank] = r;
    else S.arena[(size_t)nxt * CHUNK + (rank - room)] = r;
  }
  if (cnt > room) {
    S.cur = nxt;
    S.pos = cnt - room;
  } else {
    S.pos += cnt;
  }
}

// marks `node` (lanes with `offer`); false when the walker's visited cap would be passed
__device__ __forceinline__ bool sw_add(const SubStore& st, bool offer, uint32_t node, uint32_t& n_vis) {
  const bool fresh = offer && st.insert(node);
  const uint32_t cnt = (uint32_t)__popc(sw_bits(__ballot(fresh)));
  if (n_vis + cnt > SW_CAP) return false;
  n_vis += cnt;
  return true;
}

// expand_root (above) on one 16-lane walker: identical records in identical order, or EXP_OVERFLOW
__device__ int expand_root_sw(const DevSnap& s, const SubStore& st, const kg_set& root, int32_t global,
                              ExpFrame* stack, uint32_t stack_cap, Stream& S, uint32_t& n_records) {
  const int gl = sw_lane(), gb = sw_base();
  S.ok = true;
  S.pos = 0;
  S.first = S.cur = sw_alloc_chunk(S);
  n_records = 0;
  if (!S.ok) return EXP_ARENA;
  int32_t d = root.max_depth;
  if (d <= 0 || global < d) d = global;  // engine.go:37-39
  if (root.sns == KG_SUBJECT_ID) {       // SubjectID -> Leaf
    sw_emit(S, gl == 0, rec_subject(s, root.sobj < 0x7FFFFFFFu ? root.sobj : 0x7FFFFFFFu));
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  const uint32_t rn = nmap_find(s, root.sns, root.srel, root.sobj);
  if (rn == NONE) return EXP_OK;  // no rows anywhere: nil
  st.reset();
  uint32_t n_vis = 0;
  sw_add(st, gl == 0, rn, n_vis);  // marks the root visited
  const uint64_t rb0 = s.row_off[rn], re0 = s.row_off[rn + 1];
  if (rb0 == re0) return EXP_OK;  // no rows: nil
  if (d <= 1) {
    sw_emit(S, gl == 0, rec_set(s, 2, rn, 0));
    n_records = 1;
    return S.ok ? EXP_OK : EXP_ARENA;
  }
  sw_emit(S, gl == 0, rec_set(s, 1, rn, (uint32_t)(re0 - rb0)));
  uint32_t count = 1;
  uint32_t sp = 0;
  ExpFrame F{rb0, rn, 0, (uint32_t)(re0 - rb0), d};
  int status = EXP_OK;
  for (;;) {
    const uint64_t rb = F.rb, re = F.rb + F.len;
    const bool can_expand = F.d - 1 >= 2;
    bool pushed = false;
    while (rb + F.cursor < re) {
      if (count > SW_RECS) {
        status = EXP_OVERFLOW;
        break;
      }
      const uint64_t i = rb + F.cursor + gl;
      const bool valid = i < re;
      const uint32_t sub = valid ? s.row_subj[i] : 0;
      bool cand = false;
      uint64_t crb = 0, cre = 0;
      if (valid && can_expand && (sub & SET_BIT)) {
        const uint32_t c = sub & ~SET_BIT;
        crb = s.row_off[c];
        cre = s.row_off[c + 1];
        cand = cre > crb && !st.contains(c);
      }
      const uint32_t mc = sw_bits(__ballot(cand));
      const uint32_t p = mc ? (uint32_t)(__ffs(mc) - 1) : (uint32_t)SW;
      const bool leaf = valid && (uint32_t)gl < p;
      if (!can_expand && !sw_add(st, leaf && (sub & SET_BIT), sub & ~SET_BIT, n_vis)) {
        status = EXP_OVERFLOW;
        break;
      }
      sw_emit(S, leaf, rec_subject(s, sub));
      count += (uint32_t)__popc(sw_bits(__ballot(leaf)));
      if (!S.ok) return EXP_ARENA;
      if (p == (uint32_t)SW) {
        F.cursor += (uint32_t)min<uint64_t>(SW, re - (rb + F.cursor));
        continue;
      }
      const int src = gb + (int)p;
      const uint32_t csub = __shfl(sub, src, 64);
      const uint32_t cnode = csub & ~SET_BIT;
      const uint32_t clen = (uint32_t)__shfl((uint32_t)(cre - crb), src, 64);
      const uint64_t cbeg = ((uint64_t)(uint32_t)__shfl((uint32_t)(crb >> 32), src, 64) << 32) |
                            (uint32_t)__shfl((uint32_t)crb, src, 64);
      F.cursor += p + 1;
      const uint32_t before = n_vis;
      if (!sw_add(st, gl == 0, cnode, n_vis)) {
        status = EXP_OVERFLOW;
        break;
      }
      if (n_vis == before) {  // already visited: BuildTree -> nil -> Leaf{row subject}
        sw_emit(S, gl == 0, rec_subject(s, csub));
        count++;
        if (!S.ok) return EXP_ARENA;
        continue;
      }
      sw_emit(S, gl == 0, rec_set(s, 1, cnode, clen));
      count++;
      if (!S.ok) return EXP_ARENA;
      if (sp >= stack_cap) {
        status = EXP_OVERFLOW;
        break;
      }
      if (gl == 0) stack[sp] = F;
      sp++;
      F = ExpFrame{cbeg, cnode, 0, clen, F.d - 1};
      pushed = true;
      break;
    }
    if (status != EXP_OK) break;
    if (pushed) continue;
    if (sp == 0) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    sp--;
    F = stack[sp];
  }
  n_records = count;
  return status;
}

// Pass 0: every root, 16 walkers per workgroup; what a walker gives up goes to the p0 list (the 64-lane
// pass).  Roots are dequeued through ExpCtl::rhead (8 ranges), one walker at a time.
__global__ __launch_bounds__(256) void k_expand_sub(DevSnap s, const kg_set* __restrict__ roots, uint32_t n,
                                                    int32_t global, ExpCtl* ctl, RootOut* outs, kg_tree_node* arena,
                                                    uint32_t* next, uint32_t n_chunks, ExpFrame* stacks,
                                                    uint32_t stack_cap, uint32_t* p0_list) {
  __shared__ uint32_t vis_all[256 / SW][1 << SW_VL2];
  __shared__ unsigned long long s_recs;
  if (threadIdx.x == 0) s_recs = 0;
  __syncthreads();
  const int walker = threadIdx.x / SW, gl = sw_lane();
  const SubStore st{vis_all[walker]};
  ExpFrame* stack = stacks + ((size_t)blockIdx.x * (256 / SW) + walker) * stack_cap;
  Stream S{arena, next, n_chunks, ctl, 0, 0, 0, true};
  unsigned long long recs = 0;
  const uint32_t rper = (n + 7) / 8;
  uint32_t r_at = blockIdx.x & 7, r_tried = 0;
  for (;;) {
    uint32_t ri = NONE;
    if (gl == 0)
      for (; r_tried < 8; r_tried++, r_at = (r_at + 1) & 7) {
        const uint32_t lo = r_at * rper, hi = min(n, lo + rper);
        if (lo >= hi || ld_sc1(&ctl->rhead[r_at * 32]) >= hi - lo) continue;
        const uint32_t k = atomicAdd(&ctl->rhead[r_at * 32], 1u);
        if (k < hi - lo) {
          ri = lo + k;
          break;
        }
      }
    ri = __shfl(ri, sw_base(), 64);
    if (ri >= n) break;
    uint32_t nr = 0;
    const int r = expand_root_sw(s, st, roots[ri], global, stack, stack_cap, S, nr);
    if (gl == 0) {
      if (r == EXP_OVERFLOW) {
        p0_list[atomicAdd(&ctl->p0_count, 1u)] = ri;
        outs[ri] = RootOut{NONE, 0};
      } else {
        outs[ri] = RootOut{S.first, nr};
        recs += nr;
      }
    }
  }
  if (gl == 0 && recs) atomicAdd(&s_recs, recs);  // one device atomic per workgroup, not per walker
  __syncthreads();
  if (threadIdx.x == 0 && s_recs) atomicAdd(&ctl->records, s_recs);
}

__global__ __launch_bounds__(256) void k_expand_lds(DevSnap s, const kg_set* __restrict__ roots, uint32_t n,
                                                    int32_t global, ExpCtl* ctl, RootOut* outs, kg_tree_node* arena,
                                                    uint32_t* next, uint32_t n_chunks, ExpFrame* stacks,
                                                    uint32_t stack_cap, uint32_t* p2_list, int skip,
                                                    const uint32_t* qlist) {
  __shared__ WaveLds lds_all[4];
  const int wave = threadIdx.x >> 6, lane = lane_id();
  LdsStore st{&lds_all[wave]};
  ExpFrame* stack = stacks + (size_t)(blockIdx.x * 4 + wave) * stack_cap;
  Stream S{arena, next, n_chunks, ctl, 0, 0, 0, true};
  unsigned long long recs = 0;
  // roots in 8 ranges, each dequeued through its own head (ExpCtl::rhead; with qlist -- pass 0's
  // overflows, ctl->p0_count of them -- ExpCtl::qhead): this XCD's range first
  const uint32_t cnt = qlist ? ctl->p0_count : n;
  uint32_t* heads = qlist ? ctl->qhead : ctl->rhead;
  const uint32_t rper = (cnt + 7) / 8;
  uint32_t r_at = blockIdx.x & 7, r_tried = 0;
  for (;;) {
    uint32_t ri = NONE;
    if (lane == 0)
      for (; r_tried < 8; r_tried++, r_at = (r_at + 1) & 7) {
        const uint32_t lo = r_at * rper, hi = min(cnt, lo + rper);
        if (lo >= hi || ld_sc1(&heads[r_at * 32]) >= hi - lo) continue;
        const uint32_t k = atomicAdd(&heads[r_at * 32], 1u);
        if (k < hi - lo) {
          ri = qlist ? qlist[lo + k] : lo + k;
          break;
        }
      }
    ri = __shfl(ri, 0, 64);
    if (ri >= n) break;
    uint32_t nr = 0;
    const int r = skip ? EXP_OVERFLOW : expand_root(s, st, roots[ri], global, stack, S, nr);
    if (lane == 0) {
      if (r == EXP_OVERFLOW) {
        p2_list[atomicAdd(&ctl->p2_count, 1u)] = ri;
        outs[ri] = RootOut{NONE, 0};
      } else {
        outs[ri] = RootOut{S.first, nr};
        recs += nr;
      }
    }
  }
  if (lane == 0) atomicAdd(&ctl->records, recs);
}

// Passes 2 and 3: one wave per slot over a queue of roots.  Pass 2 (many slots): bounded HBM
// visited hash + list (HashStore); a root that overflows it zeroes its table (keys inserted but
// never listed would stay behind) and moves to pass 3.  Pass 3 (one slot): HBM bitmap over the
// whole graph + a list that holds every node; marks are always listed so they can be cleared.
template <class Store>
__device__ void expand_slot_loop(const DevSnap& s, const kg_set* __restrict__ roots, int32_t global, ExpCtl* ctl,
                                 RootOut* outs, kg_tree_node* arena, uint32_t* next, uint32_t n_chunks,
                                 ExpFrame* stack, const uint32_t* qlist, uint32_t count, uint32_t* head, Store& st,
                                 uint32_t* clear_base, uint64_t clear_words, uint32_t* p3_list) {
  __shared__ ExpLds X;
  const int lane = lane_id();
  Stream S{arena, next, n_chunks, ctl, 0, 0, 0, true};
  unsigned long long recs = 0;
  for (;;) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(head, 1u);
    k = __shfl(k, 0, 64);
    if (k >= count) break;
    const uint32_t ri = qlist[k];
    uint32_t nr = 0;
    // the walk with LDS-cached frames (round 3; the "expand_tail" knob that kept round 2's walk beside
    // it was removed in round 6)
    const int r = expand_root_x(s, st, roots[ri], global, stack, S, nr, X);
    if (r == EXP_OVERFLOW && p3_list) {
      uint4* b4 = reinterpret_cast<uint4*>(clear_base);  // clear_words: multiple of 4, 16-B aligned
      for (uint64_t i = lane; i < clear_words / 4; i += 64) b4[i] = make_uint4(0, 0, 0, 0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (lane == 0) p3_list[atomicAdd(&ctl->p3_count, 1u)] = ri;
      continue;
    }
    if (lane == 0) {
      outs[ri] = r == EXP_OK ? RootOut{S.first, nr} : RootOut{NONE, 0xFFFFFFFFu};
      recs += nr;
    }
  }
  if (lane == 0) atomicAdd(&ctl->records, recs);
}

__global__ __launch_bounds__(64) void k_expand_hash(DevSnap s, const kg_set* __restrict__ roots, int32_t global,
                                                    ExpCtl* ctl, RootOut* outs, kg_tree_node* arena, uint32_t* next,
                                                    uint32_t n_chunks, ExpFrame* stacks, uint32_t stack_cap,
                                                    const uint32_t* qlist, const uint32_t* qcount, uint32_t* qhead,
                                                    uint32_t* tabs, uint64_t tsize, uint32_t* lists, uint64_t cap,
                                                    uint32_t* p3_list) {
  __shared__ uint32_t pref[64];
  uint32_t* tab = tabs + (size_t)blockIdx.x * tsize;
  HashStore st{tab, (uint32_t)(tsize - 1), lists + (size_t)blockIdx.x * cap, cap, pref};
  expand_slot_loop(s, roots, global, ctl, outs, arena, next, n_chunks, stacks + (size_t)blockIdx.x * stack_cap, qlist,
                   *qcount, qhead, st, tab, tsize, p3_list);
}

__global__ __launch_bounds__(64) void k_expand_hbm(DevSnap s, const kg_set* __restrict__ roots, int32_t global,
                                                   ExpCtl* ctl, RootOut* outs, kg_tree_node* arena, uint32_t* next,
                                                   uint32_t n_chunks, ExpFrame* stack, const uint32_t* p3_list,
                                                   uint32_t* bm, uint64_t words, uint32_t* list, uint64_t cap) {
  __shared__ uint32_t pref[64];
  GlobalStore st{bm, list, cap, pref};
  expand_slot_loop(s, roots, global, ctl, outs, arena, next, n_chunks, stack, p3_list, ctl->p3_count, &ctl->p3_head, st,
                   bm, words, nullptr);
}

// ------------------------------------------------------------------ gather-then-walk (pass 2)
// A large root's pre-order walk is one wave's chain of dependent round trips: per expanded set, the
// 64-wide row chunk (row_subj), then the children's row ranges, node triples and visited lookups --
// two trips to HBM, ~2.8 us, so C5's largest tree (~115 k records) took ~42 ms alone.  Here a
// workgroup first GATHERS the root's neighbourhood in parallel and the walk then runs on that copy:
//   * level-synchronous BFS from the root to distance D-2 (the nodes the walk can expand: a node
//     expanded at rest depth >= 2 lies on a path of length <= D-2).  Every node within distance
//     D-1 that has rows gets a dense LOCAL id (an open-addressing map, epoch-tagged so it is never
//     cleared); every node within D-2 also gets its row COPIED into the slot's entry array, each
//     entry carrying everything the walk needs: the leaf record's triple, the child's local id, its
//     row length (the union record's child count) and the first entry of its copied row;
//   * a level's entries are one contiguous range (rows are allocated by a bump counter while the
//     level before runs), so the next level is edge-parallel over that range: a run-head mark per
//     row start and the head of each 64-entry tile find an entry's source row position;
//   * the walk (one wave) is expand_root_x's order over the copy: one trip per chunk (the slot's
//     recently written lines, L2 / MALL) and the visited set is an LDS bitmap over local ids.
// The output is identical to expand_root's (same candidates in the same order).  A root that outgrows
// a slot (entries, local ids, map probes) goes on to the next pass: small slots -> large slots ->
// the hash pass (expand_slot_loop) -> the whole-graph bitmap pass.
struct GwEnt {
  uint32_t sub;   // the row subject as stored (SET_BIT | node, or a subject id)
  uint32_t loc;   // the child set's local id (a set with rows), else NONE; during the gather: its map slot
  uint32_t ns, obj, rel;  // the leaf record's triple (KG_SUBJECT_ID, id, 0 for a subject id)
  uint32_t len;   // the child's row length (its union record's child count)
  uint32_t cb;    // first entry of the child's copied row (NONE: not copied, never expanded)
  uint32_t pad;
};
static_assert(sizeof(GwEnt) == 32, "two 16-B loads per entry");

struct GwSlots {
  GwEnt* ent;           // [slot][ent_cap]
  uint64_t* hsrc;       // [slot][ent_cap] source row position of a run head
  uint32_t* hmark;      // [slot][ent_cap] epoch at a run head
  uint32_t* tfirst;     // [slot][ent_cap / 64 + 1] run head of each 64-entry tile's first entry
  unsigned long long* map;  // [slot][2 * map_cap] key (epoch << 32 | node), value (cb << 32 | local id)
  uint32_t* epoch;      // [slot]
  uint32_t ent_cap, map_cap;  // map_cap: a power of two
  uint32_t loc_cap;           // local ids (<= GW_LDS_LOC, the walk's LDS bitmap)
};
constexpr uint32_t GW_LDS_LOC = 262144;


constexpr int GW_PROBES = 64;
// The map slot of `node` for this root (inserting it; *won: this thread inserted it), or -1 (probe bound).
__device__ __forceinline__ int64_t gw_insert(unsigned long long* map, uint32_t mask, uint32_t epoch, uint32_t node,
                                             bool* won) {
  const unsigned long long key = ((unsigned long long)epoch << 32) | node;
  uint32_t h = (uint32_t)mix64(node) & mask;
  *won = false;
  for (int p = 0; p < GW_PROBES; p++) {
    unsigned long long cur = ld_sc1(&map[2 * (size_t)h]);
    for (;;) {
      if (cur == key) return h;
      if ((uint32_t)(cur >> 32) == epoch) break;  // another node of this root
      const unsigned long long old = atomicCAS(&map[2 * (size_t)h], cur, key);
      if (old == cur) {
        *won = true;
        return h;
      }
      cur = old;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

// Marks the run [cb, cb + len) as copied from row position r0: head mark + the tile heads it starts.
__device__ __forceinline__ void gw_run(const GwSlots& g, uint64_t* hsrc, uint32_t* hmark, uint32_t* tfirst,
                                       uint32_t epoch, uint32_t cb, uint32_t len, uint64_t r0) {
  hsrc[cb] = r0;
  hmark[cb] = epoch;
  for (uint32_t t = (cb + 63) / 64; t * 64 < cb + len; t++) tfirst[t] = cb;
}

// A root handed on: ga (from a small slot; published as ri + 1 for the waiting large slots) or gb (from
// a large slot; read by the hash pass, a later kernel).  A ga entry whose ticket holder gave up waiting
// (GW_ABANDON, see k_expand_gw) goes to gb instead: the hash pass expands any root.
#define GW_ABANDON 0xFFFFFFFFu
__device__ __forceinline__ void gw_publish(uint32_t* list, uint32_t* count, uint32_t ri, bool big, uint32_t* gb_list,
                                           uint32_t* gb_count) {
  const uint32_t at = atomicAdd(count, 1u);
  if (big) list[at] = ri;
  else if (atomicCAS(&list[at], 0u, ri + 1) == GW_ABANDON) gb_list[atomicAdd(gb_count, 1u)] = ri;
}

// One launch, two slot classes: workgroups [0, n_big) hold large slots, the rest small ones.  Every
// workgroup takes pass-1 overflows (p2) from one queue; a root that outgrows a small slot is published
// on the ga queue, which the large slots drain once p2 is empty -- so the giant trees start as soon as
// a large slot is free instead of after the whole small-slot pass (two launches: ~12 + ~25 ms per C5
// call in series).  A large slot waits for ga items with s_sleep and leaves when every small
// workgroup has finished and the queue is drained (small workgroups never wait: the exit is reached).
// The wait is bounded (`wait_ticks`, kg_snapshot_tune("expand_gw_wait_us")): the small workgroups are
// dispatched after the large ones and need free CUs, so with other kernels holding the CUs a large slot
// must not depend on them forever.  Past the bound it abandons its ticket (CAS 0 -> GW_ABANDON; a root
// published there later goes to the hash pass) and leaves.  What outgrows a large slot goes on to the
// hash pass (gb).
__global__ __launch_bounds__(256) void k_expand_gw(DevSnap s, const kg_set* __restrict__ roots, int32_t global,
                                                   ExpCtl* ctl, RootOut* outs, kg_tree_node* arena, uint32_t* next,
                                                   uint32_t n_chunks, ExpFrame* stacks, uint32_t stack_cap,
                                                   const uint32_t* p2_list, uint32_t* ga_list, uint32_t* gb_list,
                                                   uint32_t n_roots, uint32_t n_big, GwSlots g_small, GwSlots g_big,
                                                   uint64_t wait_ticks) {
  __shared__ uint32_t vis[GW_LDS_LOC / 32];
  __shared__ uint32_t s_k, s_nloc, s_nent, s_bad, s_epoch, s_ri, s_src, s_p2dry;
  __shared__ ExpFrame s_fr[XF];
  // The walk's records are staged in LDS and leave one full arena chunk at a time: on CDNA a wave's
  // vmcnt counts stores as well as loads, so a record store per step made every next load of the copy
  // wait for the previous step's stores as well (the walk's step was ~1 us)
  __shared__ uint4 s_out[CHUNK * sizeof(kg_tree_node) / 16];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const bool big = blockIdx.x < n_big;
  const GwSlots& g = big ? g_big : g_small;
  const size_t slot = big ? blockIdx.x : blockIdx.x - n_big;
  const uint32_t n_small = gridDim.x - n_big;
  uint32_t* ovf_list = big ? gb_list : ga_list;
  uint32_t* ovf_count = big ? &ctl->gb_count : &ctl->ga_count;
  GwEnt* E = g.ent + slot * g.ent_cap;
  uint64_t* hsrc = g.hsrc + slot * g.ent_cap;
  uint32_t* hmark = g.hmark + slot * g.ent_cap;
  uint32_t* tfirst = g.tfirst + slot * (g.ent_cap / 64 + 1);
  unsigned long long* map = g.map + slot * 2 * (size_t)g.map_cap;
  ExpFrame* gstack = stacks + (size_t)blockIdx.x * stack_cap;
  const uint32_t mmask = g.map_cap - 1;
  const uint32_t p2_count = ctl->p2_count;  // written by pass 1 (the previous kernel)
  Stream S{arena, next, n_chunks, ctl, 0, 0, 0, true};
  unsigned long long recs = 0;
  if (threadIdx.x == 0) s_p2dry = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      uint32_t src = 0, ri = 0;
      if (!s_p2dry) {
        const uint32_t k = atomicAdd(&ctl->gs_head, 1u);
        if (k < p2_count) {
          src = 1;
          ri = p2_list[k];
        } else {
          s_p2dry = 1;
        }
      }
      if (!src && big) {
        const uint32_t k = atomicAdd(&ctl->ga_head, 1u);
        const uint64_t w0 = wall_clock64();
        // the list holds n_roots entries at most: a ticket past it can never be served
        for (; k < n_roots;) {
          const uint32_t v = ld_sc1(&ga_list[k]);  // ri + 1 once published (the list is zeroed per call)
          if (v) {
            src = 2;
            ri = v - 1;
            break;
          }
          if (ld_sc1(&ctl->gw_small_done) == n_small && ld_sc1(&ctl->ga_count) <= k) break;
          if (wall_clock64() - w0 >= wait_ticks) {  // give the ticket up; a publication that won the race is ours
            const uint32_t old = atomicCAS(&ga_list[k], 0u, GW_ABANDON);
            if (old) {
              src = 2;
              ri = old - 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(16);
        }
      }
      s_src = src;
      s_ri = ri;
    }
    __syncthreads();
    if (!s_src) break;
    const uint32_t ri = s_ri;
    const kg_set root = roots[ri];
    int32_t d0 = root.max_depth;
    if (d0 <= 0 || global < d0) d0 = global;  // engine.go:37-39
    const uint32_t rn = root.sns == KG_SUBJECT_ID ? NONE : nmap_find(s, root.sns, root.srel, root.sobj);
    const uint64_t rb0 = rn == NONE ? 0 : s.row_off[rn];
    const uint64_t len0 = rn == NONE ? 0 : s.row_off[rn + 1] - rb0;
    // pass 1 answers these itself; anything else unusual is left to the passes after this one
    bool bad = rn == NONE || len0 == 0 || d0 <= 1 || len0 > g.ent_cap;
    const unsigned long long t0 = wall_clock64();
    if (!bad) {
      if (threadIdx.x == 0) {
        s_epoch = ++g.epoch[slot];  // only this workgroup touches its slot
        s_nloc = 1;
        s_nent = (uint32_t)len0;
        s_bad = 0;
        bool won;
        const int64_t h = gw_insert(map, mmask, s_epoch, rn, &won);
        if (h < 0) s_bad = 1;
        else map[2 * (size_t)h + 1] = 0ull;  // copied at entry 0, local id 0
      }
      __syncthreads();
      const uint32_t epoch = s_epoch;
      if (threadIdx.x == 0) {
        hsrc[0] = rb0;
        hmark[0] = epoch;
      }
      for (uint32_t t = threadIdx.x; t * 64 < len0; t += 256) tfirst[t] = 0;
      __syncthreads();
      uint32_t lo = 0, hi = (uint32_t)len0;
      for (int lv = 0; lv <= d0 - 2 && lo < hi && !s_bad; lv++) {
        const bool alloc_next = lv + 1 <= d0 - 2;  // the children's rows are copied (the walk may expand them)
        // phase 1: every entry of the level's rows, 64-entry tiles per wave
        for (uint32_t t = lo / 64 + wave; t * 64 < hi; t += 4) {
          const uint32_t e = t * 64 + lane;
          const bool valid = e >= lo && e < hi;
          const bool head = valid && ld_sc1(&hmark[e]) == epoch;
          uint32_t hv = head ? e + 1 : 0u;
          if (lane == 0 && !head) hv = ld_sc1(&tfirst[t]) + 1;
          const uint32_t hpos = wave_incl_scan<DppMax>(hv) - 1;  // the run this entry belongs to
          if (valid) {
            const uint64_t src = ld_sc1(&hsrc[hpos]) + (e - hpos);
            const uint32_t sub = s.row_subj[src];
            const bool is_set = (sub & SET_BIT) != 0;
            const uint32_t c = is_set ? sub & ~SET_BIT : 0u;
            const uint64_t r0 = s.row_off[c], r1 = s.row_off[c + 1];
            const uint32_t ns = s.nd_ns[c], ob = s.nd_obj[c], rl = s.nd_rel[c];
            const uint32_t len = is_set ? (uint32_t)(r1 - r0) : 0u;
            GwEnt x{sub, NONE, is_set ? ns : (uint32_t)KG_SUBJECT_ID, is_set ? ob : sub, is_set ? rl : 0u, len, NONE, 0};
            if (len > 0) {
              bool won;
              const int64_t h = gw_insert(map, mmask, epoch, c, &won);
              if (h < 0) {
                s_bad = 1;
              } else {
                x.loc = (uint32_t)h;  // resolved to the local id in phase 2
                if (won) {
                  const uint32_t loc = atomicAdd(&s_nloc, 1u);
                  uint32_t cb = NONE;
                  if (loc >= g.loc_cap) s_bad = 1;
                  if (alloc_next) {
                    cb = atomicAdd(&s_nent, len);
                    if ((uint64_t)cb + len > g.ent_cap) {
                      s_bad = 1;
                      cb = NONE;
                    } else {
                      gw_run(g, hsrc, hmark, tfirst, epoch, cb, len, r0);
                    }
                  }
                  map[2 * (size_t)h + 1] = ((unsigned long long)cb << 32) | loc;
                }
              }
            }
            E[e] = x;
          }
        }
        __syncthreads();
        if (s_bad) break;
        // phase 2: the children's local ids and copied rows, now that every insert of the level is done
        for (uint32_t e = lo + threadIdx.x; e < hi; e += 256) {
          const uint32_t sub = ld_sc1(&E[e].sub), len = ld_sc1(&E[e].len);
          if ((sub & SET_BIT) && len > 0) {
            const unsigned long long v = ld_sc1(&map[2 * (size_t)ld_sc1(&E[e].loc) + 1]);
            E[e].loc = (uint32_t)v;
            E[e].cb = (uint32_t)(v >> 32);
          }
        }
        __syncthreads();
        lo = hi;
        hi = s_nent;
      }
      bad = s_bad != 0;
    }
    if (bad) {
      if (threadIdx.x == 0) gw_publish(ovf_list, ovf_count, ri, big, gb_list, &ctl->gb_count);
      __syncthreads();
      continue;
    }
    // the walk: wave 0 over the copy; the visited bitmap covers the root's local ids
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) atomicMax(&ctl->gw_ticks[big ? 2 : 0], t1 - t0);
    const uint32_t nloc = s_nloc;
    for (uint32_t w = threadIdx.x; w < (nloc + 31) / 32; w += 256) vis[w] = 0;
    __syncthreads();
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the copy was written by every wave: drop stale L1 lines
      int status = EXP_OK;
      uint32_t cnt = 0;
      S.ok = true;
      S.first = S.cur = NONE;
      uint32_t nbuf = 0;  // records staged in s_out (wave-uniform)
      kg_tree_node* sbuf = reinterpret_cast<kg_tree_node*>(s_out);
      // staged -> a new arena chunk (linked after the root's previous one); n records, n <= CHUNK
      auto flush = [&](uint32_t n) {
        uint32_t c = 0;
        if (lane == 0) c = claim_chunk(ctl, S.n_chunks);
        c = __shfl(c, 0, 64);
        if (c >= S.n_chunks) {
          if (lane == 0) ctl->overflow = 1;
          S.ok = false;
          return;
        }
        if (lane == 0) {
          S.next[c] = NONE;
          if (S.cur != NONE) S.next[S.cur] = c;
        }
        if (S.first == NONE) S.first = c;
        S.cur = c;
        uint4* dst = reinterpret_cast<uint4*>(S.arena + (size_t)c * CHUNK);
        const uint32_t words = (n * (uint32_t)sizeof(kg_tree_node) + 15) / 16;
        for (uint32_t i = lane; i < words; i += 64) dst[i] = s_out[i];
      };
      // lanes with pred append one record each, in lane order
      auto emit_l = [&](bool pred, const kg_tree_node& rr) {
        const uint64_t m = __ballot(pred);
        if (!m || !S.ok) return;
        const uint32_t k = __popcll(m), rank = lanes_below(m), room = CHUNK - nbuf;
        if (pred && rank < room) sbuf[nbuf + rank] = rr;
        if (k < room) {
          nbuf += k;
          return;
        }
        __builtin_amdgcn_wave_barrier();
        flush(CHUNK);
        __builtin_amdgcn_wave_barrier();
        if (pred && rank >= room) sbuf[rank - room] = rr;
        nbuf = k - room;
      };
      if (status == EXP_OK) {
        if (lane == 0) vis[0] = 1u;
        emit_l(lane == 0, rec_set(s, 1, rn, (uint32_t)len0));
        cnt = 1;
        int sp = 0;
        uint32_t st_chunks = 0, st_u[4] = {0, 0, 0, 0}, st_pops = 0;
        ExpFrame F{0, 0, 0, (uint32_t)len0, d0};
        // a pushed child's first chunk, loaded as soon as the child is chosen (before its union record and
        // the parent's leaves are emitted and the frame is pushed), so that work hides part of the load
        GwEnt pre{};
        bool have_pre = false;
        for (;;) {
          const uint64_t eb = F.rb, ee = F.rb + F.len;
          const bool can_expand = F.d - 1 >= 2;
          bool pushed = false;
          while (eb + F.cursor < ee) {
            const uint64_t at0 = eb + F.cursor;
            // (caching each frame level's chunk in LDS, as expand_root_x does, measured slower here: the
            // walk is bound by its own instruction chain, ~1 us per chunk, not by the copy's latency)
            const uint32_t width = (uint32_t)min<uint64_t>(64, ee - at0);
            const bool valid = (uint32_t)lane < width;
            const GwEnt x = have_pre ? pre : E[valid ? at0 + lane : at0];
            have_pre = false;
            st_chunks++;
            const bool is_set = valid && (x.sub & SET_BIT);
            const bool has_loc = is_set && x.loc != NONE;
            kg_tree_node r;
            r.type = 2;
            r.is_set = is_set ? 1 : 0;
            r.pad = 0;
            r.ns = x.ns;
            r.obj = x.obj;
            r.rel = x.rel;
            r.n_children = 0;
            bool leave = false;
            // lanes [lo, width) of the chunk are still to be emitted; a candidate whose children all sit
            // at rest depth 1 is expanded inline, and the chunk continues from registers
            for (uint32_t lo = 0;;) {
              bool cand = false;
              if (has_loc && can_expand && (uint32_t)lane >= lo) cand = !((vis[x.loc >> 5] >> (x.loc & 31)) & 1u);
              const uint64_t mc = __ballot(cand);
              const uint32_t p = mc ? (uint32_t)(__ffsll((unsigned long long)mc) - 1) : 64u;
              const bool leaf = valid && (uint32_t)lane >= lo && (uint32_t)lane < p;
              // rest depth <= 1 below: child sets become leaves but are still marked (BuildTree marks
              // before it looks at the depth); sets without rows need no mark
              if (!can_expand && leaf && has_loc) atomicOr(&vis[x.loc >> 5], 1u << (x.loc & 31));
              emit_l(leaf, r);
              cnt += __popcll(__ballot(leaf));
              if (!S.ok) {
                status = EXP_ARENA;
                leave = true;
                break;
              }
              if (p == 64u) {
                F.cursor = (uint32_t)(at0 - eb) + width;
                break;
              }
              // p is wave-uniform (a ballot's first lane): v_readlane, no LDS round trip per field
              auto rl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)p); };
              const uint32_t cloc = rl(x.loc), ccb = rl(x.cb), clen = rl(x.len);
              // the child's first chunk (the pushed frame's first load; inline children read it below)
              if (ccb != NONE) {
                const uint32_t cw0 = min(64u, clen);
                pre = E[(uint32_t)lane < cw0 ? (uint64_t)ccb + lane : (uint64_t)ccb];
              }
              kg_tree_node u;
              u.type = 1;
              u.is_set = 1;
              u.pad = 0;
              u.ns = rl(x.ns);
              u.obj = rl(x.obj);
              u.rel = rl(x.rel);
              u.n_children = clen;
              if (ccb == NONE || sp >= 0x7FFF) {  // cannot happen (see the header); left to the next pass
                status = EXP_OVERFLOW;
                leave = true;
                break;
              }
              if (lane == 0) vis[cloc >> 5] |= 1u << (cloc & 31);
              st_u[min(3, max(0, F.d - 1 - 2))]++;
              emit_l(lane == 0, u);
              cnt++;
              if (!S.ok) {
                status = EXP_ARENA;
                leave = true;
                break;
              }
              if (F.d - 1 == 2) {
                // the child's children are at rest depth 1: all leaves, the sets among them marked
                for (uint64_t c0 = ccb; c0 < (uint64_t)ccb + clen; c0 += 64) {
                  const uint32_t cw = (uint32_t)min<uint64_t>(64, (uint64_t)ccb + clen - c0);
                  const bool cv = (uint32_t)lane < cw;
                  const GwEnt y = c0 == ccb ? pre : E[cv ? c0 + lane : c0];
                  st_chunks++;
                  const bool yset = cv && (y.sub & SET_BIT);
                  if (yset && y.loc != NONE) atomicOr(&vis[y.loc >> 5], 1u << (y.loc & 31));
                  kg_tree_node ry;
                  ry.type = 2;
                  ry.is_set = yset ? 1 : 0;
                  ry.pad = 0;
                  ry.ns = y.ns;
                  ry.obj = y.obj;
                  ry.rel = y.rel;
                  ry.n_children = 0;
                  emit_l(cv, ry);
                  cnt += cw;
                  if (!S.ok) break;
                }
                if (!S.ok) {
                  status = EXP_ARENA;
                  leave = true;
                  break;
                }
                lo = p + 1;
                if (lo >= width) {
                  F.cursor = (uint32_t)(at0 - eb) + width;
                  break;
                }
                continue;
              }
              // a deeper child: push (the parent's chunk is reloaded from the copy on the pop)
              F.cursor = (uint32_t)(at0 - eb) + p + 1;
              if (lane == 0) {
                if (sp < XF) s_fr[sp] = F;
                else gstack[sp] = F;
              }
              sp++;
              __builtin_amdgcn_wave_barrier();
              F = ExpFrame{ccb, cloc, 0, clen, F.d - 1};
              have_pre = true;
              pushed = true;
              leave = true;
              break;
            }
            if (leave) break;
          }
          if (status != EXP_OK) break;
          if (pushed) continue;
          if (sp == 0) break;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          sp--;
          st_pops++;
          have_pre = false;  // (a pushed child always has rows, so its prefetched chunk was used)
          F = sp < XF ? s_fr[sp] : gstack[sp];
        }
        if (status == EXP_OK && S.ok && nbuf) {
          __builtin_amdgcn_wave_barrier();
          flush(nbuf);
        }
        if (status == EXP_OK && !S.ok) status = EXP_ARENA;
        if (lane == 0) {
          atomicAdd(&ctl->gw_stat[0], (unsigned long long)st_chunks);
          for (int q = 0; q < 4; q++) atomicAdd(&ctl->gw_stat[1 + q], (unsigned long long)st_u[q]);
          atomicAdd(&ctl->gw_stat[5], (unsigned long long)st_pops);
          atomicAdd(&ctl->gw_stat[6], (unsigned long long)s_nent);
        }
      }
      if (lane == 0) {
        atomicMax(&ctl->gw_ticks[big ? 3 : 1], wall_clock64() - t1);
        if (status == EXP_OVERFLOW) {
          gw_publish(ovf_list, ovf_count, ri, big, gb_list, &ctl->gb_count);
        } else {
          outs[ri] = RootOut{S.first, cnt};
          recs += cnt;
        }
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (recs) atomicAdd(&ctl->records, recs);
    if (!big) {  // this workgroup's ga publications happen-before its count (the large slots' exit test)
      __threadfence();
      atomicAdd(&ctl->gw_small_done, 1u);
    }
  }
}

// After k_expand_gw: ga entries no large slot ever held a ticket for (every large slot gave up waiting
// before they were published) go to the hash pass.  Entries below the last ticket were taken, or
// abandoned and redirected by their publisher (gw_publish); stream order makes the kernel race-free.
__global__ void k_gw_sweep(ExpCtl* ctl, const uint32_t* ga_list, uint32_t* gb_list) {
  const uint32_t cnt = ctl->ga_count, head = ctl->ga_head;
  for (uint32_t i = min(head, cnt) + threadIdx.x; i < cnt; i += blockDim.x) {
    const uint32_t v = ga_list[i];
    if (v && v != GW_ABANDON) gb_list[atomicAdd(&ctl->gb_count, 1u)] = v - 1;
  }
}

__global__ void k_expand_compact(const RootOut* outs, uint32_t n, const uint64_t* off, const kg_tree_node* arena,
                                 const uint32_t* next, kg_tree_node* dst) {
  const uint32_t r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  uint32_t c = outs[r].first_chunk, left = outs[r].count;
  uint64_t o = off[r];
  while (left > 0 && c != NONE) {
    const uint32_t take = left < CHUNK ? left : CHUNK;
    for (uint32_t i = lane; i < take; i += 64) dst[o + i] = arena[(size_t)c * CHUNK + i];
    o += take;
    left -= take;
    c = next[c];
  }
}

// Device-resident trees (kg_expand_batch_device): every root's record count as a u64 (a stack overflow
// counts 0 and is tallied in cnt[n + 1]); cnt[n] = 0, so the exclusive sum over n + 1 entries ends in the
// total.  One thread per root, coalesced.
__global__ void k_root_counts(const RootOut* outs, uint32_t n, unsigned long long* cnt) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  if (r == n) {
    cnt[n] = 0;
    return;
  }
  const uint32_t c = outs[r].count;
  if (c == 0xFFFFFFFFu) atomicAdd(&cnt[n + 1], 1ull);
  cnt[r] = c == 0xFFFFFFFFu ? 0ull : c;
}

// Device buffers of one lane's expand calls (kg_expand_batch: one lane per calling thread and
// replica), grown on demand and kept: hipMalloc / hipFree per call stall the device and would
// serialise concurrent callers.
struct ExpandBufs {
  int device = -1;
  kg_set* d_roots = nullptr;
  RootOut* outs = nullptr;
  uint32_t* p2 = nullptr;  // pass-2 | pass-3 queues
  size_t n_cap = 0;        // roots the three above hold
  ExpCtl* ctl = nullptr;
  ExpFrame* stacks = nullptr;
  size_t stacks_bytes = 0;
  uint32_t* bm = nullptr;  // [pass-2 tables | pass-3 bitmap] | pass-2 lists | pass-3 list
  size_t bm_bytes = 0;
  // the pass-2 tables and the pass-3 bitmap need clearing: fresh memory, or a call that ended early (an
  // arena rerun or an error can leave keys behind; a completed call leaves them clear -- every root's
  // walk removes its keys, an overflowing one zeroes its table)
  bool bm_dirty = true;
  kg_tree_node* arena = nullptr;
  uint32_t* next = nullptr;
  uint32_t chunks = 0;
  kg_tree_node* dst = nullptr;
  size_t dst_cap = 0;
  uint64_t* d_off = nullptr;
  size_t off_cap = 0;
  unsigned long long* cnt = nullptr;  // device-resident trees: per-root counts (+ total, + overflow tally)
  size_t cnt_cap = 0;
  void* scan_tmp = nullptr;  // hipcub scan temporary
  size_t scan_cap = 0;
  void* gw[2] = {nullptr, nullptr};  // gather-walk slots: small, large (allocated once, epochs zeroed)
  GwSlots gws[2] = {};
  uint32_t gw_slots[2] = {0, 0};
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t sync_ev = nullptr;  // blocking-sync: a caller waits asleep (16 batches in flight, 16 CPUs)
  // Waits for everything enqueued on st so far without spinning a core.
  hipError_t wait(hipStream_t st) {
    hipError_t e = hipSuccess;
    if (!sync_ev && (e = hipEventCreateWithFlags(&sync_ev, hipEventBlockingSync | hipEventDisableTiming)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(sync_ev, st)) != hipSuccess) return e;
    return hipEventSynchronize(sync_ev);
  }
  ~ExpandBufs() {
    if (device >= 0) hipSetDevice(device);
    for (void* p : {(void*)d_roots, (void*)outs, (void*)p2, (void*)ctl, (void*)stacks, (void*)bm, (void*)arena,
                    (void*)next, (void*)dst, (void*)d_off, (void*)cnt, scan_tmp, gw[0], gw[1]})
      if (p) hipFree(p);
    for (auto& e : ev)
      if (e) hipEventDestroy(e);
    if (sync_ev) hipEventDestroy(sync_ev);
  }
};

void expand_bufs_free(void* p) { delete static_cast<ExpandBufs*>(p); }

// Tree outputs go to pinned host memory from a process-wide pool: a device->host copy of a C5
// batch's ~130 MB of records into fresh pageable memory took ~50 ms (page faults + staging), more
// than the batch's kernels once batches overlap.  Buffers are size-classed (powers of two from
// 1 MiB) and returned by kg_tree_free; at most POOL_KEEP bytes stay cached.
namespace {
constexpr size_t POOL_KEEP = 4ull << 30;
std::mutex pool_mu;
std::vector<std::pair<size_t, void*>> pool_free;
size_t pool_cached = 0;
size_t pool_class(size_t bytes) {
  size_t c = 1 << 20;
  while (c < bytes) c <<= 1;
  return c;
}
}  // namespace

void* tree_pool_get(size_t bytes) {
  const size_t c = pool_class(bytes);
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    for (size_t i = 0; i < pool_free.size(); i++)
      if (pool_free[i].first == c) {
        void* p = pool_free[i].second;
        pool_free[i] = pool_free.back();
        pool_free.pop_back();
        pool_cached -= c;
        return p;
      }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void tree_pool_put(void* p, size_t bytes) {
  if (!p) return;
  const size_t c = pool_class(bytes);
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    if (pool_cached + c <= POOL_KEEP) {
      pool_free.emplace_back(c, p);
      pool_cached += c;
      return;
    }
  }
  (void)hipHostFree(p);
}

// Device-resident tree outputs (kg_expand_batch_device) come from a per-device pool of the same size
// classes, returned by kg_tree_free: hipMalloc / hipFree per call stall the device.  At most
// DEV_POOL_KEEP bytes per device stay cached (C5: ~90 MB of records per call, 16 calls in flight).
namespace {
constexpr size_t DEV_POOL_KEEP = 16ull << 30;
struct DevFree {
  int device;
  size_t cls;
  void* p;
};
std::vector<DevFree> dev_free;
size_t dev_cached[64] = {};
}  // namespace

void* tree_dev_get(int device, size_t bytes) {
  const size_t c = pool_class(bytes);
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    for (size_t i = 0; i < dev_free.size(); i++)
      if (dev_free[i].device == device && dev_free[i].cls == c) {
        void* p = dev_free[i].p;
        dev_free[i] = dev_free.back();
        dev_free.pop_back();
        dev_cached[device & 63] -= c;
        return p;
      }
  }
  void* p = nullptr;
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&p, c) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void tree_dev_put(int device, void* p, size_t bytes) {
  if (!p) return;
  const size_t c = pool_class(bytes);
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    if (dev_cached[device & 63] + c <= DEV_POOL_KEEP) {
      dev_free.push_back(DevFree{device, c, p});
      dev_cached[device & 63] += c;
      return;
    }
  }
  (void)hipSetDevice(device);
  (void)hipFree(p);
}

// Replaces *p with a buffer of at least `need` bytes (contents not kept).
template <class T>
static hipError_t grow(T** p, size_t& have, size_t need) {
  if (need <= have && *p) return hipSuccess;
  if (*p) hipFree(*p);
  *p = nullptr;
  have = 0;
  const hipError_t e = hipMalloc((void**)p, std::max<size_t>(need, 16));
  if (e == hipSuccess) have = need;
  return e;
}

// Gather-walk slot classes: (slots, entries, map slots, local ids).  Small:
// the bulk of the pass-1 overflows (~1 k C5 roots of 0.5-10 k records); large: the few giant trees.
constexpr uint32_t GW_LOC[2] = {16384, GW_LDS_LOC};
static hipError_t gw_alloc(ExpandBufs& B, int k, uint32_t slots, uint32_t ent_cap, hipStream_t stream) {
  if (B.gw[k]) return hipSuccess;
  const uint32_t map_cap = 2 * GW_LOC[k];
  const size_t tf = ent_cap / 64 + 1;
  const size_t per = (size_t)ent_cap * (sizeof(GwEnt) + 8 + 4) + tf * 4 + (size_t)map_cap * 16;
  char* p = nullptr;
  hipError_t e = hipMalloc((void**)&p, per * slots + (size_t)slots * 4 + 256);
  if (e != hipSuccess) return e;
  GwSlots g{};
  g.ent_cap = ent_cap;
  g.map_cap = map_cap;
  g.loc_cap = GW_LOC[k];
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = p + off;
    off += (bytes + 255) & ~size_t(255);
    return q;
  };
  g.map = (unsigned long long*)take((size_t)slots * map_cap * 16);
  g.hmark = (uint32_t*)take((size_t)slots * ent_cap * 4);
  g.epoch = (uint32_t*)take((size_t)slots * 4);
  const size_t zero = off;  // keys, run marks and epochs start at 0 (epoch 0 is never used)
  g.ent = (GwEnt*)take((size_t)slots * ent_cap * sizeof(GwEnt));
  g.hsrc = (uint64_t*)take((size_t)slots * ent_cap * 8);
  g.tfirst = (uint32_t*)take((size_t)slots * tf * 4);
  if ((e = hipMemsetAsync(p, 0, zero, stream)) != hipSuccess) {
    hipFree(p);
    return e;
  }
  B.gw[k] = p;
  B.gws[k] = g;
  B.gw_slots[k] = slots;
  return hipSuccess;
}

int expand_batch(Snapshot* s, hipStream_t stream, void** bufs, const kg_set* roots, size_t n, int32_t global,
                 kg_tree_buf* out, bool dev_io) {
  memset(out, 0, sizeof *out);
  if (global < 1) global = 5;
  HIPC(hipSetDevice(s->device));
  out->n_roots = n;
  if (dev_io) {
    // device-resident trees: root_off (n + 1 entries) and the records in the device pool
    out->pinned = KG_TREE_DEVICE | (uint64_t)(s->device & 0xFF);
    out->root_off = (uint64_t*)tree_dev_get(s->device, (n + 1) * 8);
    if (!out->root_off) return set_error(-4, "device allocation failed");
    if (n == 0) {
      HIPC(hipMemsetAsync(out->root_off, 0, 8, stream));
      HIPC(hipStreamSynchronize(stream));
      return 0;
    }
  } else {
    out->root_off = (uint64_t*)calloc(n + 1, 8);
    if (!out->root_off) return set_error(-4, "host allocation failed");
    if (n == 0) return 0;
  }
  if (!*bufs) *bufs = new ExpandBufs();
  ExpandBufs& B = *static_cast<ExpandBufs*>(*bufs);
  B.device = s->device;
  const uint32_t stack_cap = (uint32_t)std::min<int64_t>(0x8000, (int64_t)global + 2);
  bool gw_on = s->expand_gw != 0;
  const uint32_t gw_n[2] = {std::max<uint32_t>(1, (uint32_t)s->n_cu / 2), 4};
  const uint32_t grid1 = (uint32_t)s->n_cu * 2, slots1 = grid1 * 4;
  // pass 0 (16-lane walkers, 16 per workgroup) unless expand_skip_lds says otherwise (1: no LDS pass
  // at all, 2: the 64-lane pass takes every root)
  const bool sub_on = s->expand_skip_lds == 0;
  const uint32_t grid0 = (uint32_t)s->n_cu * 2, slots0 = sub_on ? grid0 * (256 / SW) : 0u;
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1), words = ((nn + 31) / 32 + 1 + 3) & ~3ull;
  // pass 2: 2 slots per CU, each a visited hash + list of up to 256 Ki nodes (~5 MB a slot, <= 2 GiB;
  // 4 per CU measured the same on C5)
  const uint64_t cap2 = (std::min<uint64_t>(nn, 1ull << 18) + 3) & ~3ull;
  uint64_t tsize = 64;
  while (tsize < 2 * cap2 + 128) tsize <<= 1;
  const uint32_t slots2 =
      (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)s->n_cu * 2, (2ull << 30) / ((tsize + cap2) * 4)));
  uint32_t n_chunks = (uint32_t)std::min<uint64_t>(1u << 22, std::max<uint64_t>(4096, n * 2 + slots1 + slots0));
  n_chunks = std::max(n_chunks, B.chunks);  // an arena that grew for earlier calls stays grown
  const size_t clear_words = (size_t)slots2 * tsize + words;
  int rc = 0;
  auto fail = [&](const char* what, hipError_t e) { rc = set_error(-1, "%s: %s", what, hipGetErrorString(e)); };
  hipError_t e = hipSuccess;
  if (n > B.n_cap) {
    size_t a = 0, b = 0, c = 0;
    const size_t cap = std::max(n, 2 * B.n_cap);
    B.n_cap = 0;
    if ((e = grow(&B.d_roots, a, cap * sizeof(kg_set))) != hipSuccess || (e = grow(&B.outs, b, cap * sizeof(RootOut))) != hipSuccess ||
        (e = grow(&B.p2, c, cap * 20)) != hipSuccess)  // p2 | p3 | ga | gb | p0 queues
      fail("hipMalloc", e);
    else
      B.n_cap = cap;
  }
  if (!rc && !B.ctl && (e = hipMalloc(&B.ctl, sizeof(ExpCtl))) != hipSuccess) fail("hipMalloc", e);
  if (!rc && (e = grow(&B.stacks, B.stacks_bytes,
                       (size_t)(slots1 + slots2 + 1 + gw_n[0] + gw_n[1] + slots0) * stack_cap * sizeof(ExpFrame))) != hipSuccess)
    fail("hipMalloc", e);
  // gather-walk slots (~0.9 GB a lane); without them the pass-1 overflows go to the hash pass directly
  for (int k = 0; k < 2 && gw_on && !rc; k++)
    if (gw_alloc(B, k, gw_n[k], k == 0 ? 65536u : (2u << 20), stream) != hipSuccess) {
      (void)hipGetLastError();
      gw_on = false;
    }
  {
    const uint32_t* bm0 = B.bm;
    if (!rc && (e = grow(&B.bm, B.bm_bytes, (clear_words + (size_t)slots2 * cap2 + nn) * 4)) != hipSuccess)
      fail("hipMalloc", e);
    if (B.bm != bm0) B.bm_dirty = true;
  }
  for (auto& x : B.ev)
    if (!rc && !x && (e = hipEventCreate(&x)) != hipSuccess) fail("hipEventCreate", e);
  uint32_t* lists = B.bm + clear_words;
  // the roots: the caller's device array (dev_io) or staged from host memory
  const kg_set* d_roots = dev_io ? roots : B.d_roots;
  if (!dev_io && !rc && (e = hipMemcpyAsync(B.d_roots, roots, n * sizeof(kg_set), hipMemcpyHostToDevice, stream)) != hipSuccess)
    fail("H2D", e);
  ExpCtl h{};
  for (int attempt = 0; !rc; attempt++) {
    if (n_chunks > B.chunks) {
      size_t a = 0, b = 0;
      B.chunks = 0;
      if ((e = grow(&B.arena, a, (size_t)n_chunks * CHUNK * sizeof(kg_tree_node))) != hipSuccess ||
          (e = grow(&B.next, b, (size_t)n_chunks * 4)) != hipSuccess) {
        fail("hipMalloc(arena)", e);
        break;
      }
      B.chunks = n_chunks;
    }
    // every attempt starts from clear visited tables (an arena overflow aborts roots mid-way); a lane whose
    // last call completed has them clear already (C5: ~1.6 GB of memset per call before round 6)
    if (((B.bm_dirty || attempt > 0) && (e = hipMemsetAsync(B.bm, 0, clear_words * 4, stream)) != hipSuccess) ||
        (e = hipMemsetAsync(B.ctl, 0, sizeof(ExpCtl), stream)) != hipSuccess ||
        (gw_on && (e = hipMemsetAsync(B.p2 + 2 * n, 0, n * 4, stream)) != hipSuccess)) {  // ga: published as ri + 1
      fail("memset", e);
      break;
    }
    (void)hipEventRecord(B.ev[0], stream);
    if (sub_on)
      hipLaunchKernelGGL(k_expand_sub, dim3(grid0), dim3(256), 0, stream, s->ds, d_roots, (uint32_t)n, global, B.ctl,
                         B.outs, B.arena, B.next, n_chunks,
                         B.stacks + (size_t)(slots1 + slots2 + 1 + gw_n[0] + gw_n[1]) * stack_cap, stack_cap, B.p2 + 4 * n);
    hipLaunchKernelGGL(k_expand_lds, dim3(grid1), dim3(256), 0, stream, s->ds, d_roots, (uint32_t)n, global, B.ctl,
                       B.outs, B.arena, B.next, n_chunks, B.stacks, stack_cap, B.p2, s->expand_skip_lds == 1 ? 1 : 0,
                       sub_on ? (const uint32_t*)(B.p2 + 4 * n) : nullptr);
    // pass-1 overflows: gather-walk small slots -> large slots -> the hash pass (or straight to it)
    uint32_t* q_hash = B.p2;
    uint32_t* c_hash = &B.ctl->p2_count;
    uint32_t* h_hash = &B.ctl->p2_head;
    if (gw_on) {
      ExpFrame* gst = B.stacks + (size_t)(slots1 + slots2 + 1) * stack_cap;
      hipLaunchKernelGGL(k_expand_gw, dim3(gw_n[0] + gw_n[1]), dim3(256), 0, stream, s->ds, d_roots, global, B.ctl,
                         B.outs, B.arena, B.next, n_chunks, gst, stack_cap, B.p2, B.p2 + 2 * n, B.p2 + 3 * n,
                         (uint32_t)n, gw_n[1], B.gws[0], B.gws[1], (uint64_t)s->expand_gw_wait_us * 100);  // 100 MHz clock
      hipLaunchKernelGGL(k_gw_sweep, dim3(1), dim3(256), 0, stream, B.ctl, B.p2 + 2 * n, B.p2 + 3 * n);
      q_hash = B.p2 + 3 * n;
      c_hash = &B.ctl->gb_count;
      h_hash = &B.ctl->gb_head;
    }
    hipLaunchKernelGGL(k_expand_hash, dim3(slots2), dim3(64), 0, stream, s->ds, d_roots, global, B.ctl, B.outs,
                       B.arena, B.next, n_chunks, B.stacks + (size_t)slots1 * stack_cap, stack_cap, q_hash, c_hash,
                       h_hash, B.bm, tsize, lists, cap2, B.p2 + n);
    hipLaunchKernelGGL(k_expand_hbm, dim3(1), dim3(64), 0, stream, s->ds, d_roots, global, B.ctl, B.outs, B.arena,
                       B.next, n_chunks, B.stacks + (size_t)(slots1 + slots2) * stack_cap, B.p2 + n,
                       B.bm + (size_t)slots2 * tsize, words, lists + (size_t)slots2 * cap2, nn);
    (void)hipEventRecord(B.ev[1], stream);
    if ((e = hipGetLastError()) != hipSuccess) {
      fail("launch", e);
      break;
    }
    if ((e = hipMemcpyAsync(&h, B.ctl, sizeof h, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = B.wait(stream)) != hipSuccess) {
      fail("expand", e);
      break;
    }
    if (!h.overflow) {
      if (getenv("KG_EXPAND_TRACE"))  // diagnostics: the longest gather / walk of one root per slot class
        fprintf(stderr, "kg expand: gw small gather %.1f us walk %.1f us (queue %u) | large gather %.1f us walk %.1f us (queue %u) | hash queue %u\n",
                h.gw_ticks[0] / 100.0, h.gw_ticks[1] / 100.0, h.p2_count, h.gw_ticks[2] / 100.0, h.gw_ticks[3] / 100.0,
                h.ga_count, h.gb_count);
      if (getenv("KG_EXPAND_TRACE"))
        fprintf(stderr, "kg expand: gw walk chunks %llu unions d2 %llu d3 %llu d4 %llu d5+ %llu pops %llu entries %llu records %llu\n",
                h.gw_stat[0], h.gw_stat[1], h.gw_stat[2], h.gw_stat[3], h.gw_stat[4], h.gw_stat[5], h.gw_stat[6], h.records);
      break;
    }
    if (n_chunks >= (1u << 30) || attempt > 8) {
      rc = set_error(KG_ERR_RESOURCE, "expand output exceeds the arena");
      break;
    }
    n_chunks *= 4;  // grow the arena and rerun (outputs are rewritten from scratch)
  }
  B.bm_dirty = rc != 0 || h.overflow != 0;  // only a completed call leaves the tables clear
  if (dev_io) {
    // offsets by a device scan of the roots' counts; the total and the overflow tally come back in one
    // readback, then the records are compacted into the output (no host pass over the roots)
    uint64_t tail[2] = {0, 0};
    size_t tmp_need = 0;
    if (!rc && (e = grow(&B.cnt, B.cnt_cap, (n + 2) * 8)) != hipSuccess) fail("hipMalloc", e);
    if (!rc && (e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_need, B.cnt, (unsigned long long*)out->root_off,
                                                     (int)(n + 1), stream)) != hipSuccess)
      fail("scan", e);
    if (!rc && (e = grow((char**)&B.scan_tmp, B.scan_cap, tmp_need)) != hipSuccess) fail("hipMalloc", e);
    if (!rc && (e = hipMemsetAsync(B.cnt + n + 1, 0, 8, stream)) != hipSuccess) fail("memset", e);
    if (!rc) {
      hipLaunchKernelGGL(k_root_counts, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, stream, B.outs, (uint32_t)n,
                         B.cnt);
      if ((e = hipcub::DeviceScan::ExclusiveSum(B.scan_tmp, tmp_need, B.cnt, (unsigned long long*)out->root_off,
                                                (int)(n + 1), stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&tail[0], out->root_off + n, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&tail[1], B.cnt + n + 1, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = B.wait(stream)) != hipSuccess)
        fail("root offsets", e);
    }
    if (!rc && tail[1]) rc = set_error(KG_ERR_RESOURCE, "%llu expand root(s) exceeded the stack", (unsigned long long)tail[1]);
    const uint64_t total = rc ? 0 : tail[0];
    if (!rc && total) {
      out->nodes = (kg_tree_node*)tree_dev_get(s->device, total * sizeof(kg_tree_node));
      if (!out->nodes) rc = set_error(-4, "device allocation failed");
    }
    if (!rc && total) {
      (void)hipEventRecord(B.ev[2], stream);
      hipLaunchKernelGGL(k_expand_compact, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, stream, B.outs, (uint32_t)n,
                         out->root_off, B.arena, B.next, out->nodes);
      (void)hipEventRecord(B.ev[3], stream);
      if ((e = hipGetLastError()) != hipSuccess || (e = B.wait(stream)) != hipSuccess) fail("compact", e);
    }
    out->n_nodes = total;
    if (!rc) {
      float a = 0, b = 0;
      (void)hipEventElapsedTime(&a, B.ev[0], B.ev[1]);
      if (total) (void)hipEventElapsedTime(&b, B.ev[2], B.ev[3]);
      out->kernel_ms = (double)a + (double)b;
    } else {
      B.bm_dirty = true;
      tree_dev_put(s->device, out->nodes, total * sizeof(kg_tree_node));
      tree_dev_put(s->device, out->root_off, (n + 1) * 8);
      memset(out, 0, sizeof *out);
    }
    return rc;
  }
  std::vector<RootOut> ho(n);
  if (!rc && (e = hipMemcpyAsync(ho.data(), B.outs, n * sizeof(RootOut), hipMemcpyDeviceToHost, stream)) != hipSuccess)
    fail("D2H", e);
  if (!rc && (e = B.wait(stream)) != hipSuccess) fail("D2H", e);
  if (!rc) {
    for (size_t r = 0; r < n; r++) {
      if (ho[r].count == 0xFFFFFFFFu) {
        rc = set_error(KG_ERR_RESOURCE, "expand root %zu exceeded the stack", r);
        break;
      }
      out->root_off[r + 1] = out->root_off[r] + ho[r].count;
    }
  }
  const uint64_t total = rc ? 0 : out->root_off[n];
  if (!rc && total) {
    out->nodes = (kg_tree_node*)tree_pool_get(total * sizeof(kg_tree_node));
    out->pinned = 1;
    if (!out->nodes) rc = set_error(-4, "pinned host allocation failed");
    // grown only when this call's records do not fit, then to twice the old size at least (a request
    // of "twice the capacity" on every call doubled the buffer per call: a long-lived lane ran the
    // device out of memory)
    const size_t dst_need = total * sizeof(kg_tree_node);
    if (!rc && dst_need > B.dst_cap &&
        (e = grow(&B.dst, B.dst_cap, std::max<size_t>(dst_need, 2 * B.dst_cap))) != hipSuccess)
      fail("hipMalloc", e);
    if (!rc && (e = grow(&B.d_off, B.off_cap, (n + 1) * 8)) != hipSuccess) fail("hipMalloc", e);
    if (!rc && (e = hipMemcpyAsync(B.d_off, out->root_off, (n + 1) * 8, hipMemcpyHostToDevice, stream)) != hipSuccess)
      fail("H2D", e);
    if (!rc) {
      (void)hipEventRecord(B.ev[2], stream);
      hipLaunchKernelGGL(k_expand_compact, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, stream, B.outs, (uint32_t)n,
                         B.d_off, B.arena, B.next, B.dst);
      (void)hipEventRecord(B.ev[3], stream);
      if ((e = hipMemcpyAsync(out->nodes, B.dst, total * sizeof(kg_tree_node), hipMemcpyDeviceToHost, stream)) !=
              hipSuccess ||
          (e = B.wait(stream)) != hipSuccess)
        fail("compact", e);
    }
  }
  out->n_nodes = total;
  if (!rc) {
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, B.ev[0], B.ev[1]);
    if (total) (void)hipEventElapsedTime(&b, B.ev[2], B.ev[3]);
    out->kernel_ms = (double)a + (double)b;
  }
  if (rc) {
    B.bm_dirty = true;
    if (out->pinned) tree_pool_put(out->nodes, total * sizeof(kg_tree_node));
    free(out->root_off);
    memset(out, 0, sizeof *out);
  }
  return rc;
}

}  // namespace kg
