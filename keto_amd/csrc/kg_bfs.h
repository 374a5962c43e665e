// kg_bfs.h -- wave64 building blocks shared by the check kernels (device only).
//
// wave_bfs_run(): level-synchronous, depth-bounded BFS of ONE wave over the set-adjacency CSR,
// starting from a deduplicated root set at rest depth d0.  It answers, for rewrite-free nodes,
// the reference's checkIsAllowed recursion (internal/check/engine.go:183-207):
//   level k node at rest depth d = d0-k:  checkDirect(d-1)   -> probe the exact tuple if d >= 1
//                                          checkExpandSubject -> children at d-1, if d >= 2
// with the group rule "first IsMember wins" (checkgroup/concurrent_checkgroup.go:104-115) as the
// early exit.  Marking every node at its shallowest level gives the schedule-free answer
// (SURVEY.md 8a); storage is either the wave's LDS (fast tier, bounded) or a per-slot HBM
// bitmap + list (unbounded tier).
#pragma once
#include <hip/hip_runtime.h>

#include "kg_internal.h"

namespace kg {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Loads of random lines a batch touches about once (node-map slots, dset buckets, holder-bitmap
// words, the query records): plain loads.  (A non-temporal variant, built as a separate library with
// KG_NT_RANDOM, measured 6 % slower in round 5 -- profiles/r5nt_nontemporal_random_ab.jsonl -- and was
// removed in round 6.)
template <class T>
__device__ __forceinline__ T ld_once(const T* p) {
  return *p;
}

// Node-map lookup: the slot of (ns, rel, obj), or nullptr.  The first slot is passed in when the
// caller already issued its load (k_resolve overlaps it with other lookups).
__device__ __forceinline__ const NSlot* nmap_slot(const DevSnap& s, uint64_t key, uint64_t i) {
  for (uint64_t p = 0; p < s.nmap_n; p++) {  // load <= 0.625: ends at an empty slot long before
    const uint64_t k = s.nmap[i].key;
    if (k == key) return &s.nmap[i];
    if (k == EMPTY64) return nullptr;
    i = hash_next(i, s.nmap_n);
  }
  return nullptr;
}

__device__ __forceinline__ bool nmap_key_ok(uint32_t ns, uint32_t rel, uint32_t obj) {
  return ns < 0xFFFFu && rel < 0xFFFFu && obj < 0x7FFFFFFFu;
}

__device__ __forceinline__ uint32_t nmap_find(const DevSnap& s, uint32_t ns, uint32_t rel, uint32_t obj) {
  if (!nmap_key_ok(ns, rel, obj)) return NONE;
  const uint64_t key = nmap_key(ns, rel, obj);
  const NSlot* sl = nmap_slot(s, key, hash_home(key, s.nmap_n));
  return sl ? sl->node : NONE;
}

// checkDirect: does the exact tuple (node, subject) exist?  One 16-B bucket (two keys) per probe;
// at load <= 0.25 the first bucket nearly always decides.
__device__ __forceinline__ bool dset_probe(const DevSnap& s, uint32_t node, uint32_t subj) {
  static_assert(DSET_BUCKET == 2, "one ulonglong2 per bucket");
  uint64_t key = dset_key(node, subj);
  uint64_t b = dset_home(key, s.dset_nb);
  for (uint64_t n = 0; n < s.dset_nb; n++) {
    const ulonglong2 a = ld_once(reinterpret_cast<const ulonglong2*>(s.dset + b * DSET_BUCKET));
    if (a.x == key || a.y == key) return true;
    if (a.y == EMPTY64) return false;  // buckets fill front to back
    b = hash_next(b, s.dset_nb);
  }
  return false;
}

// checkDirect at a root whose node-map slot is at hand: its inline check-row subjects when the slot
// carries them (the whole row), else the dset probe.
__device__ __forceinline__ bool nslot_probe(const DevSnap& s, const NSlot* sl, uint32_t node, uint32_t subj) {
  if (sl && nslot_inline(sl->pad1)) return nslot_inline_has(nslot_inline(sl->pad1), sl->pad1, sl->sig, subj);
  return dset_probe(s, node, subj);
}

// Holders of a tagged subject: hold[first, first+count) are the nodes whose row contains it.
// Requires s.radj (reverse indexes built).  Unknown subject -> count 0.
__device__ __forceinline__ uint2 holders_find(const DevSnap& s, uint32_t subj) {
  if (subj == NONE) return make_uint2(0, 0);
  uint64_t h = mix64(subj) & s.hmask;
  for (uint64_t p = 0; p <= s.hmask; p++) {  // load <= 0.5
    const HSlot sl = s.hslots[h];
    if (sl.key == subj) return make_uint2(sl.first, sl.count);
    if (sl.key == NONE) break;
    h = (h + 1) & s.hmask;
  }
  return make_uint2(0, 0);
}

// Wave64 scans on DPP (GFX9 data-parallel primitives): every step is one VALU op on registers,
// no LDS round trip (a __shfl is a ds_bpermute).  row_shr:n = 0x110+n shifts inside rows of 16
// lanes (lanes without a source read 0), row_bcast:15 / row_bcast:31 (0x142 / 0x143) carry row
// totals across rows.  Must be called with every lane of the wave active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, true);
}
struct DppAdd {
  __device__ static uint32_t op(uint32_t a, uint32_t b) { return a + b; }
};
struct DppOr {
  __device__ static uint32_t op(uint32_t a, uint32_t b) { return a | b; }
};
struct DppMax {
  __device__ static uint32_t op(uint32_t a, uint32_t b) { return a > b ? a : b; }
};
// inclusive scan over the 64 lanes for an operator whose identity is 0
template <class Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v = Op::op(v, dpp0<0x111, 0xf>(v));
  v = Op::op(v, dpp0<0x112, 0xf>(v));
  v = Op::op(v, dpp0<0x114, 0xf>(v));
  v = Op::op(v, dpp0<0x118, 0xf>(v));
  v = Op::op(v, dpp0<0x142, 0xa>(v));
  v = Op::op(v, dpp0<0x143, 0xc>(v));
  return v;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t* total) {
  const uint32_t v = wave_incl_scan<DppAdd>(x);
  *total = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  return v - x;
}

__device__ __forceinline__ void wave_append(bool pred, uint32_t val, uint32_t* list, uint32_t* count) {
  uint64_t m = __ballot(pred);
  if (!m) return;
  int lane = lane_id();
  int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  if (pred) list[base + __popcll(m & ((1ull << lane) - 1))] = val;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int off) {
  const uint32_t lo = __shfl_up((uint32_t)v, off, 64), hi = __shfl_up((uint32_t)(v >> 32), off, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) { return __popcll(m & ((1ull << lane_id()) - 1)); }

// largest j in [0, n) with pref[j] <= e (pref non-decreasing, pref[0] = 0)
__device__ __forceinline__ int owner_search(const uint32_t* pref, int n, uint32_t e) {
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (pref[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------------ per-wave BFS storage
constexpr int VIS_LOG2 = 10;  // LDS visited-hash slots per wave
constexpr int VIS = 1 << VIS_LOG2;
constexpr int LIST = 512;  // LDS BFS list per wave (visited cap; hash load <= 0.5)

template <int VL2 = VIS_LOG2, int LST = LIST>
struct WaveLdsT {
  uint32_t vis[1 << VL2];
  uint32_t list[LST];
  uint32_t pref[64];
};
using WaveLds = WaveLdsT<>;

template <int VL2 = VIS_LOG2, int LST = LIST>
struct LdsStoreT {
  static constexpr int NV = 1 << VL2;
  static_assert(LST + 64 < NV, "the list cap keeps the visited hash below full");
  WaveLdsT<VL2, LST>* L;
  __device__ uint32_t* list() const { return L->list; }
  __device__ uint32_t* pref() const { return L->pref; }
  __device__ uint64_t cap() const { return LST; }
  __device__ void reset() {
    const int lane = lane_id();
    for (int i = lane * 4; i < NV; i += 256) *reinterpret_cast<uint4*>(&L->vis[i]) = make_uint4(NONE, NONE, NONE, NONE);
    __builtin_amdgcn_wave_barrier();
  }
  // Bounded probe: callers check the list cap after every 64-wide step, so the table never holds
  // more than LST + 64 < NV keys; the bound only guarantees termination.
  __device__ bool insert(uint32_t key) {
    uint32_t h = (key * 2654435761u) >> (32 - VL2);
    for (int p = 0; p < NV; p++) {
      uint32_t old = atomicCAS(&L->vis[h], NONE, key);
      if (old == NONE) return true;
      if (old == key) return false;
      h = (h + 1) & (NV - 1);
    }
    return true;
  }
  // lookup only (no insert): the key was inserted earlier by this wave
  __device__ bool contains(uint32_t key) const {
    uint32_t h = (key * 2654435761u) >> (32 - VL2);
    for (int p = 0; p < NV; p++) {
      const uint32_t k = L->vis[h];
      if (k == key) return true;
      if (k == NONE) return false;
      h = (h + 1) & (NV - 1);
    }
    return false;
  }
  __device__ void sync() { __builtin_amdgcn_wave_barrier(); }
  __device__ void finish(uint32_t) {}
};
using LdsStore = LdsStoreT<>;

// HBM tier: visited bitmap (n_nodes bits, left all-clear between runs) + BFS list; LDS prefix.
struct GlobalStore {
  uint32_t* bm;
  uint32_t* lst;
  uint64_t capacity;
  uint32_t* pf;
  __device__ uint32_t* list() const { return lst; }
  __device__ uint32_t* pref() const { return pf; }
  __device__ uint64_t cap() const { return capacity; }
  __device__ void reset() {}
  __device__ bool insert(uint32_t key) {
    uint32_t bit = 1u << (key & 31);
    return !(atomicOr(&bm[key >> 5], bit) & bit);
  }
  __device__ bool contains(uint32_t key) const {  // coherent load (the marks are device atomics)
    return (__hip_atomic_load(&bm[key >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (key & 31)) & 1u;
  }
  // contains() that also returns where an absent key goes (expand's known-new insert)
  __device__ bool find(uint32_t key, uint32_t& at) const {
    at = key;
    return contains(key);
  }
  // inserts a key known to be absent (find() said so and nothing was inserted since): no return
  // value is needed, so nothing is waited for
  __device__ void put_new(uint32_t key, uint32_t) { atomicOr(&bm[key >> 5], 1u << (key & 31)); }
  __device__ void sync() {
    // list entries written by other lanes of this wave must be visible to its loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __device__ void finish(uint32_t n) {
    sync();
    for (uint32_t i = lane_id(); i < n; i += 64) atomicAnd(&bm[lst[i] >> 5], 0u);
    sync();
  }
};

// HBM tier with a bounded footprint: open-addressing visited hash (tmask+1 >= 2 x cap slots,
// entries key+1 so the zeroed pool is empty) + BFS list of cap nodes.  The list cap is checked
// after every 64-wide step, so the table stays below half full and a probe always ends.  finish()
// removes the listed keys (a lookup of a key known to be present skips zeroed slots, so the
// removal order does not matter); after an overflow the caller zeroes the whole table.
struct HashStore {
  uint32_t* tab;
  uint32_t tmask;
  uint32_t* lst;
  uint64_t capacity;
  uint32_t* pf;
  __device__ uint32_t* list() const { return lst; }
  __device__ uint32_t* pref() const { return pf; }
  __device__ uint64_t cap() const { return capacity; }
  __device__ void reset() {}
  __device__ uint32_t home(uint32_t key) const { return (key * 2654435761u) & tmask; }
  __device__ bool insert(uint32_t key) {
    uint32_t h = home(key);
    for (uint32_t p = 0; p <= tmask; p++) {
      const uint32_t old = atomicCAS(&tab[h], 0u, key + 1);
      if (old == 0u) return true;
      if (old == key + 1) return false;
      h = (h + 1) & tmask;
    }
    return true;
  }
  __device__ bool contains(uint32_t key) const {  // coherent loads (the entries are device atomics)
    uint32_t h = home(key);
    for (uint32_t p = 0; p <= tmask; p++) {
      const uint32_t k = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == key + 1) return true;
      if (k == 0u) return false;
      h = (h + 1) & tmask;
    }
    return false;
  }
  // contains() that also returns the empty slot an absent key would take
  __device__ bool find(uint32_t key, uint32_t& at) const {
    uint32_t h = home(key);
    at = h;
    for (uint32_t p = 0; p <= tmask; p++) {
      const uint32_t k = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == key + 1) return true;
      if (k == 0u) {
        at = h;
        return false;
      }
      h = (h + 1) & tmask;
    }
    return false;
  }
  // a key known to be absent goes to the slot find() returned: the table belongs to one wave and
  // nothing was inserted since, so a plain (coherent) store takes it -- no CAS round trip
  __device__ void put_new(uint32_t key, uint32_t at) {
    __hip_atomic_store(&tab[at], key + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __device__ void finish(uint32_t n) {
    sync();
    for (uint32_t i = lane_id(); i < n; i += 64) {
      const uint32_t key = lst[i];
      uint32_t h = home(key);
      for (uint32_t p = 0; p <= tmask; p++) {
        if (atomicCAS(&tab[h], key + 1, 0u) == key + 1) break;
        h = (h + 1) & tmask;
      }
    }
    sync();
  }
};

struct BfsStats {
  unsigned long long rows = 0, edges = 0, probes = 0;
};

enum : int { BFS_N = 0, BFS_M = 1, BFS_OVERFLOW = 2 };

// Each lane offers at most one candidate root; deduplicated roots are appended to the list.
// Returns false on overflow (the caller gives up on this store tier).
template <class Store>
__device__ __forceinline__ bool wave_add_roots(Store& st, bool offer, uint32_t node, uint32_t& n_list) {
  const bool fresh = offer && st.insert(node);
  const uint64_t m = __ballot(fresh);
  const uint32_t cnt = __popcll(m);
  if (n_list + cnt > st.cap()) return false;
  if (fresh) st.list()[n_list + lanes_below(m)] = node;
  n_list += cnt;
  return true;
}

template <class Store>
__device__ int wave_bfs_run(const DevSnap& s, Store& st, uint32_t n_roots, int d0, uint32_t subj, BfsStats& bs) {
  const int lane = lane_id();
  uint32_t* list = st.list();
  uint32_t* pref = st.pref();
  uint32_t lvl_b = 0, lvl_e = n_roots, n_list = n_roots;
  int res = BFS_N;
  st.sync();
  for (int k = 0; lvl_b < lvl_e; k++) {
    const int d = d0 - k;       // rest depth of this level's checkIsAllowed calls
    if (d < 1) break;           // checkDirect needs d-1 >= 0
    const bool expand = d >= 2; // children need d-1 >= 1 to probe anything
    for (uint32_t base = lvl_b; base < lvl_e; base += 64) {
      const uint32_t i = base + lane;
      const bool valid = i < lvl_e;
      const uint32_t node = valid ? list[i] : 0;
      uint64_t rb = 0, re = 0;
      if (valid && expand) {
        rb = s.adj_off[node];
        re = s.adj_off[node + 1];
      }
      const bool h = valid && dset_probe(s, node, subj);
      const uint64_t nvalid = __ballot(valid);
      bs.probes += __popcll(nvalid);
      if (__ballot(h)) {
        res = BFS_M;
        break;
      }
      if (!expand) continue;
      bs.rows += __popcll(nvalid);
      uint32_t total;
      const uint32_t excl = wave_excl_scan((uint32_t)(re - rb), &total);
      pref[lane] = excl;
      __builtin_amdgcn_wave_barrier();
      bs.edges += total;
      for (uint32_t eb = 0; eb < total; eb += 64) {
        const uint32_t e = eb + lane;
        const bool act = e < total;
        const int own = act ? owner_search(pref, 64, e) : 0;
        const uint64_t src_b = shfl64(rb, own);
        uint32_t child = NONE;
        if (act) child = s.adj[src_b + (e - pref[own])];
        const bool fresh = act && st.insert(child);
        const uint64_t m = __ballot(fresh);
        const uint32_t cnt = __popcll(m);
        if (n_list + cnt > st.cap()) {
          res = BFS_OVERFLOW;
          break;
        }
        if (fresh) list[n_list + lanes_below(m)] = child;
        n_list += cnt;
      }
      __builtin_amdgcn_wave_barrier();
      if (res != BFS_N) break;
    }
    if (res != BFS_N) break;
    st.sync();
    lvl_b = lvl_e;
    lvl_e = n_list;
  }
  st.finish((uint32_t)min<uint64_t>(n_list, st.cap()));
  return res;
}

}  // namespace kg
