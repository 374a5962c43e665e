// kg_grid.hip -- the grid tier: queries whose BFS outgrew the wave tiers and the backward tier
// (thousands to millions of expanded nodes).  All of them advance together, level-synchronously,
// and every level is spread edge-balanced over the whole GPU, ONE kernel launch per level:
//   log              entries (slot, adjx row start, edge start within its level): level L is
//                    log[base_L, base_L + n_L); entries of a level are laid out in edge order, so
//                    its edges form one range [0, total_L)
//   tile_first       for every GT-edge tile of a level, the entry holding its first edge
//   H                one shared open-addressing visited table of (epoch | slot | node) keys
//   per level        one thread per edge: the tile's entries are staged in LDS and each edge
//                    finds its entry by LDS binary search; children are probed (checkDirect) at
//                    discovery, and children that will themselves be expanded (rest depth >= 2,
//                    non-empty set row, read inline from adjx) are marked and appended
// Appends are workgroup-aggregated through ONE 64-bit atomic that packs (entries << 36 | edges):
// the returned old value gives both the entries' log position and their edge start, so the next
// level's edge prefix sums and tile_first come out of the appends themselves (no scan pass).
// Semantics are those of k_stream / k_medium (kg_check.hip): bounded reachability with every node
// probed once at its shallowest depth.  A round that overflows the log is rerun with fewer slots.
//
// (Rounds 3-5 also had a bidirectional mode -- backward turns from the subject's holders alternating
// with the forward ones, kg_snapshot_tune "grid_bidir" -- off by default since it measured slower on
// both C2 and the heavy-tail point (profiles/r3d_heavy_grid_bidir_ab.jsonl); removed in
// round 6.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kg_bfs.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

// edges per thread of k_grid_level's 256-thread workgroup (-DKG_GRID_EPT=4 builds 1024-edge tiles for A/Bs)
#ifndef KG_GRID_EPT
#define KG_GRID_EPT 2
#endif
constexpr int GEPT = KG_GRID_EPT;
constexpr uint32_t GT = 256u * GEPT;          // edges per tile
constexpr uint64_t TILE_CAP = 1ull << 24;    // tiles per level with a tile_first entry (beyond: log search)
constexpr int EDGE_BITS = 36;                // packed level counter: entries (28 bits) | edges (36 bits)
constexpr uint64_t EDGE_MASK = (1ull << EDGE_BITS) - 1;
constexpr uint64_t ENTRY_MAX = (1ull << (64 - EDGE_BITS)) - 1;

// Level L's counters live in lv[L % 3]: level L reads its own, appends into lv[(L+1) % 3] and
// clears lv[(L+2) % 3] (read by level L-1, appended by level L+1).
struct GridLv {
  unsigned long long base;    // first log index of the level
  unsigned long long packed;  // entries << EDGE_BITS | edges
};

struct GridCtl {
  GridLv lv[3];   // the log's level counters
  uint32_t overflow, pad;
  unsigned long long logged;  // entries over all levels (stats: rows opened)
  unsigned long long edges;   // edges over all levels (stats)
  unsigned long long probes8[8][16];  // per-XCD shards (one 128-B line each)
};

// Per-slot state of a round.  hit: 0 live, 1 IsMember.
struct GridSlots {
  uint32_t* q;     // query index
  uint2* info;     // (tagged subject, rest depth of the root)
  uint32_t* hit;
};

// Visited sets of all slots in ONE open-addressing table of 64-bit keys
//   epoch (15) | 0 (1) | slot (16) | node (32)
// Entries of older epochs (earlier rounds / batches) count as empty, so the table is never
// cleared between rounds; it is zeroed once per 32767 rounds.  Within a round an entry never
// changes once written, so a (possibly stale) plain load that shows this round's epoch is final.
constexpr int GH_PROBES = 128;
constexpr int GH_EPOCH_SHIFT = 49;
constexpr uint32_t GH_EPOCH_WRAP = 0x8000;
__device__ __forceinline__ uint64_t gh_key(uint64_t epoch, uint32_t slot, uint32_t node) {
  return (epoch << GH_EPOCH_SHIFT) | ((uint64_t)slot << 32) | node;
}
__device__ __forceinline__ int gh_insert(uint64_t* H, uint64_t mask, uint64_t key) {
  const uint64_t ep = key >> GH_EPOCH_SHIFT;
  uint64_t h = mix64(key & ((1ull << GH_EPOCH_SHIFT) - 1)) & mask;
  for (int p = 0; p < GH_PROBES; p++) {
    uint64_t cur = H[h];
    for (;;) {
      if (cur == key) return 0;                   // already visited
      if ((cur >> GH_EPOCH_SHIFT) == ep) break;   // another key of this round: next slot
      const uint64_t old = atomicCAS((unsigned long long*)&H[h], (unsigned long long)cur, (unsigned long long)key);
      if (old == cur) return 1;      // inserted
      cur = old;
    }
    h = (h + 1) & mask;
  }
  return -1;  // probe bound: the round is rerun with fewer slots
}

struct GridLog {
  uint32_t* slot;  // slot of the entry
  uint32_t* rb;    // first adjx index of the node's set row
  uint64_t* ex;    // edge start of the entry within its level
  uint2* info;     // the slot's (tagged subject, rest depth of the root), carried by every entry (round 6: a
                   // level reads it with the entry instead of a dependent sl.info[slot] round trip)
  uint32_t* tile_first[2];  // level parity -> tile -> entry (level-relative)
  uint64_t cap;
};

// Workgroup-aggregated append of the lanes with `app` set (entry slot / row start rb / row length
// len) to level counters lv[nl] (tile map tile_first[np]); every thread of the workgroup must call it.
__device__ __forceinline__ void grid_append(GridCtl* ctl, GridLv* lvs, const GridLog& lg, int nl, int np,
                                            uint64_t next_base, bool app, uint32_t slot, uint32_t rb, uint32_t len,
                                            uint2 info) {
  __shared__ uint32_t s_wcnt[4];
  __shared__ uint64_t s_wedge[4];
  __shared__ unsigned long long s_old;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(app);
  // wave-inclusive prefix of row lengths over appending lanes
  uint64_t v = app ? len : 0;
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = shfl_up64(v, off);
    if (lane >= off) v += y;
  }
  if (lane == 63) {
    s_wcnt[wave] = __popcll(m);
    s_wedge[wave] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t tc = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    const uint64_t te = s_wedge[0] + s_wedge[1] + s_wedge[2] + s_wedge[3];
    s_old = tc ? atomicAdd(&lvs[nl].packed, (unsigned long long)((tc << EDGE_BITS) | te)) : 0ull;
  }
  __syncthreads();
  if (app) {
    uint64_t at = s_old >> EDGE_BITS, ex = s_old & EDGE_MASK;
    for (int w = 0; w < wave; w++) {
      at += s_wcnt[w];
      ex += s_wedge[w];
    }
    at += lanes_below(m);
    ex += v - len;
    const uint64_t gi = next_base + at;
    if (gi < lg.cap && at < ENTRY_MAX && ex + len <= EDGE_MASK) {
      lg.slot[gi] = slot;
      lg.rb[gi] = rb;
      lg.ex[gi] = ex;
      lg.info[gi] = info;
      // tiles whose first edge lies in [ex, ex + len): exactly one entry writes each tile
      for (uint64_t t = (ex + GT - 1) / GT; t * GT < ex + len && t < TILE_CAP; t++) lg.tile_first[np][t] = (uint32_t)at;
    } else {
      ctl->overflow = 1;
    }
  }
  __syncthreads();
}

// k_grid_level's appends, buffered in LDS across the workgroup's tiles and flushed with ONE packed
// atomic per GB_BUF entries (round 6): every append of a level hits the same counter, and same-address
// atomics serialise at the memory side (~11 ns each, MI355X_MICROARCH.md "dequeue") -- one per 256-edge
// tile with an append was the level's floor on C3 (~52 us per level, profiles/r6a_c3_timeline.txt).
constexpr uint32_t GB_BUF = 512;
struct GridBuf {
  uint32_t slot[GB_BUF], rb[GB_BUF], len[GB_BUF], pre[GB_BUF];
  uint2 info[GB_BUF];
  uint32_t n, edges;
  uint32_t wcnt[4], wedge[4];
  unsigned long long old;
};

__device__ void grid_flush(GridCtl* ctl, GridLv* lvs, const GridLog& lg, int nl, int np, uint64_t next_base,
                           GridBuf& B) {
  if (threadIdx.x == 0)
    B.old = atomicAdd(&lvs[nl].packed, (unsigned long long)(((uint64_t)B.n << EDGE_BITS) | B.edges));
  __syncthreads();
  const uint64_t at0 = B.old >> EDGE_BITS, ex0 = B.old & EDGE_MASK;
  for (uint32_t i = threadIdx.x; i < B.n; i += blockDim.x) {
    const uint64_t at = at0 + i, ex = ex0 + B.pre[i], gi = next_base + at;
    const uint32_t len = B.len[i];
    if (gi < lg.cap && at < ENTRY_MAX && ex + len <= EDGE_MASK) {
      lg.slot[gi] = B.slot[i];
      lg.rb[gi] = B.rb[i];
      lg.ex[gi] = ex;
      lg.info[gi] = B.info[i];
      // tiles whose first edge lies in [ex, ex + len): exactly one entry writes each tile
      for (uint64_t t = (ex + GT - 1) / GT; t * GT < ex + len && t < TILE_CAP; t++) lg.tile_first[np][t] = (uint32_t)at;
    } else {
      ctl->overflow = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    B.n = 0;
    B.edges = 0;
  }
  __syncthreads();
}

// Every thread of the workgroup (256) calls it; flushes first when the tile's appends do not fit.
__device__ __forceinline__ void grid_push(GridCtl* ctl, GridLv* lvs, const GridLog& lg, int nl, int np,
                                          uint64_t next_base, GridBuf& B, bool app, uint32_t slot, uint32_t rb,
                                          uint32_t len, uint2 info) {
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(app);
  uint32_t x = app ? len : 0u;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) {
    B.wcnt[wave] = (uint32_t)__popcll(m);
    B.wedge[wave] = x;
  }
  __syncthreads();
  const uint32_t tc = B.wcnt[0] + B.wcnt[1] + B.wcnt[2] + B.wcnt[3];
  const uint32_t te = B.wedge[0] + B.wedge[1] + B.wedge[2] + B.wedge[3];
  uint32_t n0 = B.n, e0 = B.edges;  // read by every thread before a flush changes them
  if (tc && (n0 + tc > GB_BUF || e0 + te < e0)) {
    grid_flush(ctl, lvs, lg, nl, np, next_base, B);
    n0 = 0;
    e0 = 0;
  }
  if (app) {
    uint32_t at = n0 + lanes_below(m), pre = e0 + x - len;
    for (int w = 0; w < wave; w++) {
      at += B.wcnt[w];
      pre += B.wedge[w];
    }
    B.slot[at] = slot;
    B.rb[at] = rb;
    B.len[at] = len;
    B.pre[at] = pre;
    B.info[at] = info;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    B.n = n0 + tc;
    B.edges = e0 + te;
  }
  __syncthreads();
}

// slots of a round: queries [base, base + G) of the list, clamped to its device-side length
__device__ __forceinline__ uint32_t round_slots(const uint32_t* d_count, uint32_t base, uint32_t G) {
  const uint32_t c = *d_count;
  return c > base ? min(G, c - base) : 0u;
}

// Level 0: the roots (already probed by k_resolve), one per slot.
__global__ __launch_bounds__(256) void k_grid_init(const RQuery* __restrict__ rq, const uint32_t* __restrict__ qlist,
                                                   const uint32_t* d_count, uint32_t base, uint32_t G, GridLog lg,
                                                   GridSlots sl, uint64_t* H, uint64_t mask, uint64_t epoch,
                                                   GridCtl* ctl) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < round_slots(d_count, base, G);
  uint32_t rb = 0, len = 0;
  uint2 info = make_uint2(0u, 0u);
  if (valid) {
    const uint32_t qi = qlist[base + i];
    const RQuery q = rq[qi];
    sl.q[i] = qi;
    info = make_uint2(q.subj, (uint32_t)q.depth);
    sl.info[i] = info;
    sl.hit[i] = 0;  // the root was already probed (k_resolve)
    if (gh_insert(H, mask, gh_key(epoch, i, q.node)) < 0) ctl->overflow = 1;
    rb = q.beg;
    len = q.len;
  }
  grid_append(ctl, ctl->lv, lg, 0, 0, 0, valid, i, rb, len, info);
}

// Largest j in [lo, hi) with ex[base + j] <= e: the entry holding edge e (search in the log).
__device__ __forceinline__ uint64_t entry_of(const uint64_t* ex, uint64_t base, uint64_t lo, uint64_t hi, uint64_t e) {
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (ex[base + mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Two visited-set inserts whose first probes are issued together (k_grid_level: a thread's two edges).
__device__ __forceinline__ void gh_insert2(uint64_t* H, uint64_t mask, bool a0, uint64_t k0, bool a1, uint64_t k1,
                                           int& r0, int& r1) {
  const uint64_t h0 = mix64(k0 & ((1ull << GH_EPOCH_SHIFT) - 1)) & mask, h1 = mix64(k1 & ((1ull << GH_EPOCH_SHIFT) - 1)) & mask;
  const uint64_t c0 = a0 ? H[h0] : 0ull, c1 = a1 ? H[h1] : 0ull;
  r0 = r1 = 0;
  // the common case: the home slot is this key (seen) or empty of this round (CAS it)
  const uint64_t ep0 = k0 >> GH_EPOCH_SHIFT, ep1 = k1 >> GH_EPOCH_SHIFT;
  bool done0 = !a0, done1 = !a1;
  if (a0 && c0 == k0) done0 = true;
  if (a1 && c1 == k1) done1 = true;
  if (!done0 && (c0 >> GH_EPOCH_SHIFT) != ep0) {
    const uint64_t old = atomicCAS((unsigned long long*)&H[h0], (unsigned long long)c0, (unsigned long long)k0);
    if (old == c0) {
      r0 = 1;
      done0 = true;
    } else if (old == k0) {
      done0 = true;
    }
  }
  if (!done1 && (c1 >> GH_EPOCH_SHIFT) != ep1) {
    const uint64_t old = atomicCAS((unsigned long long*)&H[h1], (unsigned long long)c1, (unsigned long long)k1);
    if (old == c1) {
      r1 = 1;
      done1 = true;
    } else if (old == k1) {
      done1 = true;
    }
  }
  if (!done0) r0 = gh_insert(H, mask, k0);  // the general probe from the home slot
  if (!done1) r1 = gh_insert(H, mask, k1);
}

// One level: two edges per thread (e and e + 256), one GT = 512-edge tile per workgroup iteration
// (round 6; one edge per thread before: a tile's chain of dependent trips covers twice the edges).  Level
// L expands the nodes found at hop L (rest depth D - L >= 2) into hop L + 1: every child is probed
// (checkDirect at its shallowest depth) and kept for the next level while D - (L + 1) >= 2 and its set
// row is non-empty.
// The tile's chain of dependent HBM round trips (round 6, second session: 7 -> 5): tile map -> entries
// (slot, row, edge start and the slot's subject / depth, carried by the entry) -> the slot's answered
// flag and the adjx record together (an answered slot's record is loaded for nothing) -> the visited-set
// word and the child's first dset bucket together (a kept child already visited this round is probed
// again: the same answer) -> the insert's CAS.  The C2 tail tier is a few hundred queries whose levels
// are this chain plus a launch (~12-30 us each, profiles/r6i_headline_timed_timeline.txt).
__global__ __launch_bounds__(256) void k_grid_level(DevSnap s, GridLog lg, int level, GridSlots sl, uint64_t* H,
                                                    uint64_t mask, uint64_t epoch, GridCtl* ctl) {
  __shared__ uint64_t s_beg[GT + 2];
  __shared__ uint32_t s_slot[GT + 2], s_rb[GT + 2];
  __shared__ uint2 s_info[GT + 2];  // per entry: its slot's (subject, rest depth of the root)
  __shared__ uint64_t s_j0, s_cnt;
  __shared__ uint32_t s_void;
  __shared__ GridBuf B;
  if (threadIdx.x == 0) {
    s_void = ctl->overflow;  // one read for the whole workgroup (the loop below has barriers)
    B.n = 0;
    B.edges = 0;
  }
  __syncthreads();
  if (s_void) return;  // the round is void (entries past the log were dropped)
  GridLv* lvs = ctl->lv;
  const int cl3 = level % 3, nl = (level + 1) % 3, zl = (level + 2) % 3;
  const uint64_t lb = lvs[cl3].base, packed = lvs[cl3].packed;
  const uint64_t n = packed >> EDGE_BITS, total = packed & EDGE_MASK;
  const uint64_t next_base = lb + n;
  const uint32_t* tf = lg.tile_first[level & 1];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    lvs[nl].base = next_base;
    lvs[zl].packed = 0;
    ctl->edges += total;
    ctl->logged += n;
  }
  uint32_t probes = 0;
  const int lane = lane_id();
  for (uint64_t t0 = (uint64_t)blockIdx.x * GT; t0 < total; t0 += (uint64_t)gridDim.x * GT) {
    const uint64_t t1 = t0 + GT < total ? t0 + GT : total;
    if (threadIdx.x == 0) {
      const uint64_t t = t0 / GT;
      uint64_t j0, jl;
      if (t + 1 < TILE_CAP) {
        j0 = tf[t];
        jl = t1 < total ? tf[t + 1] : n - 1;  // an entry at or after the tile's last edge
      } else {
        j0 = entry_of(lg.ex, lb, 0, n, t0);
        jl = entry_of(lg.ex, lb, j0, n, t1 - 1);
      }
      s_j0 = j0;
      s_cnt = jl - j0 + 1;
    }
    __syncthreads();
    const uint64_t j0 = s_j0, cnt = s_cnt;
    const bool use_lds = cnt <= GT + 2;  // entries are non-empty: a tile spans <= GT + 1 of them
    if (use_lds)
      for (uint32_t i = threadIdx.x; i < cnt; i += 256) {
        s_beg[i] = lg.ex[lb + j0 + i];
        s_slot[i] = lg.slot[lb + j0 + i];
        s_rb[i] = lg.rb[lb + j0 + i];
        s_info[i] = lg.info[lb + j0 + i];
      }
    __syncthreads();
    // both edges' entry (LDS), then their slots' answered flags and adjx records in flight at once
    bool inr[GEPT];
    uint32_t slot[GEPT], subj[GEPT], hv[GEPT];
    int D[GEPT];
    AdjX x[GEPT];
#pragma unroll
    for (int h = 0; h < GEPT; h++) {
      slot[h] = subj[h] = 0u;
      D[h] = 0;
      const uint64_t e = t0 + threadIdx.x + (uint64_t)h * 256;
      uint64_t beg = 0;
      uint32_t rb = 0;
      inr[h] = e < t1;
      if (inr[h]) {
        uint2 info;
        if (use_lds) {
          uint32_t lo = 0, hi = (uint32_t)cnt;  // largest i < cnt with s_beg[i] <= e
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_beg[mid] <= e) lo = mid;
            else hi = mid;
          }
          beg = s_beg[lo];
          slot[h] = s_slot[lo];
          rb = s_rb[lo];
          info = s_info[lo];
        } else {
          const uint64_t j = entry_of(lg.ex, lb, j0, j0 + cnt, e);
          beg = lg.ex[lb + j];
          slot[h] = lg.slot[lb + j];
          rb = lg.rb[lb + j];
          info = lg.info[lb + j];
        }
        subj[h] = info.x;
        D[h] = (int)info.y;
      }
      hv[h] = inr[h] ? sl.hit[slot[h]] : 1u;  // plain load: a stale 0 only costs this level's work
      x[h] = s.adjx[inr[h] ? rb + (uint32_t)(e - beg) : 0u];
    }
    bool act[GEPT], keep[GEPT], sigok[GEPT];
    uint32_t clen[GEPT], cb[GEPT];
    uint64_t pk[GEPT];
    ulonglong2 pb[GEPT];
#pragma unroll
    for (int h = 0; h < GEPT; h++) {
      act[h] = inr[h] && hv[h] == 0;  // answered at tile start (or no edge): nothing more for this edge
      cb[h] = x[h].begin;
      clen[h] = act[h] ? adjx_len(s, x[h]) : 0u;
      // hop level+1 is expanded at the next level while its rest depth D - (level + 1) >= 2
      keep[h] = act[h] && clen[h] > 0 && level + 2 <= D[h] - 1;
      // the signature rules out most misses; the first bucket of the rest is loaded now, beside the
      // visited-set words below
      sigok[h] = act[h] && sig_maybe(x[h].lsig, x[h].sig, subj_sig(subj[h]));
      pk[h] = dset_key(x[h].node, subj[h]);
      pb[h] = ld_once(
          reinterpret_cast<const ulonglong2*>(s.dset + (sigok[h] ? dset_home(pk[h], s.dset_nb) : 0ull) * DSET_BUCKET));
    }
    int ins[GEPT];
#pragma unroll
    for (int h = 0; h < GEPT; h += 2)
      gh_insert2(H, mask, keep[h], gh_key(epoch, slot[h], x[h].node), keep[h + 1], gh_key(epoch, slot[h + 1], x[h + 1].node),
                 ins[h], ins[h + 1]);
    bool app[GEPT];
#pragma unroll
    for (int h = 0; h < GEPT; h++) {
      if (keep[h] && ins[h] < 0) ctl->overflow = 1;
      const bool fresh = act[h] && (!keep[h] || ins[h] > 0);
      if (fresh && sigok[h]) {
        probes++;
        bool hit = pb[h].x == pk[h] || pb[h].y == pk[h];
        if (!hit && pb[h].y != EMPTY64) hit = dset_probe(s, x[h].node, subj[h]);  // past a full first bucket
        if (hit) atomicExch(&sl.hit[slot[h]], 1u);
      }
      app[h] = fresh && keep[h];
    }
#pragma unroll
    for (int h = 0; h < GEPT; h++)
      grid_push(ctl, lvs, lg, nl, (level + 1) & 1, next_base, B, app[h], slot[h], cb[h], clen[h],
                make_uint2(subj[h], (uint32_t)D[h]));
  }
  if (B.n) grid_flush(ctl, lvs, lg, nl, (level + 1) & 1, next_base, B);
  for (int off = 32; off; off >>= 1) probes += __shfl_xor(probes, off, 64);
  if (lane == 0 && probes) atomicAdd(&ctl->probes8[blockIdx.x & 7][threadIdx.x >> 6], (unsigned long long)probes);
}

static_assert(sizeof(GridCtl) % 8 == 0 && sizeof(GridCtl) / 8 + 1 <= GRID_SUM_WORDS,
              "a round's counters and the list length fit GRID_SUM_WORDS");
__global__ void k_grid_finish(GridSlots sl, const uint32_t* d_count, uint32_t base, uint32_t G, uint8_t* out,
                              uint32_t* err, const GridCtl* ctl, uint64_t* sum) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // the list length next to the round's counters (which live in sum) for the batch's single readback
  if (sum && i == 0) sum[sizeof(GridCtl) / 8] = *d_count;
  if (i >= round_slots(d_count, base, G) || ctl->overflow) return;
  const uint32_t qi = sl.q[i];
  out[qi] = sl.hit[i] == 1 ? KG_IS_MEMBER : KG_NOT_MEMBER;
  if (err) err[qi] = KG_ERR_NONE;
}

// Host driver: qlist / count live on the device.  A round is launched without knowing the count
// (the kernels clamp to it); the host reads the counters once per round, after its last kernel.
// phase 0: run every round synchronously.  phase 1: enqueue the first round and its readback, return
// 1 without waiting (the caller synchronises the stream once for the whole batch).  phase 2: resume
// after that synchronisation: read the first round's result and run further rounds if needed.
static uint64_t grid_full_cap(const Snapshot* s) {
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  return std::max<uint64_t>(nn + 1024, 64ull << 20);  // one slot logs each node at most once
}
constexpr uint32_t G0 = 0xFFFF;  // slot field is 16 bits

struct GridView {  // pointers into a pool laid out for `cap` log entries (per direction)
  uint64_t cap = 0, hcap = 0;
  uint64_t* H = nullptr;
  GridLog lg{};
  GridSlots sl{};
  GridCtl* ctl = nullptr;       // the running round's counters
  GridCtl* ctl_pool = nullptr;  // the pool's own block
};

// One log and a visited table sized for twice the logged entries (load <= 0.5).
static int grid_layout(GridPool* P, uint64_t cap, hipStream_t stream, GridView* v) {
  uint64_t hcap = 1;
  while (hcap < 2 * cap) hcap <<= 1;
  const size_t log_bytes = cap * (4 + 4 + 8 + 8) + 2 * TILE_CAP * 4;
  const size_t need = hcap * 8 + log_bytes + (size_t)G0 * 16 + sizeof(GridCtl) + 4096;
  if (need > P->bytes) {
    P->release();
    HIPC(hipMalloc(&P->mem, need));
    HIPC(hipMemsetAsync(P->mem, 0, hcap * 8, stream));  // epoch 0 = empty
    P->bytes = need;
  }
  P->cap = cap;
  char* p = (char*)P->mem;
  v->cap = cap;
  v->hcap = hcap;
  v->H = (uint64_t*)p;
  p += hcap * 8;
  GridLog* lg = &v->lg;
  lg->cap = cap;
  lg->ex = (uint64_t*)p;
  p += cap * 8;
  lg->slot = (uint32_t*)p;
  p += cap * 4;
  lg->rb = (uint32_t*)p;
  p += cap * 4;
  lg->info = (uint2*)p;
  p += cap * 8;
  lg->tile_first[0] = (uint32_t*)p;
  p += TILE_CAP * 4;
  lg->tile_first[1] = (uint32_t*)p;
  p += TILE_CAP * 4;
  v->sl.info = (uint2*)p;
  p += (size_t)G0 * 8;
  v->sl.q = (uint32_t*)p;
  v->sl.hit = v->sl.q + G0;
  p += (size_t)G0 * 8;
  v->ctl = v->ctl_pool = (GridCtl*)(((uintptr_t)p + 255) & ~uintptr_t(255));
  return 0;
}

int grid_reserve(Snapshot* s) {
  HIPC(hipSetDevice(s->device));
  std::lock_guard<std::mutex> lk(s->giant_mu);
  GridView v;
  if (int rc = grid_layout(&s->giant, grid_full_cap(s), s->stream, &v)) return rc;
  HIPC(hipStreamSynchronize(s->stream));
  return 0;
}

// Host driver: qlist / count live on the device.  A round is launched without knowing the count
// (the kernels clamp to it); the host reads the counters once per round, after its last kernel.
// phase 0: run every round synchronously.  phase 1: enqueue the first round and its readback, return
// 1 without waiting (the caller synchronises the stream once for the whole batch).  phase 2: resume
// after that synchronisation: read the first round's result and run further rounds if needed.
//
// Memory: the queries that reach this tier touch far fewer nodes than the graph holds, so a
// workspace's pool has a log of min(n_nodes, 16 Mi) entries (~0.6 GB with its hash and tile maps,
// instead of ~7 GB at 1 B tuples and ~27 GB at C3's 688 M nodes -- per batch in flight).  A round
// that overflows reruns with a quarter of the slots; a single query that overflows the workspace
// pool on its own reruns in the snapshot's shared full-size pool (allocated once, lazily or by
// kg_snapshot_tune "grid_reserve"; one query at a time), so no workspace ever reallocates.  After
// a round succeeds the slot count grows back (x4), so one giant query does not serialise the rest.
int grid_tier(Snapshot* s, Workspace* w, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count, int global_max_depth,
              uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs, int phase, bool allow_ms, uint64_t* dsum,
              const uint64_t* hsum) {
  static_assert(sizeof(GridCtl) + 64 <= 32768, "grid readback fits the upper half of the pinned buffer");
  // graphs small enough for dense per-node masks: 64 queries share each walk (kg_msbfs.hip)
  if (allow_ms && ms_usable(s, global_max_depth)) {
    const int rc = ms_tier(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    if (rc != 2) return rc;
    // a single group overflowed the MS-BFS level buffers: every query of the list runs the per-query
    // rounds (answers already written are rewritten with the same values)
    if (int rc2 = grid_tier(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, 0, false)) return rc2;
    w->grid_reran = true;
    return 0;
  }
  char* pin = (char*)w->host_buf(65536);
  if (!pin) return set_error(-1, "pinned host buffer");
  uint32_t* hb = (uint32_t*)(pin + 32768);  // the lower half holds the batch's Ctl readback
  const uint64_t full_cap = grid_full_cap(s);
  const uint64_t small_cap = std::min<uint64_t>(full_cap, s->grid_small_cap ? s->grid_small_cap : 16ull << 20);
  GridPool* gp = &w->grid;
  std::unique_lock<std::mutex> giant_lk(s->giant_mu, std::defer_lock);
  GridView v;
  if (int rc = grid_layout(gp, small_cap, stream, &v)) return rc;
  uint32_t G = G0;
  int64_t count = -1;  // unknown until the first readback
  bool resume = phase == 2;
  for (uint32_t done = 0; count < 0 || done < (uint64_t)count;) {
   if (!resume) {
    if (phase == 1) w->grid_reran = false;
    if (phase == 2) w->grid_reran = true;  // rounds past the first: the caller re-reads the results
    if (++gp->epoch == GH_EPOCH_WRAP) {  // epoch wrap: the table is zeroed once per 32767 rounds
      HIPC(hipMemsetAsync(v.H, 0, v.hcap * 8, stream));
      gp->epoch = 1;
    }
    const uint64_t epoch = gp->epoch;
    const uint32_t slot_blocks = (G + 255) / 256;
    const uint32_t lgrid = (uint32_t)s->n_cu * s->grid_wgs;
    // the first round of a batch keeps its counters in the caller's zeroed Ctl (kg_grid.h), later
    // rounds in the pool's own block
    const bool fold = phase == 1 && dsum;
    v.ctl = fold ? reinterpret_cast<GridCtl*>(dsum) : v.ctl_pool;
    if (!fold) HIPC(hipMemsetAsync(v.ctl, 0, sizeof(GridCtl), stream));
    hipLaunchKernelGGL(k_grid_init, dim3(slot_blocks), dim3(256), 0, stream, rq, qlist, d_count, done, G, v.lg, v.sl,
                       v.H, v.hcap - 1, epoch, v.ctl);
    HIPC(hipGetLastError());
    // Levels run back to back on the device (sizes never come back to the host; an empty level
    // costs one near-empty launch): level k expands nodes at rest depth D-k >= 2, so at most
    // global_max_depth-1 levels exist
    const int max_levels = std::max(1, global_max_depth - 1);
    for (int t = 0; t < max_levels; t++) {
      w->lev_mark(stream, false, 1);
      hipLaunchKernelGGL(k_grid_level, dim3(lgrid), dim3(256), 0, stream, s->ds, v.lg, t, v.sl, v.H, v.hcap - 1, epoch,
                         v.ctl);
      HIPC(hipGetLastError());
      w->lev_mark(stream, true, 1);
    }
    hipLaunchKernelGGL(k_grid_finish, dim3(slot_blocks), dim3(256), 0, stream, v.sl, d_count, done, G, out, err, v.ctl,
                       fold ? dsum : nullptr);
    HIPC(hipGetLastError());
    if (!fold) {
      HIPC(hipMemcpyAsync(hb, v.ctl, sizeof(GridCtl), hipMemcpyDeviceToHost, stream));
      HIPC(hipMemcpyAsync(hb + sizeof(GridCtl) / 4, d_count, 4, hipMemcpyDeviceToHost, stream));
    }
    if (phase == 1) return 1;  // first round enqueued; the caller synchronises and resumes
    HIPC(hipStreamSynchronize(stream));
   }
    GridCtl h{};
    if (resume && hsum) {  // the first round's summary came back with the caller's readback
      memcpy(&h, hsum, sizeof h);
      count = (int64_t)(uint32_t)hsum[sizeof(GridCtl) / 8];
    } else {
      memcpy(&h, hb, sizeof h);
      count = hb[sizeof(GridCtl) / 4];
    }
    resume = false;
    const uint32_t cnt = count > done ? (uint32_t)std::min<int64_t>(G, count - done) : 0u;
    if (gs) {
      gs->rows += h.logged;
      gs->edges += h.edges;
    }
    if (h.overflow) {  // log or probe bound exceeded: rerun these queries with fewer slots
      if (G == 1) {
        if (gp == &s->giant) return set_error(KG_ERR_RESOURCE_CODE, "grid tier capacity exceeded");
        // one query alone overflowed the workspace pool: rerun it in the shared full-size pool
        giant_lk.lock();
        gp = &s->giant;
        if (int rc = grid_layout(gp, full_cap, stream, &v)) return rc;
        continue;
      }
      G = std::max<uint32_t>(1, std::min(G, cnt) / 4);
      continue;
    }
    if (gs) {
      for (int x = 0; x < 8; x++)
        for (int k = 0; k < 16; k++) gs->probes += h.probes8[x][k];
      gs->done += cnt;
      gs->logged += h.logged;
    }
    done += cnt;
    if (gp == &s->giant) {  // back to the workspace pool for the rest
      gp = &w->grid;
      if (int rc = grid_layout(gp, small_cap, stream, &v)) return rc;
      giant_lk.unlock();
    }
    if (G < G0) G = (uint32_t)std::min<uint64_t>(G0, (uint64_t)G * 4);
  }
  return 0;
}

}  // namespace kg
