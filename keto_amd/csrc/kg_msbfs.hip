// kg_msbfs.hip -- the grid tier's queries as a multi-source bit-parallel BFS (MS-BFS), for graphs
// whose node count is small enough for dense per-node masks (the heavy-tail point: ~2 x 10^5 nodes,
// ~250 set edges per node).
//
// Why: on such a graph every root reaches the same hub groups within two hops, so the per-query
// forward searches of the grid tier (kg_grid.hip) walk the SAME edges again and again -- ~1 M edge
// visits per query, 30-70 G per 250 k-check batch, at the HBM rate of the adjacency stream.  Here 64
// queries share one walk: every node holds a 64-bit mask per group of 64 queries (bit j = query j of
// the group), a level expands each frontier node's set row ONCE for all the group's queries that
// reached it at that hop, and the work per level is the union of the 64 frontiers instead of their
// sum.  Per query the semantics are exactly the grid tier's / k_stream's (bounded reachability,
// engine.go:87-145 checkExpandSubject over checkDirect engine.go:148-177, every node expanded once at
// its shallowest hop): a bit of a node's frontier mask is set only at the hop where that query first
// reaches the node, and it is expanded only while the query's rest depth allows.
//
//   VIS[g][node]  queries of group g that reached the node (and may expand it)
//   FR[2][g][node] frontier masks of the current / next level
//   TG[g][node]   queries of group g whose subject the node holds (its check row has the exact tuple:
//                 the holder index hold[], i.e. checkDirect's answer for every query at once) -- for
//                 subjects with at most tg_cap holders; a popular subject's queries are probed in
//                 dset per newly reached node instead (marking 10^4..10^5 holders per query cost
//                 more than the whole walk)
//   HIT[g]        queries of group g answered IsMember; their bits stop propagating at the next tile
//   PM / EM[g][h] queries whose rest depth lets a node at hop h be probed (D-1 >= h) / expanded (D-2 >= h)
// Levels are edge-balanced over the whole GPU like the grid tier's: entries (group, node, row) of a
// level are appended with one packed 64-bit atomic per workgroup (entries << 36 | edges), which
// yields each entry's edge offset, and tile_first maps every 256-edge tile to its first entry.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kg_bfs.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

namespace {

constexpr uint64_t MS_TILE_CAP = 1ull << 24;  // tiles per level with a tile_first entry (beyond: search)
constexpr int MS_EDGE_BITS = 36;
constexpr uint64_t MS_EDGE_MASK = (1ull << MS_EDGE_BITS) - 1;
constexpr uint64_t MS_ENTRY_MAX = (1ull << (64 - MS_EDGE_BITS)) - 1;
constexpr int MS_HOPS = 32;  // depth masks per group (global max depth <= 32 here)
// edges per tile of k_ms_level: one lane per edge (the LDS staging is (TE + 2) x K words x 2)
constexpr uint32_t ms_tile_edges(int K) { return K <= 8 ? 256u : 128u; }

struct MsCtl {
  unsigned long long packed[3];  // per level buffer (2: the compacted level): entries << 36 | edges
  unsigned long long edges, logged;
  uint32_t overflow, pad;
  unsigned long long eload, wact;  // k_ms_level: adjx records loaded, (edge, 64-query word) pairs with work
};

// A group is 64 * K queries; every per-node mask is K consecutive 64-bit words (node-major), so the
// K lanes that handle one edge touch one contiguous 8K-byte run of each mask array.
struct MsView {
  uint32_t n;      // nodes
  uint32_t G;      // groups of this round
  uint64_t cap;    // entries per level buffer
  // VIS and TG of one (group, node) share one 16K-byte record (round 6; separate arrays before): the
  // level reads both for an edge with new bits, so they are one random line (K = 8: 128 B) instead of two
  uint64_t* vt;    // [G][n][2K]: VIS words, then TG words
  uint64_t* fr[2];  // [G][n][K] each
  uint32_t* stamp;  // [G][n]: 1 + the last hop the node was appended at (one entry per hop)
  uint64_t* hit;   // [G][K]
  uint64_t* many;  // [G][K]: queries whose subject has more than tg_cap holders (probed, no TG bits)
  uint32_t* gmany;  // [G]: 1 when any word of many[g] is non-zero
  uint32_t* qs;    // [G][64K] tagged subject
  uint32_t tg_cap;
  uint64_t* pm;    // [G][MS_HOPS][K]
  uint64_t* em;    // [G][MS_HOPS][K]
  uint32_t* qi;    // [G][64K] query index (NONE: empty bit)
  uint32_t* qd;    // [G][64K] rest depth
  // level buffers 0 / 1 alternate (level L reads L & 1, appends to the other); buffer 2 holds level
  // L's live entries after k_ms_compact, which k_ms_level walks
  uint32_t* eg[3];  // entry group
  uint32_t* en[3];  // entry node
  uint32_t* erb[3];  // entry row start (adjx)
  uint64_t* ex[3];  // entry edge offset within its level
  uint32_t* tf[3];  // tile -> first entry
  MsCtl* ctl;
};

__device__ __forceinline__ uint32_t ms_round_slots(const uint32_t* d_count, uint32_t base, uint32_t cap) {
  const uint32_t c = *d_count;
  return c > base ? min(cap, c - base) : 0u;
}

// Workgroup-aggregated append to level buffer b (every thread of the workgroup calls it); TE edges
// per tile of the level kernel that will read the buffer.
template <uint32_t TE>
__device__ __forceinline__ void ms_append(const MsView& v, int b, bool app, uint32_t g, uint32_t node, uint32_t rb,
                                          uint32_t len) {
  __shared__ uint32_t s_wcnt[4];
  __shared__ uint64_t s_wedge[4];
  __shared__ unsigned long long s_old;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(app);
  uint64_t x = app ? len : 0;
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = shfl_up64(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) {
    s_wcnt[wave] = __popcll(m);
    s_wedge[wave] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t tc = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    const uint64_t te = s_wedge[0] + s_wedge[1] + s_wedge[2] + s_wedge[3];
    s_old = tc ? atomicAdd(&v.ctl->packed[b], (unsigned long long)((tc << MS_EDGE_BITS) | te)) : 0ull;
  }
  __syncthreads();
  if (app) {
    uint64_t at = s_old >> MS_EDGE_BITS, e0 = s_old & MS_EDGE_MASK;
    for (int w = 0; w < wave; w++) {
      at += s_wcnt[w];
      e0 += s_wedge[w];
    }
    at += lanes_below(m);
    e0 += x - len;
    if (at < v.cap && at < MS_ENTRY_MAX && e0 + len <= MS_EDGE_MASK) {
      v.eg[b][at] = g;
      v.en[b][at] = node;
      v.erb[b][at] = rb;
      v.ex[b][at] = e0;
      for (uint64_t t = (e0 + TE - 1) / TE; t * TE < e0 + len && t < MS_TILE_CAP; t++) v.tf[b][t] = (uint32_t)at;
    } else {
      v.ctl->overflow = 1;
    }
  }
  __syncthreads();
}

// The level kernel's appends, buffered in LDS across its tiles and flushed with ONE packed atomic per
// MS_BUF entries (round 6): every append hits the same counter, and same-address atomics serialise at
// the memory side (~11 ns each, MI355X_MICROARCH.md "dequeue"); one per tile was ~0.8 M per heavy-tail
// batch.  The entries of one flush keep their order, so edge offsets are the buffer's own prefix sums.
constexpr uint32_t MS_BUF = 512;
struct MsBuf {
  uint32_t g[MS_BUF], node[MS_BUF], rb[MS_BUF], len[MS_BUF], pre[MS_BUF];
  uint32_t n, edges;
  uint32_t wcnt[4], wedge[4];
  unsigned long long old;
};

template <uint32_t TE>
__device__ void ms_flush(const MsView& v, int b, MsBuf& B) {
  if (threadIdx.x == 0)
    B.old = atomicAdd(&v.ctl->packed[b], (unsigned long long)(((uint64_t)B.n << MS_EDGE_BITS) | B.edges));
  __syncthreads();
  const uint64_t at0 = B.old >> MS_EDGE_BITS, e00 = B.old & MS_EDGE_MASK;
  for (uint32_t i = threadIdx.x; i < B.n; i += blockDim.x) {
    const uint64_t at = at0 + i, e0 = e00 + B.pre[i];
    const uint32_t len = B.len[i];
    if (at < v.cap && at < MS_ENTRY_MAX && e0 + len <= MS_EDGE_MASK) {
      v.eg[b][at] = B.g[i];
      v.en[b][at] = B.node[i];
      v.erb[b][at] = B.rb[i];
      v.ex[b][at] = e0;
      for (uint64_t t = (e0 + TE - 1) / TE; t * TE < e0 + len && t < MS_TILE_CAP; t++) v.tf[b][t] = (uint32_t)at;
    } else {
      v.ctl->overflow = 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    B.n = 0;
    B.edges = 0;
  }
  __syncthreads();
}

// Every thread of the workgroup calls it (256 threads); flushes first when the tile's appends do not fit.
template <uint32_t TE>
__device__ __forceinline__ void ms_push(const MsView& v, int b, MsBuf& B, bool app, uint32_t g, uint32_t node,
                                        uint32_t rb, uint32_t len) {
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
  if (tc && (n0 + tc > MS_BUF || e0 + te < e0)) {
    ms_flush<TE>(v, b, B);
    n0 = 0;
    e0 = 0;
  }
  if (app) {
    uint32_t at = n0 + lanes_below(m), pre = e0 + x - len;
    for (int w = 0; w < wave; w++) {
      at += B.wcnt[w];
      pre += B.wedge[w];
    }
    B.g[at] = g;
    B.node[at] = node;
    B.rb[at] = rb;
    B.len[at] = len;
    B.pre[at] = pre;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    B.n = n0 + tc;
    B.edges = e0 + te;
  }
  __syncthreads();
}

// The round's queries: bit b of group g = query base + 64K g + b (word b / 64).  Roots are hop 0
// (k_resolve probed them); each (group, root) pair becomes one level-0 entry.
template <int K>
__global__ __launch_bounds__(256) void k_ms_init(const RQuery* __restrict__ rq, const uint32_t* __restrict__ qlist,
                                                 const uint32_t* d_count, uint32_t base, MsView v) {
  constexpr uint32_t Q = 64u * K;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nq = ms_round_slots(d_count, base, v.G * Q);
  const bool inside = i < v.G * Q;
  const uint32_t g = i / Q, b = i % Q;
  bool app = false;
  uint32_t node = 0, rb = 0, len = 0;
  if (inside) {
    uint32_t qidx = NONE, d = 0, subj = NONE;
    if (i < nq) {
      qidx = qlist[base + i];
      const RQuery q = rq[qidx];
      d = (uint32_t)max(q.depth, 0);
      subj = q.subj;
      node = q.node;
      rb = q.beg;
      len = q.len;
      const uint64_t bit = 1ull << (b & 63);
      const size_t at = ((size_t)g * v.n + node) * K + (b >> 6);
      atomicOr((unsigned long long*)&v.vt[((size_t)g * v.n + node) * 2 * K + (b >> 6)], (unsigned long long)bit);
      atomicOr((unsigned long long*)&v.fr[0][at], (unsigned long long)bit);
      app = len > 0 && atomicMax(&v.stamp[(size_t)g * v.n + node], 1u) < 1u;
    }
    v.qi[i] = qidx;
    v.qd[i] = d;
    v.qs[i] = subj;
  }
  ms_append<ms_tile_edges(K)>(v, 0, app, g, node, rb, len);
}

// One thread per (group, hop, word): the depth masks (and, at hop 0, a clear hit word).
template <int K>
__global__ void k_ms_masks(MsView v) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= v.G * (uint32_t)MS_HOPS * K) return;
  const uint32_t g = i / (MS_HOPS * K), r = i % (MS_HOPS * K);
  const int h = (int)(r / K), k = (int)(r % K);
  uint64_t pm = 0, em = 0;
  for (int j = 0; j < 64; j++) {
    const int d = (int)v.qd[(size_t)g * 64 * K + k * 64 + j];
    if (d - 1 >= h) pm |= 1ull << j;
    if (d - 2 >= h) em |= 1ull << j;
  }
  v.pm[i] = pm;
  v.em[i] = em;
  if (h == 0) {
    v.hit[(size_t)g * K + k] = 0;
    v.many[(size_t)g * K + k] = 0;
    if (k == 0) v.gmany[g] = 0;
  }
}

// One wave per query: its subject's holders get the query's bit in TG (checkDirect for every node).
template <int K>
__global__ __launch_bounds__(256) void k_ms_holders(DevSnap s, const RQuery* __restrict__ rq, MsView v) {
  constexpr uint32_t Q = 64u * K;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= v.G * Q) return;
  const uint32_t qidx = v.qi[i];
  if (qidx == NONE) return;
  const uint2 hr = holders_find(s, v.qs[i]);
  const uint32_t g = i / Q, b = i % Q;
  const uint64_t bit = 1ull << (b & 63);
  if (hr.y > v.tg_cap) {
    if (lane_id() == 0) {
      atomicOr((unsigned long long*)&v.many[(size_t)g * K + (b >> 6)], (unsigned long long)bit);
      v.gmany[g] = 1u;
    }
    return;
  }
  for (uint32_t k = lane_id(); k < hr.y; k += 64)
    atomicOr((unsigned long long*)&v.vt[((size_t)g * v.n + s.hold[hr.x + k]) * 2 * K + K + (b >> 6)],
             (unsigned long long)bit);
}

__device__ __forceinline__ uint64_t ms_entry_of(const uint64_t* ex, uint64_t lo, uint64_t hi, uint64_t e) {
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (ex[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Level L: the frontier (hop L) in buffer cur is expanded into hop L+1, appended to buffer cur ^ 1.
// ONE lane per edge (round 6; rounds 3-5 ran K lanes per edge, one mask word each, 2 edges per lane
// group: a 64-edge tile per workgroup iteration, whose chain of dependent round trips -- tile map,
// staged entries, adjx record, child masks, hop stamp, two append atomics on one counter -- was the
// level's time at ~6 us per tile, profiles/r6a_heavy_kernel_stats.csv).  A lane loads its edge's adjx
// record, then the child's K VIS words (and its TG words only when a new bit may use them) as 16-B
// loads, and does the K words' logic itself: TE = 256 edges per tile (128 at K = 16), one append per
// tile.  A tile's entries are staged in LDS with their frontier masks already filtered by depth and
// answered queries at tile start (`want`: may probe the child at hop L+1, `s_em`: may expand it), so an
// edge whose K words are all empty is not even loaded.
//
// Per edge the updates are blind ORs on the masks loaded once (no returning atomic on the chain): the
// bits new to the child are `want & ~vis` as loaded.  Two edges of one level that reach the same
// child can both see a bit as new; both then OR the same bits into vis / the next frontier / hit
// (idempotent) and probe the same subjects -- duplicated work, the same answer, since a bit absent
// from vis when this level started can only have been set by this level, i.e. at the same hop.  The
// one returning atomic is the node's hop stamp (one level entry per (group, node, hop)), skipped when
// the loaded stamp already says so.
template <int K>
__device__ __forceinline__ void ms_load_words(const uint64_t* p, uint64_t (&w)[K]) {
  if constexpr (K == 1) {
    w[0] = p[0];
  } else {
    const uint4* q = reinterpret_cast<const uint4*>(p);  // K words of one node: 8K-byte aligned
#pragma unroll
    for (int j = 0; j < K / 2; j++) {
      const uint4 x = q[j];
      w[2 * j] = (uint64_t)x.x | ((uint64_t)x.y << 32);
      w[2 * j + 1] = (uint64_t)x.z | ((uint64_t)x.w << 32);
    }
  }
}

// (256, 4): 4 workgroups per CU fit the LDS (~33 KB each: staged want words + the append buffer)
template <int K>
// cur: the entry buffer walked (2: the compacted level); the frontier masks of hop L are fr[L & 1] and
// hop L+1's go to fr[nx = (L & 1) ^ 1]
__global__ __launch_bounds__(256, 4) void k_ms_level(DevSnap s, MsView v, int L, int cur, int nx) {
  constexpr uint32_t TE = ms_tile_edges(K);
  __shared__ uint64_t s_want[TE + 2][K];
  __shared__ uint64_t s_beg[TE + 2];
  __shared__ uint32_t s_g[TE + 2], s_rb[TE + 2], s_gm[TE + 2];
  __shared__ uint64_t s_j0, s_cnt;
  __shared__ uint32_t s_void;
  __shared__ MsBuf B;
  if (threadIdx.x == 0) {
    s_void = v.ctl->overflow;  // one read for the whole workgroup (the loop below has barriers)
    B.n = 0;
    B.edges = 0;
  }
  __syncthreads();
  if (s_void) return;
  const uint64_t packed = v.ctl->packed[cur];
  const uint64_t n_e = packed >> MS_EDGE_BITS, total = packed & MS_EDGE_MASK;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    v.ctl->edges += total;
    v.ctl->logged += n_e;
  }
  const uint32_t n = v.n;
  const int h0 = min(L, MS_HOPS - 1), h1 = min(L + 1, MS_HOPS - 1);
  const uint32_t want_st = (uint32_t)L + 2;
  // work counters (kg_stats ms_edges_loaded / ms_words_active): per lane, one atomic per wave at the end
  unsigned long long c_eload = 0, c_wact = 0;
  for (uint64_t t0 = (uint64_t)blockIdx.x * TE; t0 < total; t0 += (uint64_t)gridDim.x * TE) {
    const uint64_t t1 = t0 + TE < total ? t0 + TE : total;
    if (threadIdx.x == 0) {
      const uint64_t t = t0 / TE;
      uint64_t j0, jl;
      if (t + 1 < MS_TILE_CAP) {
        j0 = v.tf[cur][t];
        jl = t1 < total ? v.tf[cur][t + 1] : n_e - 1;
      } else {
        j0 = ms_entry_of(v.ex[cur], 0, n_e, t0);
        jl = ms_entry_of(v.ex[cur], j0, n_e, t1 - 1);
      }
      s_j0 = j0;
      s_cnt = jl - j0 + 1;
    }
    __syncthreads();
    const uint64_t j0 = s_j0, cnt = s_cnt;  // entries are non-empty: a tile spans <= TE + 1 of them
    for (uint32_t w = threadIdx.x; w < cnt * K; w += 256) {
      const uint32_t i = w / K, kk = w % K;
      const uint64_t q = j0 + i;
      const uint32_t g = v.eg[cur][q];
      if (kk == 0) {
        s_beg[i] = v.ex[cur][q];
        s_rb[i] = v.erb[cur][q];
        s_g[i] = g;
        s_gm[i] = v.gmany[g];
      }
      // the queries of the word that reach the child first at hop L+1 and may still probe there (a
      // later arrival has less rest depth: its probe and expansion are subsets of the first one's)
      s_want[i][kk] = v.fr[nx ^ 1][((size_t)g * n + v.en[cur][q]) * K + kk] & v.em[((size_t)g * MS_HOPS + h0) * K + kk] &
                      ~v.hit[(size_t)g * K + kk] & v.pm[((size_t)g * MS_HOPS + h1) * K + kk];
    }
    __syncthreads();
    const uint64_t e = t0 + threadIdx.x;
    bool app = false;
    uint32_t child = 0, cb = 0, clen = 0, g = 0;
    if (threadIdx.x < TE && e < t1) {
      uint32_t lo = 0, hi = (uint32_t)cnt;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_beg[mid] <= e) lo = mid;
        else hi = mid;
      }
      g = s_g[lo];
      uint64_t want[K];
      uint64_t any = 0;
#pragma unroll
      for (int k = 0; k < K; k++) {
        want[k] = s_want[lo][k];
        any |= want[k];
        c_wact += want[k] ? 1u : 0u;
      }
      if (any) {
        c_eload++;
        const AdjX x = s.adjx[s_rb[lo] + (uint32_t)(e - s_beg[lo])];
        const size_t base = ((size_t)g * n + x.node) * K, vbase = 2 * base;  // fr / vt record of the child
        uint64_t vis0[K];
        ms_load_words<K>(v.vt + vbase, vis0);
        const uint32_t st0 = v.stamp[(size_t)g * n + x.node];
        uint64_t nw[K], anynw = 0;
#pragma unroll
        for (int k = 0; k < K; k++) {
          nw[k] = want[k] & ~vis0[k];
          anynw |= nw[k];
        }
        if (anynw) {
          // checkDirect: TG bits for subjects with few holders, dset probes for popular ones
          uint64_t many[K];
#pragma unroll
          for (int k = 0; k < K; k++) many[k] = s_gm[lo] ? v.many[(size_t)g * K + k] : 0ull;
          uint64_t tg0[K];
          ms_load_words<K>(v.vt + vbase + K, tg0);
          const bool can_expand = adjx_len16(x) != 0;
          uint64_t anyex = 0;
#pragma unroll
          for (int k = 0; k < K; k++) {
            if (!nw[k]) continue;
            atomicOr((unsigned long long*)&v.vt[vbase + k], (unsigned long long)nw[k]);
            uint64_t hits = nw[k] & ~many[k] & tg0[k];
            for (uint64_t m = nw[k] & many[k]; m; m &= m - 1) {
              const uint32_t subj = v.qs[(size_t)g * 64 * K + k * 64 + __builtin_ctzll(m)];
              if (sig_maybe(x.lsig, x.sig, subj_sig(subj)) && dset_probe(s, x.node, subj)) hits |= m & (~m + 1);
            }
            if (hits) atomicOr((unsigned long long*)&v.hit[(size_t)g * K + k], (unsigned long long)hits);
            // expansion: those that may expand it at hop L+1 (a tiny per-group table: L1 / L2 hits)
            const uint64_t ex = can_expand ? (nw[k] & v.em[((size_t)g * MS_HOPS + h1) * K + k]) : 0ull;
            if (ex) atomicOr((unsigned long long*)&v.fr[nx][base + k], (unsigned long long)ex);
            anyex |= ex;
          }
          if (anyex) {
            app = st0 < want_st && atomicMax(&v.stamp[(size_t)g * n + x.node], want_st) < want_st;
            child = x.node;
            cb = x.begin;
            clen = adjx_len(s, x);
          }
        }
      }
    }
    ms_push<TE>(v, nx, B, app, g, child, cb, clen);
  }
  if (B.n) ms_flush<TE>(v, nx, B);
  for (int off = 32; off; off >>= 1) {
    c_eload += __shfl_xor(c_eload, off, 64);
    c_wact += __shfl_xor(c_wact, off, 64);
  }
  if (lane_id() == 0 && c_wact) {
    atomicAdd(&v.ctl->eload, c_eload);
    atomicAdd(&v.ctl->wact, c_wact);
  }
}

// Before level L: the entries of buffer `cur` that still have work -- a frontier bit that may probe at
// hop L+1 and whose query is not answered yet -- are copied to buffer 2 (any order: a level's updates
// are order-free), which the level walks.  On the heavy-tail point 84 % of the logged edges belonged
// to entries whose queries had all been answered when their level began (round 6: 243 M edge slots per
// batch, 40 M loaded): a dead entry still held a whole row's worth of tile lanes.
template <int K>
__global__ __launch_bounds__(256) void k_ms_compact(MsView v, int L, int cur) {
  __shared__ MsBuf B;
  __shared__ uint32_t s_void;
  if (threadIdx.x == 0) {
    s_void = v.ctl->overflow;
    B.n = 0;
    B.edges = 0;
  }
  __syncthreads();
  if (s_void) return;
  constexpr uint32_t TE = ms_tile_edges(K);
  const uint64_t packed = v.ctl->packed[cur];
  const uint64_t n_e = packed >> MS_EDGE_BITS, total = packed & MS_EDGE_MASK;
  const int h0 = min(L, MS_HOPS - 1), h1 = min(L + 1, MS_HOPS - 1);
  const uint32_t n = v.n;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < n_e; b0 += stride) {
    const uint64_t q = b0 + threadIdx.x;
    bool live = false;
    uint32_t g = 0, node = 0, rb = 0, len = 0;
    if (q < n_e) {
      g = v.eg[cur][q];
      node = v.en[cur][q];
      rb = v.erb[cur][q];
      const uint64_t e0 = v.ex[cur][q], e1 = q + 1 < n_e ? v.ex[cur][q + 1] : total;
      len = (uint32_t)(e1 - e0);
      uint64_t any = 0;
#pragma unroll
      for (int k = 0; k < K; k++)
        any |= v.fr[cur][((size_t)g * n + node) * K + k] & v.em[((size_t)g * MS_HOPS + h0) * K + k] &
               ~v.hit[(size_t)g * K + k] & v.pm[((size_t)g * MS_HOPS + h1) * K + k];
      live = any != 0 && len > 0;
    }
    ms_push<TE>(v, 2, B, live, g, node, rb, len);
  }
  if (B.n) ms_flush<TE>(v, 2, B);
}

// After level L: the level's frontier masks are cleared (the buffer is the level after next's): one
// thread per entry, its K words as 16-B stores (one per word of 8 B before round 6: ~4 ms of a heavy-tail
// batch in k_ms_clear, profiles/r6c_heavy_kernel_stats.csv).
template <int K>
__global__ __launch_bounds__(256) void k_ms_clear(MsView v, int cur) {
  const uint64_t n_e = v.ctl->packed[cur] >> MS_EDGE_BITS;
  const uint64_t lim = n_e < v.cap ? n_e : v.cap;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < lim; q += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t* w = v.fr[cur] + ((size_t)v.eg[cur][q] * v.n + v.en[cur][q]) * K;
    if constexpr (K == 1) {
      w[0] = 0;
    } else {
#pragma unroll
      for (int j = 0; j < K / 2; j++) reinterpret_cast<uint4*>(w)[j] = make_uint4(0, 0, 0, 0);
    }
  }
}

// A round's masks start clear: 16-B stores over the whole chip (the runtime's fill kernel moved
// ~1.3 TB/s on these GB-sized arrays: ~2.7 ms of fills per heavy-tail batch, profiles/r6c_heavy_*).
struct MsZero {
  uint4* p[4];
  uint64_t n16[4];
};
__global__ __launch_bounds__(256) void k_ms_zero(MsZero z4) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; r++)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < z4.n16[r]; i += stride) z4.p[r][i] = z;
}

template <int K>
__global__ void k_ms_finish(MsView v, const uint32_t* d_count, uint32_t base, uint8_t* out, uint32_t* err) {
  constexpr uint32_t Q = 64u * K;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ms_round_slots(d_count, base, v.G * Q) || v.ctl->overflow) return;
  const uint32_t qidx = v.qi[i], g = i / Q, b = i % Q;
  out[qidx] = ((v.hit[(size_t)g * K + (b >> 6)] >> (b & 63)) & 1ull) ? KG_IS_MEMBER : KG_NOT_MEMBER;
  if (err) err[qidx] = KG_ERR_NONE;
}

size_t ms_group_bytes(uint32_t n, int K) {
  return (size_t)n * (8 * 4 * K + 4) + (size_t)K * (16 + 2 * MS_HOPS * 8 + 64 * 12);
}

// Pool layout for G groups of K words and level buffers of `cap` entries.  Every array starts on a
// 256-B boundary (k_ms_zero and the mask loads use 16-B accesses).
int ms_layout(GridPool* P, uint32_t n, int K, uint32_t G, uint64_t cap, MsView* v) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t gn = al((size_t)G * n * K * 8);
  const size_t small = al((size_t)G * K * 8);
  const size_t need = 4 * gn + 2 * small + al((size_t)G * 4) + 2 * al((size_t)G * MS_HOPS * K * 8) +
                      3 * al((size_t)G * 64 * K * 4) + al((size_t)G * n * 4) +
                      3 * (al(cap * 8) + 3 * al(cap * 4) + al(MS_TILE_CAP * 4)) + al(sizeof(MsCtl)) + 8192;
  if (need > P->bytes) {
    P->release();
    HIPC(hipMalloc(&P->mem, need));
    P->bytes = need;
  }
  char* p = (char*)P->mem;
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  v->n = n;
  v->G = G;
  v->cap = cap;
  v->vt = (uint64_t*)take(2 * gn);
  v->fr[0] = (uint64_t*)take(gn);
  v->fr[1] = (uint64_t*)take(gn);
  v->hit = (uint64_t*)take((size_t)G * K * 8);
  v->many = (uint64_t*)take((size_t)G * K * 8);
  v->gmany = (uint32_t*)take((size_t)G * 4);
  v->pm = (uint64_t*)take((size_t)G * MS_HOPS * K * 8);
  v->em = (uint64_t*)take((size_t)G * MS_HOPS * K * 8);
  v->qi = (uint32_t*)take((size_t)G * 64 * K * 4);
  v->qd = (uint32_t*)take((size_t)G * 64 * K * 4);
  v->qs = (uint32_t*)take((size_t)G * 64 * K * 4);
  v->stamp = (uint32_t*)take((size_t)G * n * 4);
  for (int b = 0; b < 3; b++) {
    v->ex[b] = (uint64_t*)take(cap * 8);
    v->eg[b] = (uint32_t*)take(cap * 4);
    v->en[b] = (uint32_t*)take(cap * 4);
    v->erb[b] = (uint32_t*)take(cap * 4);
    v->tf[b] = (uint32_t*)take(MS_TILE_CAP * 4);
  }
  v->ctl = (MsCtl*)take(sizeof(MsCtl));
  return 0;
}

// Words per mask for this snapshot: the configured width, halved until one group's masks fit an
// eighth of the budget (0: none fits).
int ms_words(const Snapshot* s) {
  for (int K = s->grid_ms_words; K >= 1; K >>= 1)
    if (ms_group_bytes(s->ds.n_nodes, K) * 8 <= s->grid_ms_bytes) return K;
  return 0;
}

template <int K>
int ms_rounds(Snapshot* s, Workspace* w, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count,
              int global_max_depth, uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs, int phase) {
  constexpr uint32_t Q = 64u * K;
  char* pin = (char*)w->host_buf(65536);
  if (!pin) return set_error(-1, "pinned host buffer");
  uint32_t* hb = (uint32_t*)(pin + 32768);
  const uint32_t n = s->ds.n_nodes;
  const uint32_t g_max =
      (uint32_t)std::max<size_t>(1, std::min<size_t>((1u << 20) / Q, s->grid_ms_bytes / ms_group_bytes(n, K)));
  const uint64_t cap = s->grid_ms_cap ? s->grid_ms_cap : 16ull << 20;  // entries per level buffer
  GridPool* gp = &w->ms;
  MsView v{};
  uint32_t G = g_max;
  v.tg_cap = s->grid_ms_tg_cap;
  if (int rc = ms_layout(gp, n, K, G, std::min<uint64_t>(cap, (uint64_t)G * n + 1024), &v)) return rc;
  const int levels = std::max(0, global_max_depth - 1);  // level L expands hop L (D - 2 >= L)
  // at least 4 workgroups per CU: an MS-BFS level walks whole hub layers (the per-query grid tier's few
  // edges per level prefer grid_wgs = 2; the heavy-tail point lost 12 % at 2, profiles/r4h2_heavy_knobs_ab.jsonl)
  const uint32_t lgrid = (uint32_t)s->n_cu * (uint32_t)std::max(4, s->grid_wgs);
  int64_t count = -1;
  bool resume = phase == 2;
  for (uint32_t done = 0; count < 0 || done < (uint64_t)count;) {
    if (!resume) {
      if (phase == 1) w->grid_reran = false;
      if (phase == 2) w->grid_reran = true;
      v.G = G;
      const size_t gn = (size_t)G * n * K * 8;
      // the round's masks start clear (frontier buffers are cleared level by level, but an
      // overflowed round may leave them dirty)
      // arrays start on 256-B boundaries and are padded to them (ms_layout): whole 16-B words
      const MsZero z4{{(uint4*)v.vt, (uint4*)v.fr[0], (uint4*)v.fr[1], (uint4*)v.stamp},
                      {(2 * gn + 15) / 16, (gn + 15) / 16, (gn + 15) / 16, ((size_t)G * n * 4 + 15) / 16}};
      hipLaunchKernelGGL(k_ms_zero, dim3((uint32_t)s->n_cu * 8), dim3(256), 0, stream, z4);
      HIPC(hipGetLastError());
      HIPC(hipMemsetAsync(v.ctl, 0, sizeof(MsCtl), stream));
      const uint32_t qblocks = (G * Q + 255) / 256;
      hipLaunchKernelGGL(k_ms_init<K>, dim3(qblocks), dim3(256), 0, stream, rq, qlist, d_count, done, v);
      HIPC(hipGetLastError());
      hipLaunchKernelGGL(k_ms_masks<K>, dim3((G * MS_HOPS * K + 255) / 256), dim3(256), 0, stream, v);
      HIPC(hipGetLastError());
      hipLaunchKernelGGL(k_ms_holders<K>, dim3((G * Q + 3) / 4), dim3(256), 0, stream, s->ds, rq, v);
      HIPC(hipGetLastError());
      for (int L = 0; L < levels; L++) {
        const int cur = L & 1;
        HIPC(hipMemsetAsync(&v.ctl->packed[2], 0, 8, stream));
        hipLaunchKernelGGL(k_ms_compact<K>, dim3((uint32_t)s->n_cu * 2), dim3(256), 0, stream, v, L, cur);
        HIPC(hipGetLastError());
        w->lev_mark(stream, false, 2);
        hipLaunchKernelGGL(k_ms_level<K>, dim3(lgrid), dim3(256), 0, stream, s->ds, v, L, 2, cur ^ 1);
        HIPC(hipGetLastError());
        w->lev_mark(stream, true, 2);
        hipLaunchKernelGGL(k_ms_clear<K>, dim3((uint32_t)s->n_cu * 4), dim3(256), 0, stream, v, cur);
        HIPC(hipGetLastError());
        HIPC(hipMemsetAsync(&v.ctl->packed[cur], 0, 8, stream));
      }
      hipLaunchKernelGGL(k_ms_finish<K>, dim3(qblocks), dim3(256), 0, stream, v, d_count, done, out, err);
      HIPC(hipGetLastError());
      HIPC(hipMemcpyAsync(hb, v.ctl, sizeof(MsCtl), hipMemcpyDeviceToHost, stream));
      HIPC(hipMemcpyAsync(hb + sizeof(MsCtl) / 4, d_count, 4, hipMemcpyDeviceToHost, stream));
      if (phase == 1) return 1;
      HIPC(hipStreamSynchronize(stream));
    }
    resume = false;
    MsCtl h{};
    memcpy(&h, hb, sizeof h);
    count = hb[sizeof(MsCtl) / 4];
    const uint32_t cnt = count > done ? (uint32_t)std::min<int64_t>((int64_t)G * Q, count - done) : 0u;
    if (gs) {
      gs->rows += h.logged;
      gs->edges += h.edges;
      gs->ms_eload += h.eload;
      gs->ms_wact += h.wact;
    }
    if (h.overflow) {
      if (G == 1) {  // one group alone overflows the level buffers: the per-query rounds take the list
        if (gs) gs->done -= done;
        return 2;
      }
      G = std::max<uint32_t>(1, std::min(G, (cnt + Q - 1) / Q) / 4);
      continue;
    }
    if (gs) {
      gs->done += cnt;
      gs->logged += h.logged;
    }
    done += cnt;
  }
  return 0;
}

}  // namespace

// Whether the MS-BFS path serves this snapshot's grid tier (kg_snapshot_tune "grid_ms"): one group's
// dense masks must fit an eighth of the pool budget, and the holder index must exist.
bool ms_usable(const Snapshot* s, int global_max_depth) {
  if (!s->grid_ms || !s->ds.hold || !s->ds.hslots || s->ds.n_nodes == 0 || global_max_depth > MS_HOPS) return false;
  return ms_words(s) > 0;
}

// Same protocol as grid_tier (kg_grid.hip): phase 1 enqueues the first round and returns 1, phase 2
// resumes after the batch's synchronisation; a round that overflows a level buffer reruns with a
// quarter of the groups.  Returns 2 when a single group overflows them: the caller runs the rest of
// the list (from the first query not yet answered) through the per-query rounds.
int ms_tier(Snapshot* s, Workspace* w, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count,
            int global_max_depth, uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs, int phase) {
  switch (ms_words(s)) {
    case 16: return ms_rounds<16>(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    case 8: return ms_rounds<8>(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    case 4: return ms_rounds<4>(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    case 2: return ms_rounds<2>(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    case 1: return ms_rounds<1>(s, w, rq, qlist, d_count, global_max_depth, out, err, stream, gs, phase);
    default: return set_error(-2, "MS-BFS masks do not fit");
  }
}

}  // namespace kg
