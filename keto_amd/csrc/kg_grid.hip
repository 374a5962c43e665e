// kg_grid.hip -- the grid tier: queries whose BFS outgrew the LDS workgroup tier (thousands to
// millions of expanded nodes).  All of them advance together, level-synchronously, and every level
// is spread edge-balanced over the whole GPU:
//   F/RB/lens        append-only log of (slot, node, set-row start, set-row length) entries;
//                    level L = log[lvl_b, lvl_e)
//   bitmaps[slot]    visited set of each query (n_nodes bits), cleared from the log afterwards
//   per level        device inclusive scan of the row lengths -> one thread per edge (LDS binary
//                    search of its entry within a 2048-edge tile), checkDirect probe at discovery;
//                    children that will themselves be expanded (rest depth >= 2, non-empty set
//                    row, read inline from adjx) are bit-test-and-set and appended wave-aggregated
// Semantics are those of k_light / k_medium (kg_check.hip): bounded reachability with every node
// probed once at its shallowest depth.  A round that overflows the log is rerun with fewer slots.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kg_bfs.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

struct GridCtl {
  unsigned long long n;  // entries appended to the log
  uint32_t overflow, pad;
  unsigned long long lvl_b, lvl_e, total;  // current level = log[lvl_b, lvl_e), its edge count
  unsigned long long edges;                // edges over all levels (stats)
  unsigned long long probes8[8][16];  // per-XCD shards (one 128-B line each)
};

// Visited sets of all slots in ONE open-addressing table of 64-bit keys
//   epoch (16) | slot (16) | node (32)
// Entries of older epochs (earlier rounds / batches) count as empty, so the table is never
// cleared between rounds; it is zeroed once per 65535 rounds.  Within a round an entry never
// changes once written, so a (possibly stale) plain load that shows this round's epoch is final.
constexpr int GH_PROBES = 128;
__device__ __forceinline__ int gh_insert(uint64_t* H, uint64_t mask, uint64_t key) {
  const uint64_t ep = key >> 48;
  uint64_t h = mix64(key & 0xFFFFFFFFFFFFull) & mask;
  for (int p = 0; p < GH_PROBES; p++) {
    uint64_t cur = H[h];
    for (;;) {
      if (cur == key) return 0;      // already visited
      if ((cur >> 48) == ep) break;  // another key of this round: next slot
      const uint64_t old = atomicCAS((unsigned long long*)&H[h], (unsigned long long)cur, (unsigned long long)key);
      if (old == cur) return 1;      // inserted
      cur = old;
    }
    h = (h + 1) & mask;
  }
  return -1;  // probe bound: the round is rerun with fewer slots
}

// Log entry j: F[j] = slot << 32 | node, RB[j] = first adjx index of node's set row, lens[j] = its
// length.  Only nodes with a non-empty set row are marked and logged; leaves are probed wherever
// they are reached (a probe does not depend on the depth it is made at, so this is exact).
__global__ void k_grid_init(DevSnap s, const RQuery* __restrict__ rq, const uint32_t* __restrict__ qlist,
                            uint32_t base, uint32_t cnt, uint64_t* F, uint32_t* RB, uint64_t* lens, uint32_t* slot_q,
                            uint2* slot_info, uint32_t* slot_hit, uint64_t* H, uint64_t mask, uint64_t epoch,
                            GridCtl* ctl) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    ctl->n = cnt;
    ctl->overflow = 0;
    ctl->lvl_b = ctl->lvl_e = ctl->total = ctl->edges = 0;
  }
  if (i < 8 * 16) (&ctl->probes8[0][0])[i] = 0;
  if (i >= cnt) return;
  const uint32_t qi = qlist[base + i];
  const RQuery q = rq[qi];
  const uint32_t root = q.node;
  slot_q[i] = qi;
  slot_info[i] = make_uint2(q.subj, (uint32_t)q.depth);
  slot_hit[i] = 0;  // the root was already probed (k_resolve)
  if (gh_insert(H, mask, (epoch << 48) | ((uint64_t)i << 32) | root) < 0) ctl->overflow = 1;
  F[i] = ((uint64_t)i << 32) | root;
  RB[i] = (uint32_t)s.adj_off[root];
  lens[i] = s.adj_off[root + 1] - s.adj_off[root];
}

// smallest j in [lo, hi) with incl[j] > e (incl = inclusive prefix sums of the level's row lengths)
__device__ __forceinline__ uint64_t first_above(const uint64_t* incl, uint64_t lo, uint64_t hi, uint64_t e) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (incl[mid] > e) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// ---- device-side level loop: no host round trip per level.  The next level is the entries
// logged by the previous one: [previous lvl_e, min(n, cap)).  k_grid_scan_reduce computes those
// bounds from GridCtl, k_grid_scan_top publishes them (lvl_b, lvl_e, total) for the rest of the
// level.
__device__ __forceinline__ void next_level(const GridCtl* ctl, uint64_t cap, uint64_t& lb, uint64_t& le) {
  lb = ctl->lvl_e;
  le = ctl->n < cap ? ctl->n : cap;
}

// Inclusive scan of lens[lvl_b, lvl_e) -> incl[0, n) in three fixed-size launches (the level size
// lives on the device): per-block chunk sums, one-block scan of the sums, per-block rescan.  The
// rescan also records, for every GT-edge tile of the level, the entry holding its first edge
// (tile_first), so k_grid_expand never binary-searches HBM.
constexpr uint32_t SCAN_BLOCKS = 1024;
constexpr uint32_t GT = 2048;               // edges per k_grid_expand tile
constexpr uint64_t TILE_CAP = 1ull << 22;   // tiles with a tile_first entry (beyond: HBM search)

__device__ __forceinline__ uint64_t block_sum64(uint64_t v, uint64_t* red) {
  for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const uint64_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void k_grid_scan_reduce(const uint64_t* __restrict__ lens, const GridCtl* ctl,
                                                          uint64_t* bsum, uint64_t cap) {
  __shared__ uint64_t red[4];
  uint64_t lb, le;
  next_level(ctl, cap, lb, le);
  const uint64_t n = le - lb;
  const uint64_t chunk = (n + SCAN_BLOCKS - 1) / SCAN_BLOCKS;
  const uint64_t b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  uint64_t v = 0;
  for (uint64_t j = b0 + threadIdx.x; j < b1; j += 256) v += lens[lb + j];
  v = block_sum64(v, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = v;
}

__global__ __launch_bounds__(SCAN_BLOCKS) void k_grid_scan_top(uint64_t* bsum, GridCtl* ctl, uint64_t cap) {
  __shared__ uint64_t wsum[SCAN_BLOCKS / 64];
  uint64_t lb, le;
  next_level(ctl, cap, lb, le);
  __syncthreads();  // every thread has read the previous bounds before thread 0 publishes
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t x = bsum[threadIdx.x];
  uint64_t v = x;
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = shfl_up64(v, off);
    if (lane >= off) v += y;
  }
  if (lane == 63) wsum[wave] = v;
  __syncthreads();
  uint64_t before = 0, tot = 0;
  for (int w = 0; w < (int)(SCAN_BLOCKS / 64); w++) {
    if (w < wave) before += wsum[w];
    tot += wsum[w];
  }
  bsum[threadIdx.x] = before + v - x;  // exclusive block offsets
  if (threadIdx.x == 0) {
    ctl->lvl_b = lb;
    ctl->lvl_e = le;
    ctl->total = tot;
    ctl->edges += tot;
  }
}

__global__ __launch_bounds__(256) void k_grid_scan_apply(const uint64_t* __restrict__ lens, uint64_t* incl,
                                                         const uint64_t* __restrict__ boff, const GridCtl* ctl,
                                                         uint32_t* tile_first) {
  __shared__ uint64_t wsum[4];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t lb = ctl->lvl_b, n = ctl->lvl_e - lb;
  const uint64_t chunk = (n + SCAN_BLOCKS - 1) / SCAN_BLOCKS;
  const uint64_t b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  uint64_t carry = boff[blockIdx.x];
  for (uint64_t t = b0; t < b1; t += 256) {
    const uint64_t j = t + threadIdx.x;
    const uint64_t x = j < b1 ? lens[lb + j] : 0;
    uint64_t v = x;
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = shfl_up64(v, off);
      if (lane >= off) v += y;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    uint64_t before = carry;
    for (int w = 0; w < wave; w++) before += wsum[w];
    if (j < b1) {
      const uint64_t hi = before + v, lo = hi - x;  // entry j holds edges [lo, hi)
      incl[j] = hi;
      // tiles whose first edge lies in [lo, hi): exactly one entry writes each tile
      for (uint64_t t = (lo + GT - 1) / GT; t * GT < hi && t < TILE_CAP; t++) tile_first[t] = (uint32_t)j;
    }
    carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

// One thread per edge of the level, in tiles of GT edges per workgroup: the tile's entries (edge
// start, slot, adjx row start) are staged in LDS, so each edge finds its entry with an LDS binary
// search; per-slot (subject, depth) come from one 8-B slot record.
__global__ __launch_bounds__(256) void k_grid_expand(DevSnap s, uint64_t* F, uint32_t* RB, uint64_t* lens,
                                                     const uint64_t* __restrict__ incl,
                                                     const uint32_t* __restrict__ tile_first, int level,
                                                     const uint2* __restrict__ slot_info, uint32_t* slot_hit,
                                                     uint64_t* H, uint64_t mask, uint64_t epoch, uint64_t cap,
                                                     GridCtl* ctl) {
  __shared__ uint64_t s_beg[GT + 2];
  __shared__ uint32_t s_slot[GT + 2], s_rb[GT + 2];
  __shared__ uint64_t s_j0, s_cnt;
  __shared__ uint32_t s_wcnt[4];
  __shared__ unsigned long long s_base;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const uint64_t lvl_b = ctl->lvl_b, n = ctl->lvl_e - lvl_b, total = ctl->total;
  uint32_t probes = 0;
  for (uint64_t t0 = (uint64_t)blockIdx.x * GT; t0 < total; t0 += (uint64_t)gridDim.x * GT) {
    const uint64_t t1 = t0 + GT < total ? t0 + GT : total;
    if (threadIdx.x == 0) {
      const uint64_t t = t0 / GT;
      uint64_t j0, jl;
      if (t + 1 < TILE_CAP) {
        j0 = tile_first[t];
        jl = t1 < total ? tile_first[t + 1] : n - 1;  // an entry at or after the tile's last edge
      } else {
        j0 = first_above(incl, 0, n, t0);
        jl = first_above(incl, j0, n, t1 - 1);
      }
      s_j0 = j0;
      s_cnt = jl - j0 + 1;
    }
    __syncthreads();
    const uint64_t j0 = s_j0, cnt = s_cnt;
    const bool use_lds = cnt <= GT + 1;
    if (use_lds)
      for (uint32_t i = threadIdx.x; i < cnt; i += 256) {
        s_beg[i] = j0 + i == 0 ? 0 : incl[j0 + i - 1];
        s_slot[i] = (uint32_t)(F[lvl_b + j0 + i] >> 32);
        s_rb[i] = RB[lvl_b + j0 + i];
      }
    __syncthreads();
    for (uint32_t k = 0; k < GT; k += 256) {
      const uint64_t e = t0 + k + threadIdx.x;
      bool act = e < t1, keep = false;
      uint32_t slot = 0, child = 0, cb = 0, cl = 0;
      if (act) {
        uint64_t beg;
        uint32_t rb;
        if (use_lds) {
          uint32_t lo = 0, hi = (uint32_t)cnt;  // largest i < cnt with s_beg[i] <= e
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_beg[mid] <= e) lo = mid;
            else hi = mid;
          }
          beg = s_beg[lo];
          slot = s_slot[lo];
          rb = s_rb[lo];
        } else {
          const uint64_t j = first_above(incl, j0, j0 + cnt, e);
          beg = incl[j] - lens[lvl_b + j];
          slot = (uint32_t)(F[lvl_b + j] >> 32);
          rb = RB[lvl_b + j];
        }
        if (slot_hit[slot]) {
          act = false;
        } else {
          const uint2 si = slot_info[slot];  // (tagged subject, rest depth of the root)
          const AdjX x = s.adjx[rb + (e - beg)];
          child = x.node;
          cb = x.begin;
          cl = x.len;
          keep = cl > 0 && (int)si.y - level - 1 >= 2;  // child will itself be expanded
          if (keep) {
            const int ins = gh_insert(H, mask, (epoch << 48) | ((uint64_t)slot << 32) | child);
            if (ins < 0) ctl->overflow = 1;
            if (ins == 0) act = false;
          }
          if (act && sig_maybe(x.sig, subj_sig(si.x))) {  // the signature rules out most misses
            probes++;
            if (dset_probe(s, child, si.x)) atomicExch(&slot_hit[slot], 1u);
          }
        }
      }
      // workgroup-aggregated append to the log: one atomic per 256 edges
      const bool app = act && keep;
      const uint64_t m = __ballot(app);
      if (lane == 0) s_wcnt[wave] = __popcll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint32_t t = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
        s_base = t ? atomicAdd(&ctl->n, (unsigned long long)t) : 0ull;
      }
      __syncthreads();
      if (app) {
        unsigned long long at = s_base + lanes_below(m);
        for (int w = 0; w < wave; w++) at += s_wcnt[w];
        if (at < cap) {
          F[at] = ((uint64_t)slot << 32) | child;
          RB[at] = cb;
          lens[at] = cl;
        } else {
          ctl->overflow = 1;
        }
      }
      __syncthreads();
    }
  }
  for (int off = 32; off; off >>= 1) probes += __shfl_xor(probes, off, 64);
  if (lane == 0 && probes) atomicAdd(&ctl->probes8[blockIdx.x & 7][wave], (unsigned long long)probes);
}

__global__ void k_grid_finish(const uint32_t* slot_q, const uint32_t* slot_hit, uint32_t cnt, uint8_t* out,
                              uint32_t* err, const uint32_t* overflow) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt || *overflow) return;
  const uint32_t qi = slot_q[i];
  out[qi] = slot_hit[i] ? KG_IS_MEMBER : KG_NOT_MEMBER;
  if (err) err[qi] = KG_ERR_NONE;
}

// Host driver: qlist / count live on the device (count is read back once).
int grid_tier(Snapshot* s, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count, int global_max_depth,
              uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs) {
  uint32_t* hb = (uint32_t*)s->host_buf(sizeof(GridCtl) + 64);
  if (!hb) return set_error(-1, "pinned host buffer");
  HIPC(hipMemcpyAsync(hb, d_count, 4, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  const uint32_t count = hb[0];
  if (count == 0) return 0;
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  // log capacity >= n_nodes (one slot alone always fits); hash >= 2x the log (load <= 0.5)
  const uint64_t cap = std::max<uint64_t>(nn + 1024, 64ull << 20);
  uint64_t hcap = 1;
  while (hcap < 2 * cap) hcap <<= 1;
  const uint32_t G0 = 0xFFFF;  // slot field is 16 bits
  const size_t need = hcap * 8 + cap * (8 + 4 + 8 + 8) + (size_t)G0 * 16 + TILE_CAP * 4 + sizeof(GridCtl) +
                      SCAN_BLOCKS * 8 + 4096;
  if (need > s->grid_pool_bytes) {
    if (s->grid_pool) HIPC(hipFree(s->grid_pool));
    s->grid_pool = nullptr;
    s->grid_pool_bytes = 0;
    HIPC(hipMalloc(&s->grid_pool, need));
    HIPC(hipMemsetAsync(s->grid_pool, 0, hcap * 8, stream));  // epoch 0 = empty
    s->grid_pool_bytes = need;
    s->grid_epoch = 0;
  }
  char* p = (char*)s->grid_pool;
  uint64_t* H = (uint64_t*)p;
  p += hcap * 8;
  uint64_t* F = (uint64_t*)p;
  p += cap * 8;
  uint64_t* lens = (uint64_t*)p;
  p += cap * 8;
  uint64_t* incl = (uint64_t*)p;
  p += cap * 8;
  uint32_t* RB = (uint32_t*)p;
  p += cap * 4;
  uint32_t* tile_first = (uint32_t*)p;
  p += TILE_CAP * 4;
  uint2* slot_info = (uint2*)p;
  p += (size_t)G0 * 8;
  uint32_t* slot_q = (uint32_t*)p;
  uint32_t* slot_hit = slot_q + G0;
  p += (size_t)G0 * 8;
  GridCtl* ctl = (GridCtl*)(((uintptr_t)p + 255) & ~uintptr_t(255));
  uint64_t* bsum = (uint64_t*)(((uintptr_t)(ctl + 1) + 255) & ~uintptr_t(255));  // SCAN_BLOCKS
  uint32_t G = G0;
  for (uint32_t done = 0; done < count;) {
    const uint32_t cnt = std::min(G, count - done);
    if (++s->grid_epoch == 0x10000) {  // epoch wrap: the table is zeroed once per 65535 rounds
      HIPC(hipMemsetAsync(H, 0, hcap * 8, stream));
      s->grid_epoch = 1;
    }
    const uint64_t epoch = s->grid_epoch;
    hipLaunchKernelGGL(k_grid_init, dim3((cnt + 255) / 256), dim3(256), 0, stream, s->ds, rq, qlist, done, cnt, F,
                       RB, lens, slot_q, slot_info, slot_hit, H, hcap - 1, epoch, ctl);
    HIPC(hipGetLastError());
    // Levels run back to back on the device (sizes never come back to the host); the host looks
    // at the log once per LEVELS_PER_SYNC levels to stop early on an empty level or an overflow.
    // Level k expands nodes at rest depth D-k >= 2, so at most global_max_depth-1 levels exist.
    constexpr int LEVELS_PER_SYNC = 16;
    const int max_levels = std::max(1, global_max_depth - 1);
    GridCtl h{};
    for (int level = 0; level < max_levels;) {
      const int stop = std::min(max_levels, level + LEVELS_PER_SYNC);
      for (; level < stop; level++) {
        hipLaunchKernelGGL(k_grid_scan_reduce, dim3(SCAN_BLOCKS), dim3(256), 0, stream, lens, ctl, bsum, cap);
        hipLaunchKernelGGL(k_grid_scan_top, dim3(1), dim3(SCAN_BLOCKS), 0, stream, bsum, ctl, cap);
        hipLaunchKernelGGL(k_grid_scan_apply, dim3(SCAN_BLOCKS), dim3(256), 0, stream, lens, incl, bsum, ctl,
                           tile_first);
        hipLaunchKernelGGL(k_grid_expand, dim3((uint32_t)s->n_cu * 8), dim3(256), 0, stream, s->ds, F, RB, lens,
                           incl, tile_first, level, slot_info, slot_hit, H, hcap - 1, epoch, cap, ctl);
        HIPC(hipGetLastError());
      }
      HIPC(hipMemcpyAsync(hb, ctl, sizeof h, hipMemcpyDeviceToHost, stream));
      HIPC(hipStreamSynchronize(stream));
      memcpy(&h, hb, sizeof h);
      if (h.overflow || std::min<uint64_t>(h.n, cap) == h.lvl_e) break;  // next level empty
    }
    if (gs) {
      gs->rows += std::min<uint64_t>(h.n, cap);
      gs->edges += h.edges;
    }
    hipLaunchKernelGGL(k_grid_finish, dim3((cnt + 255) / 256), dim3(256), 0, stream, slot_q, slot_hit, cnt, out, err,
                       &ctl->overflow);
    HIPC(hipGetLastError());
    if (h.overflow) {  // log or probe bound exceeded: rerun these queries with fewer slots
      if (G == 1) return set_error(KG_ERR_RESOURCE_CODE, "grid tier capacity exceeded");
      G = std::max<uint32_t>(1, std::min(G, cnt) / 4);
      continue;
    }
    if (gs) {
      for (int x = 0; x < 8; x++)
        for (int k = 0; k < 16; k++) gs->probes += h.probes8[x][k];
      gs->done += cnt;
      gs->logged += std::min<uint64_t>(h.n, cap);
    }
    done += cnt;
  }
  return 0;
}

}  // namespace kg
