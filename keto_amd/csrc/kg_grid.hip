// kg_grid.hip -- the grid tier: queries whose BFS outgrew the LDS workgroup tier (thousands to
// millions of expanded nodes).  All of them advance together, level-synchronously, and every level
// is spread edge-balanced over the whole GPU:
//   F                append-only log of (slot, node) frontier entries; level L = F[lvl_b, lvl_e)
//   bitmaps[slot]    visited set of each query (n_nodes bits), cleared from the log afterwards
//   per level        row lengths -> device exclusive scan -> one thread per edge (binary search of
//                    its entry), bit test-and-set, checkDirect probe at discovery, append if the
//                    child will itself be expanded (rest depth >= 2)
// Semantics are those of k_light / k_medium (kg_check.hip): bounded reachability with every node
// probed once at its shallowest depth.  A round that overflows the log is rerun with fewer slots.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kg_bfs.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

struct GridCtl {
  unsigned long long n;  // entries appended to the log
  uint32_t overflow, pad;
  unsigned long long rows, edges, probes;
};

__global__ void k_grid_init(const RQuery* __restrict__ rq, const uint32_t* __restrict__ qlist, uint32_t base,
                            uint32_t cnt, uint64_t* F, uint32_t* slot_q, uint32_t* slot_hit, uint32_t* bitmaps,
                            uint64_t words, GridCtl* ctl) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    ctl->n = cnt;
    ctl->overflow = 0;
  }
  if (i >= cnt) return;
  const uint32_t qi = qlist[base + i];
  const uint32_t root = rq[qi].node;
  slot_q[i] = qi;
  slot_hit[i] = 0;  // the root was already probed (k_resolve)
  bitmaps[(size_t)i * words + (root >> 5)] |= 1u << (root & 31);
  F[i] = ((uint64_t)i << 32) | root;
}

__global__ void k_grid_rowlen(DevSnap s, const RQuery* __restrict__ rq, const uint64_t* __restrict__ F,
                              uint64_t lvl_b, uint64_t n, int level, const uint32_t* slot_q,
                              const uint32_t* slot_hit, uint64_t* lens) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j > n) return;
  uint64_t len = 0;
  if (j < n) {
    const uint64_t f = F[lvl_b + j];
    const uint32_t slot = (uint32_t)(f >> 32), node = (uint32_t)f;
    const int d = rq[slot_q[slot]].depth - level;
    if (d >= 2 && !slot_hit[slot]) len = s.adj_off[node + 1] - s.adj_off[node];
  }
  lens[j] = len;
}

__global__ __launch_bounds__(256) void k_grid_expand(DevSnap s, const RQuery* __restrict__ rq, uint64_t* F,
                                                     uint64_t lvl_b, uint64_t n, const uint64_t* __restrict__ offs,
                                                     uint64_t total, int level, const uint32_t* slot_q,
                                                     uint32_t* slot_hit, uint32_t* bitmaps, uint64_t words,
                                                     uint64_t cap, GridCtl* ctl) {
  unsigned long long probes = 0;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
       e += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = 0, hi = n;  // largest j with offs[j] <= e
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (offs[mid] <= e) lo = mid;
      else hi = mid;
    }
    const uint64_t f = F[lvl_b + lo];
    const uint32_t slot = (uint32_t)(f >> 32), node = (uint32_t)f;
    if (*(volatile uint32_t*)&slot_hit[slot]) continue;
    const RQuery q = rq[slot_q[slot]];
    const int d = q.depth - level;  // >= 2 (rows of shallower nodes have length 0)
    const uint32_t child = s.adj[s.adj_off[node] + (e - offs[lo])];
    if (d - 1 >= 2) {  // child will be expanded: first mark + probe + log it
      const uint32_t bit = 1u << (child & 31);
      if (atomicOr(&bitmaps[(size_t)slot * words + (child >> 5)], bit) & bit) continue;
      probes++;
      if (dset_probe(s, child, q.subj)) atomicExch(&slot_hit[slot], 1u);
      const unsigned long long at = atomicAdd(&ctl->n, 1ull);
      if (at < cap) F[at] = ((uint64_t)slot << 32) | child;
      else ctl->overflow = 1;
    } else {  // last level: probe only
      probes++;
      if (dset_probe(s, child, q.subj)) atomicExch(&slot_hit[slot], 1u);
    }
  }
  if (probes) atomicAdd(&ctl->probes, probes);
}

__global__ void k_grid_finish(const uint32_t* slot_q, const uint32_t* slot_hit, uint32_t cnt, uint8_t* out,
                              uint32_t* err, const uint32_t* overflow) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt || *overflow) return;
  const uint32_t qi = slot_q[i];
  out[qi] = slot_hit[i] ? KG_IS_MEMBER : KG_NOT_MEMBER;
  if (err) err[qi] = KG_ERR_NONE;
}

__global__ void k_grid_clear(const uint64_t* F, uint64_t n, uint32_t* bitmaps, uint64_t words) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t f = F[j];
    bitmaps[(size_t)(f >> 32) * words + ((uint32_t)f >> 5)] = 0u;
  }
}

// Host driver: qlist / count live on the device (count is read back once).
int grid_tier(Snapshot* s, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count, uint8_t* out,
              uint32_t* err, hipStream_t stream, GridStats* gs) {
  uint32_t count = 0;
  HIPC(hipMemcpyAsync(&count, d_count, 4, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  if (count == 0) return 0;
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  const uint64_t words = (nn + 31) / 32 + 1;
  // budget: <= 16 GiB of bitmaps, <= 1024 slots; log capacity >= n_nodes (a single query always fits)
  const uint32_t G0 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (16ull << 30) / (words * 4)));
  const uint64_t cap = std::max<uint64_t>(nn + 1024, 64ull << 20);
  const size_t need = (size_t)G0 * words * 4 + cap * 8 + (cap + 1) * 8 * 2 + (size_t)G0 * 8 + sizeof(GridCtl) + 4096;
  if (need > s->grid_pool_bytes) {
    if (s->grid_pool) HIPC(hipFree(s->grid_pool));
    s->grid_pool = nullptr;
    s->grid_pool_bytes = 0;
    HIPC(hipMalloc(&s->grid_pool, need));
    HIPC(hipMemsetAsync(s->grid_pool, 0, (size_t)G0 * words * 4, stream));  // bitmaps start (and stay) clear
    s->grid_pool_bytes = need;
    s->grid_scan_tmp_bytes = 0;
  }
  char* p = (char*)s->grid_pool;
  uint32_t* bitmaps = (uint32_t*)p;
  p += (size_t)G0 * words * 4;
  uint64_t* F = (uint64_t*)p;
  p += cap * 8;
  uint64_t* lens = (uint64_t*)p;
  p += (cap + 1) * 8;
  uint64_t* offs = (uint64_t*)p;
  p += (cap + 1) * 8;
  uint32_t* slot_q = (uint32_t*)p;
  uint32_t* slot_hit = slot_q + G0;
  p += (size_t)G0 * 8;
  GridCtl* ctl = (GridCtl*)(((uintptr_t)p + 255) & ~uintptr_t(255));
  // scan scratch sized for the largest level (cap entries)
  size_t tmp_bytes = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, lens, offs, cap + 1, stream));
  if (tmp_bytes > s->grid_scan_tmp_bytes) {
    if (s->grid_scan_tmp) HIPC(hipFree(s->grid_scan_tmp));
    HIPC(hipMalloc(&s->grid_scan_tmp, tmp_bytes + 256));
    s->grid_scan_tmp_bytes = tmp_bytes;
  }
  uint32_t G = G0;
  for (uint32_t done = 0; done < count;) {
    const uint32_t cnt = std::min(G, count - done);
    HIPC(hipMemsetAsync(&ctl->rows, 0, 3 * sizeof(unsigned long long), stream));
    hipLaunchKernelGGL(k_grid_init, dim3((cnt + 255) / 256), dim3(256), 0, stream, rq, qlist, done, cnt, F, slot_q,
                       slot_hit, bitmaps, words, ctl);
    HIPC(hipGetLastError());
    uint64_t lvl_b = 0, lvl_e = cnt;
    GridCtl h{};
    for (int level = 0; lvl_b < lvl_e; level++) {
      const uint64_t n = lvl_e - lvl_b;
      hipLaunchKernelGGL(k_grid_rowlen, dim3((uint32_t)((n + 256) / 256)), dim3(256), 0, stream, s->ds, rq, F, lvl_b,
                         n, level, slot_q, slot_hit, lens);
      HIPC(hipGetLastError());
      size_t tb = s->grid_scan_tmp_bytes;
      HIPC(hipcub::DeviceScan::ExclusiveSum(s->grid_scan_tmp, tb, lens, offs, n + 1, stream));
      uint64_t total = 0;
      HIPC(hipMemcpyAsync(&total, offs + n, 8, hipMemcpyDeviceToHost, stream));
      HIPC(hipStreamSynchronize(stream));
      if (total == 0) break;
      if (gs) {
        gs->rows += n;
        gs->edges += total;
      }
      const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)s->n_cu * 16, (total + 255) / 256);
      hipLaunchKernelGGL(k_grid_expand, dim3(grid), dim3(256), 0, stream, s->ds, rq, F, lvl_b, n, offs, total, level,
                         slot_q, slot_hit, bitmaps, words, cap, ctl);
      HIPC(hipGetLastError());
      HIPC(hipMemcpyAsync(&h, ctl, sizeof h, hipMemcpyDeviceToHost, stream));
      HIPC(hipStreamSynchronize(stream));
      if (h.overflow) break;
      lvl_b = lvl_e;
      lvl_e = std::min<uint64_t>(h.n, cap);
    }
    HIPC(hipMemcpyAsync(&h, ctl, sizeof h, hipMemcpyDeviceToHost, stream));
    HIPC(hipStreamSynchronize(stream));
    hipLaunchKernelGGL(k_grid_finish, dim3((cnt + 255) / 256), dim3(256), 0, stream, slot_q, slot_hit, cnt, out, err,
                       &ctl->overflow);
    HIPC(hipGetLastError());
    if (h.overflow) {
      // some set bits have no log entry: clear the round's bitmaps wholesale, retry with fewer slots
      HIPC(hipMemsetAsync(bitmaps, 0, (size_t)cnt * words * 4, stream));
      if (G == 1) return set_error(KG_ERR_RESOURCE_CODE, "grid tier log overflow");
      G = std::max<uint32_t>(1, G / 4);
      continue;
    }
    const uint64_t logged = std::min<uint64_t>(h.n, cap);
    hipLaunchKernelGGL(k_grid_clear, dim3((uint32_t)std::min<uint64_t>(4096, (logged + 255) / 256)), dim3(256), 0,
                       stream, F, logged, bitmaps, words);
    HIPC(hipGetLastError());
    if (gs) {
      gs->probes += h.probes;
      gs->done += cnt;
      gs->logged += logged;
    }
    done += cnt;
  }
  return 0;
}

}  // namespace kg
