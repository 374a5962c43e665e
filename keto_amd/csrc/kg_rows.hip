// kg_rows.hip -- GetRelationTuples by (namespace, object, relation) on the device snapshot
// (internal/relationtuple/definitions.go:27-41 with the three set; rows in shard_id order,
// internal/persistence/sql/relationtuples.go:260-270): the rows a CheckRelationTuple tree walk
// reads (keto_amd/explain.py).  Raw rows only (row_off / row_subj): a materialised union node's
// merged check rows are not tuples of its relation.
#include <hip/hip_runtime.h>

#include <vector>

#include "kg_bfs.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

__global__ void k_rows_find(DevSnap s, const kg_set* __restrict__ keys, uint32_t n, uint32_t* node, uint64_t* len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const kg_set k = keys[i];
  const uint32_t v = nmap_find(s, k.sns, k.srel, k.sobj);
  node[i] = v;
  len[i] = v == NONE ? 0 : s.row_off[v + 1] - s.row_off[v];
}

// one wave per key: its row decoded into kg_tuple records
__global__ void k_rows_fill(DevSnap s, const uint32_t* __restrict__ node, const uint64_t* __restrict__ off, uint32_t n,
                            kg_tuple* out) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (w >= n) return;
  const uint32_t v = node[w];
  if (v == NONE) return;
  const uint64_t b = s.row_off[v], o = off[w], len = off[w + 1] - o;
  const uint32_t ns = s.nd_ns[v], obj = s.nd_obj[v], rel = s.nd_rel[v];
  for (uint64_t j = lane; j < len; j += 64) {
    const uint32_t x = s.row_subj[b + j];
    kg_tuple t{ns, obj, rel, KG_SUBJECT_ID, x, 0};
    if (x & SET_BIT) {
      const uint32_t c = x & ~SET_BIT;
      t.sns = s.nd_ns[c];
      t.sobj = s.nd_obj[c];
      t.srel = s.nd_rel[c];
    }
    out[o + j] = t;
  }
}

int64_t Snapshot::rows_of(const kg_set* keys, size_t n, uint64_t* offsets, kg_tuple* out, uint64_t cap) {
  HIPC(hipSetDevice(device));
  offsets[0] = 0;
  if (!n) return 0;
  kg_set* d_keys = nullptr;
  uint32_t* d_node = nullptr;
  uint64_t* d_len = nullptr;
  kg_tuple* d_out = nullptr;
  int64_t rc = -1;
  std::vector<uint64_t> len(n);
  auto done = [&]() {
    hipFree(d_keys);
    hipFree(d_node);
    hipFree(d_len);
    hipFree(d_out);
    return rc;
  };
  if (hipMalloc(&d_keys, n * sizeof(kg_set)) != hipSuccess || hipMalloc(&d_node, n * 4) != hipSuccess ||
      hipMalloc(&d_len, (n + 1) * 8) != hipSuccess) {
    set_error(-1, "rows: device allocation failed");
    return done();
  }
  if (hipMemcpyAsync(d_keys, keys, n * sizeof(kg_set), hipMemcpyHostToDevice, stream) != hipSuccess) return done();
  hipLaunchKernelGGL(k_rows_find, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, ds, d_keys, (uint32_t)n,
                     d_node, d_len);
  if (hipMemcpyAsync(len.data(), d_len, n * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess) {
    set_error(-1, "rows: lookup failed");
    return done();
  }
  for (size_t i = 0; i < n; i++) offsets[i + 1] = offsets[i] + len[i];
  const uint64_t total = offsets[n];
  rc = (int64_t)total;
  if (!out || !total) return done();
  if (cap < total) {
    rc = set_error(-3, "rows buffer too small (%llu < %llu)", (unsigned long long)cap, (unsigned long long)total);
    return done();
  }
  rc = -1;
  if (hipMalloc(&d_out, total * sizeof(kg_tuple)) != hipSuccess) {
    set_error(-1, "rows: device allocation failed");
    return done();
  }
  // d_len now holds the offsets
  if (hipMemcpyAsync(d_len, offsets, (n + 1) * 8, hipMemcpyHostToDevice, stream) != hipSuccess) return done();
  hipLaunchKernelGGL(k_rows_fill, dim3((uint32_t)((n * 64 + 255) / 256)), dim3(256), 0, stream, ds, d_node, d_len,
                     (uint32_t)n, d_out);
  if (hipMemcpyAsync(out, d_out, total * sizeof(kg_tuple), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess) {
    set_error(-1, "rows: copy failed");
    return done();
  }
  rc = (int64_t)total;
  return done();
}

}  // namespace kg
