// kg_delta.hip -- incremental snapshot refresh: a new snapshot = base rows + inserted - deleted.
//
// The reference persists every TransactRelationTuples in SQL (internal/persistence/sql/
// relationtuples.go:260-270: inserts, then deletes of every row equal to a tuple, :164-185) and the
// next check reads the new rows.  A full kg_snapshot_create after each transaction re-interns and
// re-sorts every row on the host (seconds at 10 M tuples); here only the delta touches the host:
//   host    intern the delta's tuples into the base's node map (handed on, not copied; new
//           (ns, obj, rel) triples get the next node ids), sort inserts by (node, order key) and
//           deletes by (node, subject)
//   device  per node: new row length (old - deleted + inserted) -> scan -> rows of untouched nodes
//           shifted by one copy kernel, touched nodes merged by order key (one thread each);
//           set-adjacency recounted and filled from the new rows; then the same derived structures
//           as every build (purity closure, rewrite materialisation, formula plans, dset, node
//           map, adjx, reverse index, holders)
// Order keys (kg_snapshot_create_ordered / kg_snapshot_apply: the persister's shard ids) keep every
// node's row in shard order, so expand trees and the DFS-order oracle see the rows the SQL
// persister would return.  Without keys, inserted rows go to the end of their node's row.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <numeric>
#include <vector>

#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

struct DeltaDev {
  const uint32_t* ins_node;  // sorted by (node, key); ins_off[v .. v+1) via binary search
  const uint32_t* ins_subj;
  const uint64_t* ins_key;
  uint32_t n_ins;
  const uint32_t* del_node;  // sorted by (node, subject)
  const uint32_t* del_subj;
  uint32_t n_del;
};

__device__ __forceinline__ uint32_t lower_node(const uint32_t* a, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// A node's deletes del_subj[db, de) are sorted by subject: binary search (a delete_all of a hub's
// rows can leave thousands on one node, and every old entry of its row asks)
__device__ __forceinline__ bool is_deleted(const DeltaDev& D, uint32_t db, uint32_t de, uint32_t subj) {
  uint32_t lo = db, hi = de;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (D.del_subj[mid] < subj) lo = mid + 1;
    else hi = mid;
  }
  return lo < de && D.del_subj[lo] == subj;
}

// Everything below is edge-parallel: a node-per-thread loop over its row leaves the whole kernel
// waiting for the longest row (a 10^5-subject hub took 40-60 ms per pass at 10 M tuples).

// Per node: touched by the delta?  Untouched nodes keep their row length (new nodes: their inserts).
__global__ void k_delta_len(const uint64_t* __restrict__ row_off, uint32_t n0, uint32_t n1, DeltaDev D,
                            uint64_t* __restrict__ newlen, uint8_t* __restrict__ touched) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n1) return;
  const uint32_t ib = lower_node(D.ins_node, D.n_ins, v), ie = lower_node(D.ins_node, D.n_ins, v + 1);
  const uint32_t db = lower_node(D.del_node, D.n_del, v), de = lower_node(D.del_node, D.n_del, v + 1);
  const bool t = ie > ib || de > db;
  touched[v] = t ? 1 : 0;
  if (!t) newlen[v] = v < n0 ? row_off[v + 1] - row_off[v] : 0u;  // touched nodes: k_delta_tlen
}

// Old row lengths of the touched nodes (scanned into their flat offsets) and node -> touched index.
__global__ void k_delta_tprep(const uint64_t* __restrict__ row_off, uint32_t n0, const uint32_t* __restrict__ tl,
                              uint32_t n_t, uint64_t* __restrict__ tlen, uint32_t* __restrict__ tslot) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_t) return;
  const uint32_t v = tl[t];
  tlen[t] = v < n0 ? row_off[v + 1] - row_off[v] : 0u;
  tslot[v] = t;
}

// Touched nodes' old entries, flattened (toff = scan of their old row lengths): kept or deleted.
__global__ void k_delta_keep(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ row_subj, uint32_t n0,
                             DeltaDev D, const uint32_t* __restrict__ tl, uint32_t n_t,
                             const uint64_t* __restrict__ toff, uint32_t* __restrict__ keep) {
  const uint64_t F = toff[n_t];
  for (uint64_t f = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; f < F; f += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t t = csr_owner(toff, n_t, f);
    const uint32_t v = tl[t];
    const uint32_t sub = row_subj[row_off[v] + (f - toff[t])];
    const uint32_t db = lower_node(D.del_node, D.n_del, v), de = lower_node(D.del_node, D.n_del, v + 1);
    keep[f] = (de > db && is_deleted(D, db, de, sub)) ? 0u : 1u;
  }
}

// Touched nodes' new lengths: kept old entries (kr = exclusive scan of keep) + their inserts.
__global__ void k_delta_tlen(const uint32_t* __restrict__ tl, uint32_t n_t, const uint64_t* __restrict__ toff,
                             const uint64_t* __restrict__ kr, DeltaDev D, uint64_t* __restrict__ newlen) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_t) return;
  const uint32_t v = tl[t];
  const uint32_t ib = lower_node(D.ins_node, D.n_ins, v), ie = lower_node(D.ins_node, D.n_ins, v + 1);
  newlen[v] = (kr[toff[t + 1]] - kr[toff[t]]) + (ie - ib);
}

// Rows of untouched nodes: one thread per old entry, shifted by the node's offset change.
__global__ void k_delta_copy(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ row_subj,
                             const uint64_t* __restrict__ row_key, uint32_t n0, uint64_t n_rows,
                             const uint64_t* __restrict__ new_off, const uint8_t* __restrict__ touched,
                             uint32_t* __restrict__ new_subj, uint64_t* __restrict__ new_key) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_rows; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = csr_owner(row_off, n0, i);
    if (touched[v]) continue;
    const uint64_t at = new_off[v] + (i - row_off[v]);
    new_subj[at] = row_subj[i];
    if (new_key) new_key[at] = row_key ? row_key[i] : 0ull;
  }
}

// Number of keys in the sorted run a[b, e) that are < k (strict) or <= k.
__device__ __forceinline__ uint32_t count_below(const uint64_t* a, uint32_t b, uint32_t e, uint64_t k, bool le) {
  uint32_t lo = b, hi = e;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (le ? a[mid] <= k : a[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo - b;
}

// Touched nodes' kept old entries: position = kept entries before it + inserts with a smaller key.
__global__ void k_delta_scatter_old(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ row_subj,
                                    const uint64_t* __restrict__ row_key, DeltaDev D, const uint32_t* __restrict__ tl,
                                    uint32_t n_t, const uint64_t* __restrict__ toff, const uint32_t* __restrict__ keep,
                                    const uint64_t* __restrict__ kr, const uint64_t* __restrict__ new_off,
                                    uint32_t* __restrict__ new_subj, uint64_t* __restrict__ new_key) {
  const uint64_t F = toff[n_t];
  for (uint64_t f = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; f < F; f += (uint64_t)gridDim.x * blockDim.x) {
    if (!keep[f]) continue;
    const uint32_t t = csr_owner(toff, n_t, f);
    const uint32_t v = tl[t];
    const uint64_t i = row_off[v] + (f - toff[t]);
    const uint64_t key = row_key ? row_key[i] : 0ull;
    const uint32_t ib = lower_node(D.ins_node, D.n_ins, v), ie = lower_node(D.ins_node, D.n_ins, v + 1);
    const uint64_t at = new_off[v] + (kr[f] - kr[toff[t]]) + count_below(D.ins_key, ib, ie, key, false);
    new_subj[at] = row_subj[i];
    if (new_key) new_key[at] = key;
  }
}

// Inserts: position = inserts of the node before it + kept old entries with a key <= its key (the
// old row is in key order; without keys every old key is 0 and inserts carry UINT64_MAX: they go last).
__global__ void k_delta_scatter_ins(const uint64_t* __restrict__ row_off, const uint64_t* __restrict__ row_key,
                                    uint32_t n0, DeltaDev D, const uint32_t* __restrict__ tslot,
                                    const uint64_t* __restrict__ toff, const uint64_t* __restrict__ kr,
                                    const uint64_t* __restrict__ new_off, uint32_t* __restrict__ new_subj,
                                    uint64_t* __restrict__ new_key) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D.n_ins) return;
  const uint32_t v = D.ins_node[j];
  const uint32_t ib = lower_node(D.ins_node, D.n_ins, v);
  uint64_t kept_before = 0;
  if (v < n0) {
    const uint64_t b = row_off[v], e = row_off[v + 1];
    uint64_t lo = b, hi = e;  // old entries with key <= the insert's key
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((row_key ? row_key[mid] : 0ull) <= D.ins_key[j]) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t t = tslot[v];  // v's index in the touched list
    kept_before = kr[toff[t] + (lo - b)] - kr[toff[t]];
  }
  const uint64_t at = new_off[v] + kept_before + (j - ib);
  new_subj[at] = D.ins_subj[j];
  if (new_key) new_key[at] = D.ins_key[j];
}

// Set-adjacency from the rows (subject sets except "..." ones, engine.go:123-126): a flag per row
// entry, scanned into positions.
__global__ void k_delta_isadj(const uint32_t* __restrict__ row_subj, uint64_t n_rows, const uint32_t* __restrict__ nd_rel,
                              uint32_t wildcard, uint32_t* __restrict__ flag) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_rows; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t s = row_subj[i];
    flag[i] = ((s & SET_BIT) && nd_rel[s & ~SET_BIT] != wildcard) ? 1u : 0u;
  }
}
__global__ void k_delta_adjfill(const uint32_t* __restrict__ row_subj, uint64_t n_rows, const uint32_t* __restrict__ flag,
                                const uint64_t* __restrict__ pos, uint32_t* __restrict__ adj) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_rows; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) adj[pos[i]] = row_subj[i] & ~SET_BIT;
}
__global__ void k_delta_adjoff(const uint64_t* __restrict__ row_off, uint32_t n, const uint64_t* __restrict__ pos,
                               uint64_t* __restrict__ adj_off) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v <= n) adj_off[v] = pos[row_off[v]];  // pos has n_rows + 1 entries (exclusive scan + total)
}

int Snapshot::create_from_delta(Snapshot* base, const kg_tuple* ins, const uint64_t* ins_keys, size_t n_ins,
                                const kg_tuple* del, size_t n_del, const kg_dict* dict, const kg_rewrite_prog* prog) {
  if (base->shard_n > 1) return set_error(-2, "kg_snapshot_apply: sharded snapshots rebuild instead");
  if (base->device != device) return set_error(-2, "kg_snapshot_apply: replica on another device");
  const uint32_t n0 = base->ds.n_nodes;
  wildcard_rel = dict ? dict->wildcard_rel : base->wildcard_rel;
  ds.wildcard_rel = wildcard_rel;
  // 1. the node map: taken over from the base (built once by kg_snapshot_create), or rebuilt from
  // the base's node triples when the base has none (synthetic, or already handed on)
  // base->mu guards the hand-over: two applies on one base (or an apply racing another host-side user
  // of these fields) take turns; the loser rebuilds the map from the device triples below
  std::unique_lock<std::mutex> base_lk(base->mu);
  if (!base->hmap.k.empty() && base->h_nd_ns.size() == n0) {
    hmap = std::move(base->hmap);
    h_nd_ns = std::move(base->h_nd_ns);
    h_nd_obj = std::move(base->h_nd_obj);
    h_nd_rel = std::move(base->h_nd_rel);
    base->hmap = HostMap{};
  } else {
    h_nd_ns.resize(n0);
    h_nd_obj.resize(n0);
    h_nd_rel.resize(n0);
    if (n0) {
      HIPC(hipMemcpy(h_nd_ns.data(), base->ds.nd_ns, (size_t)n0 * 4, hipMemcpyDeviceToHost));
      HIPC(hipMemcpy(h_nd_obj.data(), base->ds.nd_obj, (size_t)n0 * 4, hipMemcpyDeviceToHost));
      HIPC(hipMemcpy(h_nd_rel.data(), base->ds.nd_rel, (size_t)n0 * 4, hipMemcpyDeviceToHost));
    }
    hmap.init((uint64_t)n0 + n_ins + 16);
    for (uint32_t v = 0; v < n0; v++) hmap.put(nmap_key(h_nd_ns[v], h_nd_rel[v], h_nd_obj[v]), v);
  }
  base_lk.unlock();  // everything else read from the base is immutable device data
  auto intern = [&](uint32_t ns, uint32_t obj, uint32_t rel) -> uint32_t {
    const uint32_t id = (uint32_t)h_nd_ns.size();
    const uint32_t got = hmap.put(nmap_key(ns, rel, obj), id);
    if (got == id) {
      h_nd_ns.push_back(ns);
      h_nd_obj.push_back(obj);
      h_nd_rel.push_back(rel);
    }
    return got;
  };
  auto ok_ids = [](const kg_tuple& t) {
    if (t.ns >= 0xFFFF || t.rel >= 0xFFFF || t.obj >= 0x7FFFFFFF) return false;
    if (t.sns == KG_SUBJECT_ID) return t.sobj < 0x7FFFFFFF;
    return t.sns < 0xFFFF && t.srel < 0xFFFF && t.sobj < 0x7FFFFFFF;
  };
  // 2. the delta in node order
  struct Ins {
    uint32_t node, subj;
    uint64_t key;
    uint32_t seq;
  };
  std::vector<Ins> iv;
  iv.reserve(n_ins);
  for (size_t i = 0; i < n_ins; i++) {
    const kg_tuple& t = ins[i];
    if (!ok_ids(t)) return set_error(-2, "inserted tuple %zu: id out of range", i);
    const uint32_t v = intern(t.ns, t.obj, t.rel);
    const uint32_t s = t.sns == KG_SUBJECT_ID ? t.sobj : (SET_BIT | intern(t.sns, t.sobj, t.srel));
    iv.push_back(Ins{v, s, ins_keys ? ins_keys[i] : ~0ull, (uint32_t)i});
  }
  std::sort(iv.begin(), iv.end(), [](const Ins& a, const Ins& b) {
    return a.node != b.node ? a.node < b.node : (a.key != b.key ? a.key < b.key : a.seq < b.seq);
  });
  std::vector<std::pair<uint32_t, uint32_t>> dv;  // (node, subject); unknown tuples delete nothing
  for (size_t i = 0; i < n_del; i++) {
    const kg_tuple& t = del[i];
    if (!ok_ids(t)) continue;
    const uint32_t v = hmap.get(nmap_key(t.ns, t.rel, t.obj));
    if (v == NONE || v >= n0) continue;  // only base rows are deleted (inserts follow the deletes' effect)
    uint32_t s;
    if (t.sns == KG_SUBJECT_ID) {
      s = t.sobj;
    } else {
      const uint32_t c = hmap.get(nmap_key(t.sns, t.srel, t.sobj));
      if (c == NONE) continue;
      s = SET_BIT | c;
    }
    dv.emplace_back(v, s);
  }
  std::sort(dv.begin(), dv.end());
  dv.erase(std::unique(dv.begin(), dv.end()), dv.end());
  const uint32_t n1 = (uint32_t)h_nd_ns.size();
  ds.n_nodes = n1;
  // 3. device: delta arrays, new node triples
  std::vector<uint32_t> h_in(iv.size()), h_is(iv.size()), h_dn(dv.size()), h_dsub(dv.size());
  std::vector<uint64_t> h_ik(iv.size());
  for (size_t i = 0; i < iv.size(); i++) h_in[i] = iv[i].node, h_is[i] = iv[i].subj, h_ik[i] = iv[i].key;
  for (size_t i = 0; i < dv.size(); i++) h_dn[i] = dv[i].first, h_dsub[i] = dv[i].second;
  std::vector<void*> tmp;
  struct Free {
    std::vector<void*>& t;
    ~Free() {
      for (void* p : t) hipFree(p);
    }
  } free_tmp{tmp};
  auto talloc = [&](void** p, size_t bytes) -> int {
    HIPC(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return 0;
  };
  uint32_t *d_in, *d_is, *d_dn, *d_ds;
  uint64_t* d_ik;
  if (talloc((void**)&d_in, h_in.size() * 4) || talloc((void**)&d_is, h_is.size() * 4) ||
      talloc((void**)&d_ik, h_ik.size() * 8) || talloc((void**)&d_dn, h_dn.size() * 4) ||
      talloc((void**)&d_ds, h_dsub.size() * 4))
    return -1;
  if (!h_in.empty()) {
    HIPC(hipMemcpyAsync(d_in, h_in.data(), h_in.size() * 4, hipMemcpyHostToDevice, stream));
    HIPC(hipMemcpyAsync(d_is, h_is.data(), h_is.size() * 4, hipMemcpyHostToDevice, stream));
    HIPC(hipMemcpyAsync(d_ik, h_ik.data(), h_ik.size() * 8, hipMemcpyHostToDevice, stream));
  }
  if (!h_dn.empty()) {
    HIPC(hipMemcpyAsync(d_dn, h_dn.data(), h_dn.size() * 4, hipMemcpyHostToDevice, stream));
    HIPC(hipMemcpyAsync(d_ds, h_dsub.data(), h_dsub.size() * 4, hipMemcpyHostToDevice, stream));
  }
  const DeltaDev D{d_in, d_is, d_ik, (uint32_t)iv.size(), d_dn, d_ds, (uint32_t)dv.size()};
  uint32_t *d_ns, *d_obj, *d_rel;
  if (alloc((void**)&d_ns, (size_t)n1 * 4) || alloc((void**)&d_obj, (size_t)n1 * 4) || alloc((void**)&d_rel, (size_t)n1 * 4))
    return -1;
  if (n0) {
    HIPC(hipMemcpyAsync(d_ns, base->ds.nd_ns, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
    HIPC(hipMemcpyAsync(d_obj, base->ds.nd_obj, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
    HIPC(hipMemcpyAsync(d_rel, base->ds.nd_rel, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
  }
  if (n1 > n0) {
    HIPC(hipMemcpyAsync(d_ns + n0, h_nd_ns.data() + n0, (size_t)(n1 - n0) * 4, hipMemcpyHostToDevice, stream));
    HIPC(hipMemcpyAsync(d_obj + n0, h_nd_obj.data() + n0, (size_t)(n1 - n0) * 4, hipMemcpyHostToDevice, stream));
    HIPC(hipMemcpyAsync(d_rel + n0, h_nd_rel.data() + n0, (size_t)(n1 - n0) * 4, hipMemcpyHostToDevice, stream));
  }
  // 4. rows: lengths (untouched nodes directly, touched ones from their kept entries), offsets,
  // copy of untouched rows, scatter of kept + inserted entries of touched rows
  uint64_t *newlen, *d_ro;
  uint8_t* touched;
  if (talloc((void**)&newlen, ((size_t)n1 + 1) * 8) || talloc((void**)&touched, (size_t)n1 + 16) ||
      alloc((void**)&d_ro, ((size_t)n1 + 1) * 8))
    return -1;
  const uint32_t g1 = (n1 + 255) / 256;
  if (n1) {
    hipLaunchKernelGGL(k_delta_len, dim3(g1), dim3(256), 0, stream, base->ds.row_off, n0, n1, D, newlen, touched);
    HIPC(hipGetLastError());
  }
  // touched nodes (a few thousand at most): listed on the host from the delta itself
  std::vector<uint32_t> tl;
  for (const Ins& x : iv) tl.push_back(x.node);
  for (const auto& x : dv) tl.push_back(x.first);
  std::sort(tl.begin(), tl.end());
  tl.erase(std::unique(tl.begin(), tl.end()), tl.end());
  const uint32_t n_t = (uint32_t)tl.size();
  // their old row lengths scanned into flat offsets (toff), and node -> touched index (tslot)
  uint32_t *d_tl, *d_tslot;
  uint64_t *d_tlen, *d_toff;
  if (talloc((void**)&d_tl, (size_t)n_t * 4) || talloc((void**)&d_tlen, ((size_t)n_t + 1) * 8) ||
      talloc((void**)&d_toff, ((size_t)n_t + 1) * 8) || talloc((void**)&d_tslot, (size_t)n1 * 4))
    return -1;
  uint64_t F = 0;
  if (n_t) {
    HIPC(hipMemcpyAsync(d_tl, tl.data(), (size_t)n_t * 4, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_delta_tprep, dim3((n_t + 255) / 256), dim3(256), 0, stream, base->ds.row_off, n0,
                       (const uint32_t*)d_tl, n_t, d_tlen, d_tslot);
    HIPC(hipGetLastError());
  }
  HIPC(hipMemsetAsync(d_tlen + n_t, 0, 8, stream));
  {
    size_t t0b = 0;
    HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, t0b, d_tlen, d_toff, (size_t)n_t + 1, stream));
    void* t0s;
    if (talloc(&t0s, t0b + 16)) return -1;
    HIPC(hipcub::DeviceScan::ExclusiveSum(t0s, t0b, d_tlen, d_toff, (size_t)n_t + 1, stream));
    HIPC(hipMemcpyAsync(&F, d_toff + n_t, 8, hipMemcpyDeviceToHost, stream));
    HIPC(hipStreamSynchronize(stream));
  }
  uint32_t* d_keep;
  uint64_t* d_kr;
  if (talloc((void**)&d_keep, F * 4 + 4) || talloc((void**)&d_kr, (F + 1) * 8)) return -1;
  void* scratch = nullptr;
  size_t tb = 0, tb2 = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, newlen, d_ro, (size_t)n1 + 1, stream));
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, d_keep, d_kr, (size_t)F + 1, stream));
  tb = std::max(tb, tb2);
  if (F) {
    hipLaunchKernelGGL(k_delta_keep, dim3((uint32_t)std::min<uint64_t>(2048, (F + 255) / 256)), dim3(256), 0, stream,
                       base->ds.row_off, base->ds.row_subj, n0, D, (const uint32_t*)d_tl, n_t, (const uint64_t*)d_toff,
                       d_keep);
    HIPC(hipGetLastError());
  }
  HIPC(hipMemsetAsync(d_keep + F, 0, 4, stream));
  // (the scratch for every scan below: the largest of them)
  const uint64_t n_rows_max = base->h_row_off_last + iv.size();
  size_t tb3 = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, (const uint32_t*)nullptr, (uint64_t*)nullptr, (size_t)n_rows_max + 1,
                                        stream));
  tb = std::max(tb, tb3);
  if (talloc(&scratch, tb + 16)) return -1;
  HIPC(hipcub::DeviceScan::ExclusiveSum(scratch, tb, d_keep, d_kr, (size_t)F + 1, stream));
  if (n_t) {
    hipLaunchKernelGGL(k_delta_tlen, dim3((n_t + 255) / 256), dim3(256), 0, stream, (const uint32_t*)d_tl, n_t,
                       (const uint64_t*)d_toff, (const uint64_t*)d_kr, D, newlen);
    HIPC(hipGetLastError());
  }
  HIPC(hipMemsetAsync(newlen + n1, 0, 8, stream));
  HIPC(hipcub::DeviceScan::ExclusiveSum(scratch, tb, newlen, d_ro, (size_t)n1 + 1, stream));
  uint64_t total = 0;
  HIPC(hipMemcpyAsync(&total, d_ro + n1, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  uint32_t* d_rs;
  if (alloc((void**)&d_rs, total * 4 + 4)) return -1;
  const bool keyed = base->d_row_key != nullptr;
  if (keyed && alloc((void**)&d_row_key, total * 8 + 8)) return -1;
  const uint64_t old_rows = base->h_row_off_last;
  if (old_rows)
    hipLaunchKernelGGL(k_delta_copy, dim3(2048), dim3(256), 0, stream, base->ds.row_off, base->ds.row_subj,
                       base->d_row_key, n0, old_rows, (const uint64_t*)d_ro, (const uint8_t*)touched, d_rs, d_row_key);
  if (F)
    hipLaunchKernelGGL(k_delta_scatter_old, dim3((uint32_t)std::min<uint64_t>(2048, (F + 255) / 256)), dim3(256), 0,
                       stream, base->ds.row_off, base->ds.row_subj, base->d_row_key, D, (const uint32_t*)d_tl, n_t,
                       (const uint64_t*)d_toff, (const uint32_t*)d_keep, (const uint64_t*)d_kr, (const uint64_t*)d_ro,
                       d_rs, d_row_key);
  if (!iv.empty())
    hipLaunchKernelGGL(k_delta_scatter_ins, dim3((uint32_t)((iv.size() + 255) / 256)), dim3(256), 0, stream,
                       base->ds.row_off, base->d_row_key, n0, D, (const uint32_t*)d_tslot, (const uint64_t*)d_toff,
                       (const uint64_t*)d_kr, (const uint64_t*)d_ro, d_rs, d_row_key);
  HIPC(hipGetLastError());
  // 5. set-adjacency: a flag per row entry, scanned into positions
  uint32_t* flag;
  uint64_t* pos;
  if (talloc((void**)&flag, total * 4 + 8) || talloc((void**)&pos, (total + 1) * 8)) return -1;
  if (total)
    hipLaunchKernelGGL(k_delta_isadj, dim3(2048), dim3(256), 0, stream, (const uint32_t*)d_rs, total,
                       (const uint32_t*)d_rel, wildcard_rel, flag);
  HIPC(hipMemsetAsync(flag + total, 0, 4, stream));
  HIPC(hipcub::DeviceScan::ExclusiveSum(scratch, tb, flag, pos, (size_t)total + 1, stream));
  uint64_t n_adj = 0;
  HIPC(hipMemcpyAsync(&n_adj, pos + total, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  uint32_t* d_adj;
  uint64_t* d_ao;
  if (alloc((void**)&d_adj, n_adj * 4 + 4) || alloc((void**)&d_ao, ((size_t)n1 + 1) * 8)) return -1;
  if (total)
    hipLaunchKernelGGL(k_delta_adjfill, dim3(2048), dim3(256), 0, stream, (const uint32_t*)d_rs, total,
                       (const uint32_t*)flag, (const uint64_t*)pos, d_adj);
  hipLaunchKernelGGL(k_delta_adjoff, dim3((n1 + 1 + 255) / 256), dim3(256), 0, stream, (const uint64_t*)d_ro, n1,
                     (const uint64_t*)pos, d_ao);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(stream));
  ds.row_off = d_ro;
  ds.row_subj = d_rs;
  ds.adj_off = d_ao;
  ds.adj = d_adj;
  ds.nd_ns = d_ns;
  ds.nd_obj = d_obj;
  ds.nd_rel = d_rel;
  ds.nflags = nullptr;
  h_row_off_last = total;
  n_set_edges = n_adj;
  // 6. everything derived, as in a full build
  if (upload_program(dict, prog)) return -1;
  if (has_program && device_flags()) return -1;
  n_check_rows = h_row_off_last;
  if (augment_rewrites() || build_formulas()) return -1;
  return build_hash_tables();
}

}  // namespace kg
