// kg_snapshot.hip -- snapshot construction: host tuples or the device-side synthetic generator
// -> HBM-resident CSR + hash tables (layout in kg_internal.h).
//
// Replaces the read side of the SQL persister for the check path:
//   Persister.GetRelationTuples  internal/persistence/sql/relationtuples.go:203-244
//     (WHERE ns/obj/rel [/subject] ORDER BY shard_id) -> rows are laid out per (ns,obj,rel) in the
//     order given (the caller passes shard_id order), so expansion order == the reference's.
//   checkDirect's exact-tuple query (engine.go:159-163) -> dset hash probe.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "kg_internal.h"
#include "kg_snapshot.h"
#include "kg_synth.h"

namespace kg {

// ------------------------------------------------------------------ device hash-table builders
// Build kernels walk the row entries in chunks of CSR_CHUNK per thread: one owner search per chunk,
// then the owner advances across row boundaries (a thread per node waited for the longest -- hub --
// row; a search per entry cost ~28 dependent loads each at 1 B rows).
constexpr uint32_t CSR_CHUNK = 64;

__global__ void k_dset_insert_rows(uint64_t* dset, uint64_t nb, const uint64_t* row_off, const uint32_t* row_subj,
                                   uint32_t n_nodes, uint64_t n_rows) {
  const uint64_t nch = (n_rows + CSR_CHUNK - 1) / CSR_CHUNK;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    for (uint64_t i = c * CSR_CHUNK, ie = min(n_rows, i + CSR_CHUNK), v = csr_owner(row_off, n_nodes, i); i < ie; i++) {
      v = csr_advance(row_off, n_nodes, (uint32_t)v, i);
      const uint64_t key = dset_key((uint32_t)v, row_subj[i]);
      uint64_t b = dset_home(key, nb);
      for (uint64_t n = 0; n < nb; n++) {  // sized for load <= 0.25: always finds room
        uint64_t* bucket = dset + b * DSET_BUCKET;
        bool done = false;
        for (int s = 0; s < DSET_BUCKET; s++) {
          const unsigned long long old = atomicCAS((unsigned long long*)&bucket[s], (unsigned long long)EMPTY64,
                                                   (unsigned long long)key);
          if (old == EMPTY64 || old == key) {
            done = true;
            break;
          }
        }
        if (done) break;
        b = hash_next(b, nb);
      }
    }
  }
}

__global__ void k_nmap_insert(NSlot* nm, uint64_t slots, const uint32_t* nd_ns, const uint32_t* nd_obj,
                              const uint32_t* nd_rel, const uint64_t* adj_off, const uint32_t* xoff, const uint2* sig,
                              const uint8_t* flags, uint32_t n_nodes, const uint64_t* coff, const uint32_t* csub) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  uint64_t key = nmap_key(nd_ns[v], nd_rel[v], nd_obj[v]);
  uint64_t i = hash_home(key, slots);
  for (uint64_t n = 0; n < slots; n++) {  // sized for load <= 0.625: always finds room
    unsigned long long old =
        atomicCAS((unsigned long long*)&nm[i].key, (unsigned long long)EMPTY64, (unsigned long long)key);
    if (old == EMPTY64 || old == key) {
      nm[i].node = v;
      nm[i].beg = xoff ? xoff[v] : (uint32_t)adj_off[v];
      nm[i].len = (uint32_t)(adj_off[v + 1] - adj_off[v]);
      const uint2 g = sig[v];
      // node flags (k_resolve's impurity test without a random nflags read) + signature bits 0-11 in bits 20-31,
      // or a short check row in the slot (NSLOT_INL subjects at most: pad1's high word, then sig)
      const uint64_t cb = coff[v], cl = coff[v + 1] - cb;
      const uint64_t fl = flags ? flags[v] : 0u;
      if (cl <= NSLOT_INL) {
        const uint32_t s0 = cl >= 1 ? csub[cb] : NONE, s1 = cl >= 2 ? csub[cb + 1] : NONE;
        nm[i].sig = s1;
        nm[i].pad1 = fl | ((cl + 1) << 8) | ((uint64_t)s0 << 32);
      } else {
        nm[i].sig = g.y;
        nm[i].pad1 = fl | (g.x & SIG_LO);
      }
      return;
    }
    i = hash_next(i, slots);
  }
}

__global__ void k_node_owner(const uint32_t* nd_ns, const uint32_t* nd_obj, uint32_t n_nodes, uint32_t nranks,
                             uint8_t* owner) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n_nodes) owner[v] = (uint8_t)shard_owner(nd_ns[v], nd_obj[v], nranks);
}

// Bloom signature of every node's full row (direct subjects, tagged like dset keys).
__global__ void k_node_sig(const uint64_t* row_off, const uint32_t* row_subj, uint32_t n_nodes, uint2* sig) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  uint2 m = make_uint2(0u, 0u);
  for (uint64_t i = row_off[v], e = row_off[v + 1]; i < e && (m.x != SIG_LO || m.y != 0xFFFFFFFFu); i++) {
    const uint2 b = subj_sig(row_subj[i]);
    m.x |= b.x;
    m.y |= b.y;
  }
  sig[v] = m;
}

__global__ void k_build_adjx(const uint32_t* adj, const uint64_t* adj_off, const uint2* sig, uint64_t n_edges,
                             AdjX* adjx) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_edges;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = adj[e];
    const uint64_t b = adj_off[c], x = adj_off[c + 1];
    const uint2 g = sig[c];
    adjx[e] = AdjX{c, (uint32_t)b, (uint32_t)std::min<uint64_t>(x - b, ADJX_LEN_SAT) | (g.x & SIG_LO), g.y};
  }
}

// Hot-first adjx (round 5): the set rows are laid out in descending in-degree order of their nodes, so
// the rows a query batch keeps re-reading -- the popular groups every walk runs into -- share 128-B
// lines and stay in L2 / the Infinity Cache instead of sitting one per line among cold rows.  Node ids
// do not change; xoff[v] is v's row begin in adjx (nmap slots and adjx records carry it).
__global__ void k_hot_keys(const unsigned long long* indeg, uint32_t n, uint32_t* keys, uint32_t* vals) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const unsigned long long d = indeg[v];
    keys[v] = ~(uint32_t)(d < 0xFFFFFFFFull ? d : 0xFFFFFFFFull);  // ascending sort = descending in-degree
    vals[v] = v;
  }
}
__global__ void k_hot_lens(const uint32_t* order, const uint64_t* adj_off, uint32_t n, uint64_t* len) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t v = order[i];
    len[i] = adj_off[v + 1] - adj_off[v];
  }
}
__global__ void k_hot_scatter(const uint32_t* order, const uint64_t* pos, uint32_t n, uint32_t* xoff) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    xoff[order[i]] = (uint32_t)pos[i];
}
// One thread per node: its row's records at xoff[u] (long rows are build-time only)
__global__ void k_build_adjx_hot(const uint32_t* adj, const uint64_t* adj_off, const uint32_t* xoff, const uint2* sig,
                                 uint32_t n, AdjX* adjx) {
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < n; u += gridDim.x * blockDim.x) {
    const uint64_t b0 = adj_off[u], b1 = adj_off[u + 1];
    AdjX* out = adjx + xoff[u];
    for (uint64_t e = b0; e < b1; e++) {
      const uint32_t c = adj[e];
      const uint64_t l = adj_off[c + 1] - adj_off[c];
      const uint2 g = sig[c];
      out[e - b0] = AdjX{c, xoff[c], (uint32_t)std::min<uint64_t>(l, ADJX_LEN_SAT) | (g.x & SIG_LO), g.y};
    }
  }
}

// ------------------------------------------------------------------ reverse indexes
// In-degree over set-adjacency, then parents filled through per-node cursors (order within a
// parent list is irrelevant: the backward tier only asks "is the root reachable").
__global__ void k_indeg(const uint32_t* adj, uint64_t n_edges, unsigned long long* deg) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_edges; e += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&deg[adj[e]], 1ull);
}
// One thread per edge, the edge's source node precomputed (k_row_nodes over adj_off): the parents
// list slot comes from a returning atomic on the child's cursor, so a thread must not chain them (a
// chunk of edges per thread took 36 s on C3, whose union rows point at a few hot groups and
// folders), and a thread per node waits for the longest row.
__global__ void k_fill_radj(const uint32_t* __restrict__ adj, const uint32_t* __restrict__ src, uint64_t n_edges,
                            unsigned long long* cur, uint32_t* radj) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_edges; e += (uint64_t)gridDim.x * blockDim.x)
    radj[atomicAdd(&cur[adj[e]], 1ull)] = src[e];
}
// (subject, node) pairs of every row entry, to be sorted by subject
__global__ void k_row_nodes(const uint64_t* row_off, uint32_t n_nodes, uint64_t n_rows, uint32_t* node_of_row) {
  const uint64_t nch = (n_rows + CSR_CHUNK - 1) / CSR_CHUNK;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x)
    for (uint64_t i = c * CSR_CHUNK, ie = min(n_rows, i + CSR_CHUNK), v = csr_owner(row_off, n_nodes, i); i < ie; i++) {
      v = csr_advance(row_off, n_nodes, (uint32_t)v, i);
      node_of_row[i] = (uint32_t)v;
    }
}
__global__ void k_count_runs(const uint32_t* key, uint64_t n, unsigned long long* cnt) {
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
  for (int off = 32; off; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, (unsigned long long)c);
}
// Largest subject id (untagged key) of the sorted holder keys: the one key < SET_BIT whose
// successor is a tagged key or the end.
__global__ void k_hold_maxid(const uint32_t* key, uint64_t n, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (key[i] < SET_BIT && (i + 1 == n || key[i + 1] >= SET_BIT)) *out = key[i] + 1;
}
// Holder bitmap: one bit per subject id that some row holds (run starts of the sorted keys).
__global__ void k_hold_bits(const uint32_t* key, uint64_t n, uint32_t* bits) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = key[i];
    if (k < SET_BIT && (i == 0 || k != key[i - 1])) atomicOr(&bits[k >> 5], 1u << (k & 31));
  }
}
__device__ __forceinline__ uint64_t hold_slot(uint32_t key, uint64_t mask) { return mix64(key) & mask; }
// run starts insert (subject -> first index); run ends then add the count
__global__ void k_hold_insert(const uint32_t* key, uint64_t n, HSlot* hs, uint64_t mask) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (i != 0 && key[i] == key[i - 1]) continue;
    const uint32_t k = key[i];
    for (uint64_t h = hold_slot(k, mask), p = 0; p <= mask; p++, h = (h + 1) & mask) {  // load <= 0.5
      if (atomicCAS(&hs[h].key, NONE, k) == NONE) {
        hs[h].first = (uint32_t)i;
        break;
      }
    }
  }
}
__global__ void k_hold_count(const uint32_t* key, uint64_t n, HSlot* hs, uint64_t mask) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (i + 1 != n && key[i] == key[i + 1]) continue;
    const uint32_t k = key[i];
    for (uint64_t h = hold_slot(k, mask), p = 0; p <= mask; p++, h = (h + 1) & mask)
      if (hs[h].key == k) {
        hs[h].count = (uint32_t)(i + 1 - hs[h].first);
        break;
      }
  }
}

// ------------------------------------------------------------------ synthetic generator kernels
// set-adjacency keeps subject sets except "..." ones (engine.go:123-126), like the host path
__device__ __forceinline__ bool synth_is_adj(const SynthLayout& L, uint32_t sub) {
  if (!(sub & SET_BIT)) return false;
  uint32_t ns, obj, rel;
  synth_node(L, sub & ~SET_BIT, ns, obj, rel);
  return rel != 0;  // rel 0 == "..."
}

__global__ void k_synth_degrees(SynthLayout L, uint32_t n_nodes, uint32_t rank, uint32_t nranks, uint64_t* deg,
                                uint64_t* setdeg) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  uint32_t ns, obj, rel;
  synth_node(L, v, ns, obj, rel);
  // hash-sharded mode: rows of nodes owned by other ranks are empty here
  uint32_t d = shard_owner(ns, obj, nranks) == rank ? synth_degree(L, v) : 0u;
  uint32_t s = 0;
  for (uint32_t e = 0; e < d; e++) s += synth_is_adj(L, synth_subject(L, v, e)) ? 1u : 0u;
  deg[v] = d;
  setdeg[v] = s;
}

__global__ void k_synth_fill(SynthLayout L, uint32_t n_nodes, const uint64_t* row_off, const uint64_t* adj_off,
                             uint32_t* row_subj, uint32_t* adj, uint32_t* nd_ns, uint32_t* nd_obj, uint32_t* nd_rel) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  uint64_t r = row_off[v], a = adj_off[v];
  uint32_t d = (uint32_t)(row_off[v + 1] - r);
  for (uint32_t e = 0; e < d; e++) {
    uint32_t s = synth_subject(L, v, e);
    row_subj[r + e] = s;
    if (synth_is_adj(L, s)) adj[a++] = s & ~SET_BIT;
  }
  synth_node(L, v, nd_ns[v], nd_obj[v], nd_rel[v]);
}

// Purity closure on the device (the host path does it on the host): seed with the relation flags,
// then propagate "impure" backwards over set-adjacency until a fixed point.
__global__ void k_flags_init(DevSnap s, uint8_t* flags) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= s.n_nodes) return;
  const uint8_t rf = relflag(s, s.nd_ns[v], s.nd_rel[v]);
  flags[v] = rf ? (uint8_t)(NF_IMPURE | ((rf & 1) ? NF_REWRITE : 0) | ((rf & 2) ? NF_ERR : 0)) : 0;
}
__global__ void k_flags_propagate(DevSnap s, uint8_t* flags, uint32_t* changed) {
  uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= s.n_nodes || (flags[v] & NF_IMPURE)) return;
  for (uint64_t i = s.adj_off[v]; i < s.adj_off[v + 1]; i++)
    if (flags[s.adj[i]] & NF_IMPURE) {
      flags[v] |= NF_IMPURE;
      *changed = 1;
      return;
    }
}

// ------------------------------------------------------------------ Snapshot
static uint64_t pow2_at_least(uint64_t x) {
  uint64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

Snapshot::~Snapshot() {
  shard_comms_free(this);  // before the streams and buffers they use
  for (auto& set : lane_sets)
    for (Lane* l : set) delete l;  // before the workspaces: a lane's stream owns one of them
  for (Snapshot* p : peers) delete p;
  if (device >= 0) hipSetDevice(device);
  for (auto& a : allocs) hipFree(a.first);
  for (Workspace* w : wss) delete w;
  for (ShardCtx* c : shard_ctxs) delete c;
  giant.release();
  if (stream) hipStreamDestroy(stream);
}

void GridPool::release() {
  if (mem) hipFree(mem);
  mem = nullptr;
  bytes = 0;
  cap = 0;
  epoch = 0;
}

// Host-buffer batches (kg_check_batch, the batcher's dispatchers) wait asleep on a blocking-sync
// event: a spinning hipStreamSynchronize per in-flight batch burns a core each, and a server whose
// cgroup CPU quota runs out is throttled for the rest of the period -- the native batcher's p99 of
// ~70 ms at 256 callers.
int Workspace::wait(hipStream_t st, bool blocking) {
  if (!blocking) {
    HIPC(hipStreamSynchronize(st));
    return 0;
  }
  if (!sync_ev) HIPC(hipEventCreateWithFlags(&sync_ev, hipEventBlockingSync | hipEventDisableTiming));
  HIPC(hipEventRecord(sync_ev, st));
  HIPC(hipEventSynchronize(sync_ev));
  return 0;
}

Workspace::~Workspace() {
  if (device >= 0) hipSetDevice(device);
  if (sync_ev) hipEventDestroy(sync_ev);
  if (scratch) hipFree(scratch);
  grid.release();
  ms.release();
  if (interp_pool) hipFree(interp_pool);
  if (split) hipFree(split);
  if (unpacked) hipFree(unpacked);
  if (pinned) hipHostFree(pinned);
  for (auto& e : ev)
    if (e) hipEventDestroy(e);
  for (auto& e : lev_ev)
    if (e) hipEventDestroy(e);
  if (exp) expand_bufs_free(exp);
}

void* Workspace::host_buf(size_t bytes) {
  if (bytes > 65536) return nullptr;
  if (!pinned && hipHostMalloc(&pinned, 65536, hipHostMallocDefault) != hipSuccess) pinned = nullptr;
  return pinned;
}

Lane::~Lane() {
  if (device >= 0) hipSetDevice(device);
  if (h_q) hipHostFree(h_q);
  if (h_out) hipHostFree(h_out);
  if (h_err) hipHostFree(h_err);
  if (d_q) hipFree(d_q);
  if (d_out) hipFree(d_out);
  if (d_err) hipFree(d_err);
  if (d_pk) hipFree(d_pk);
  if (d_el) hipFree(d_el);
  if (h_el) hipHostFree(h_el);
  if (exp) expand_bufs_free(exp);
  // the stream's workspace belongs to the replica (freed with it); the stream itself is ours
  if (stream) hipStreamDestroy(stream);
}

int Lane::reserve(size_t n) {
  if (n <= cap) return 0;
  HIPC(hipSetDevice(device));
  // >= 64 Ki queries (2.3 MB of pinned staging): a request batcher's batches never reallocate
  // (pinned allocation and hipFree both stall), larger host batches grow it geometrically
  size_t c = std::max<size_t>(n, 65536);
  c = std::max(c, 2 * cap);
  HIPC(hipStreamSynchronize(stream));
  for (void* p : {(void*)h_q, (void*)h_out, (void*)h_err})
    if (p) hipHostFree(p);
  for (void* p : {(void*)d_q, (void*)d_out, (void*)d_err})
    if (p) hipFree(p);
  h_q = nullptr, h_out = nullptr, h_err = nullptr, d_q = nullptr, d_out = nullptr, d_err = nullptr;
  cap = 0;
  HIPC(hipHostMalloc(&h_q, c * sizeof(kg_query), hipHostMallocDefault));
  HIPC(hipHostMalloc(&h_out, c, hipHostMallocDefault));
  HIPC(hipHostMalloc(&h_err, c * 4, hipHostMallocDefault));
  HIPC(hipMalloc(&d_q, c * sizeof(kg_query)));
  HIPC(hipMalloc(&d_out, c));
  HIPC(hipMalloc(&d_err, c * 4));
  cap = c;
  return 0;
}

int Lane::reserve_packed(size_t n) {
  if (int rc = reserve(n)) return rc;  // h_q stages the packed queries, d_q holds them unpacked
  if (n <= pk_cap && d_pk) return 0;
  HIPC(hipSetDevice(device));
  HIPC(hipStreamSynchronize(stream));
  if (d_pk) hipFree(d_pk);
  if (d_el) hipFree(d_el);
  d_pk = nullptr;
  d_el = nullptr;
  pk_cap = 0;
  if (!h_el) HIPC(hipHostMalloc(&h_el, (2 + 2 * EL_PREFETCH) * 4, hipHostMallocDefault));
  HIPC(hipMalloc(&d_pk, cap * sizeof(kg_query_packed)));
  HIPC(hipMalloc(&d_el, (2 + 2 * cap) * 4));
  pk_cap = cap;
  return 0;
}

std::vector<Lane*>* Snapshot::lanes_acquire() {
  std::unique_lock<std::mutex> lk(lane_mu);
  lane_cv.wait(lk, [&] { return !lane_free.empty() || lane_sets.size() < lane_cap; });
  if (!lane_free.empty()) {
    std::vector<Lane*>* v = lane_free.back();
    lane_free.pop_back();
    return v;
  }
  std::vector<Lane*> v;
  for (size_t i = 0; i < n_replicas(); i++) {
    Snapshot* r = replica(i);
    Lane* l = new Lane();
    l->rep = r;
    l->device = r->device;
    if (hipSetDevice(r->device) != hipSuccess || hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking) != hipSuccess) {
      delete l;
      for (Lane* x : v) delete x;
      set_error(-1, "stream for a batch lane on device %d", r->device);
      return nullptr;
    }
    l->w = r->workspace(l->stream);
    v.push_back(l);
  }
  lane_sets.emplace_back(std::move(v));
  return &lane_sets.back();
}

void Snapshot::lanes_release(std::vector<Lane*>* v) {
  {
    std::lock_guard<std::mutex> lk(lane_mu);
    lane_free.push_back(v);
  }
  lane_cv.notify_one();
}

ShardCtx::~ShardCtx() {
  if (device >= 0) hipSetDevice(device);
  for (void* p : {vis, heavy, qcnt, qinfo, (void*)ref, (void*)bits, (void*)cnt8})
    if (p) hipFree(p);
}

ShardCtx* Snapshot::shard_ctx(hipStream_t st, bool create) {
  if (!st) st = stream;
  std::lock_guard<std::mutex> lk(ws_mu);
  for (ShardCtx* c : shard_ctxs)
    if (c->stream == st) return c;
  if (!create) return nullptr;
  ShardCtx* c = new (std::nothrow) ShardCtx();
  if (!c) return nullptr;
  c->stream = st;
  c->device = device;
  shard_ctxs.push_back(c);
  return c;
}

Workspace* Snapshot::workspace(hipStream_t st) {
  if (!st) st = stream;
  std::lock_guard<std::mutex> lk(ws_mu);
  for (Workspace* w : wss)
    if (w->stream == st) return w;
  Workspace* w = new Workspace();
  w->device = device;
  w->stream = st;
  wss.push_back(w);
  return w;
}

int Snapshot::alloc(void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return set_error(KG_ERR_RESOURCE_CODE, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  allocs.emplace_back(*p, bytes);
  device_bytes += bytes;
  return 0;
}

void Snapshot::free_alloc(const void* p) {
  for (size_t i = 0; i < allocs.size(); i++)
    if (allocs[i].first == p) {
      hipFree(allocs[i].first);
      device_bytes -= allocs[i].second;
      allocs[i] = allocs.back();
      allocs.pop_back();
      return;
    }
}

int Snapshot::init_device(int dev) {
  device = dev;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return set_error(-1, "hipSetDevice(%d): %s", dev, hipGetErrorString(e));
  e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  if (e != hipSuccess) return set_error(-1, "hipStreamCreate: %s", hipGetErrorString(e));
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  n_cu = cus > 0 ? cus : 256;
  return 0;
}

// Hash tables: dset sized for load <= 0.25 over 2-key (16-B) buckets; nmap for load <= 0.5.
int Snapshot::build_hash_tables() {
  // inlined child rows for the BFS (indices are u32: up to 2^32-1 set edges per snapshot)
  if (n_set_edges >= 0xFFFFFFFFull) return set_error(KG_ERR_RESOURCE_CODE, "more than 2^32-1 subject-set edges");
  AdjX* adjx = nullptr;
  if (alloc((void**)&adjx, (n_set_edges + 1) * sizeof(AdjX))) return -1;
  // per-node Bloom signature of the row subjects: inlined in adjx (child probes) and in the node map
  // (k_resolve's root probe)
  uint2* sig = nullptr;
  HIPC(hipMalloc(&sig, (size_t)ds.n_nodes * 8 + 8));
  // direct tuples as checkDirect sees them: the check rows of a materialised snapshot, else the rows
  const uint64_t* coff = ds.crow_off ? ds.crow_off : ds.row_off;
  const uint32_t* csub = ds.crow_off ? ds.crow_subj : ds.row_subj;
  if (ds.n_nodes) {
    hipLaunchKernelGGL(k_node_sig, dim3((ds.n_nodes + 255) / 256), dim3(256), 0, stream, coff, csub, ds.n_nodes, sig);
    HIPC(hipGetLastError());
  }
  // hot-first layout unless KG_ADJX_ORDER=0 (node order, adjx parallel to adj)
  const char* order_env = getenv("KG_ADJX_ORDER");
  const bool hot = n_set_edges && ds.n_nodes && !(order_env && atoi(order_env) == 0);
  uint32_t* xoff = nullptr;
  if (hot) {
    const uint32_t nn = ds.n_nodes;
    if (alloc((void**)&xoff, ((size_t)nn + 1) * 4)) return -1;
    unsigned long long* indeg = nullptr;
    uint32_t *k0, *k1, *v0, *v1;
    uint64_t *len, *pos;
    HIPC(hipMalloc(&indeg, (size_t)nn * 8));
    HIPC(hipMalloc(&k0, (size_t)nn * 4));
    HIPC(hipMalloc(&k1, (size_t)nn * 4));
    HIPC(hipMalloc(&v0, (size_t)nn * 4));
    HIPC(hipMalloc(&v1, (size_t)nn * 4));
    HIPC(hipMemsetAsync(indeg, 0, (size_t)nn * 8, stream));
    hipLaunchKernelGGL(k_indeg, dim3(4096), dim3(256), 0, stream, ds.adj, n_set_edges, indeg);
    hipLaunchKernelGGL(k_hot_keys, dim3(4096), dim3(256), 0, stream, indeg, nn, k0, v0);
    HIPC(hipGetLastError());
    hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
    size_t tmp_bytes = 0;
    HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kb, vb, (size_t)nn, 0, 32, stream));
    void* tmp = nullptr;
    size_t scan_bytes = 0;
    HIPC(hipFree(indeg));  // reuse its bytes: lengths and positions in sorted order (u64 each)
    HIPC(hipMalloc(&len, ((size_t)nn + 1) * 8));
    HIPC(hipMalloc(&pos, ((size_t)nn + 1) * 8));
    HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, len, pos, (size_t)nn, stream));
    HIPC(hipMalloc(&tmp, std::max(tmp_bytes, scan_bytes) + 16));
    HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kb, vb, (size_t)nn, 0, 32, stream));
    hipLaunchKernelGGL(k_hot_lens, dim3(4096), dim3(256), 0, stream, vb.Current(), ds.adj_off, nn, len);
    HIPC(hipGetLastError());
    HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, scan_bytes, len, pos, (size_t)nn, stream));
    hipLaunchKernelGGL(k_hot_scatter, dim3(4096), dim3(256), 0, stream, vb.Current(), pos, nn, xoff);
    HIPC(hipGetLastError());
    HIPC(hipMemsetAsync(xoff + nn, 0, 4, stream));
    hipLaunchKernelGGL(k_build_adjx_hot, dim3(4096), dim3(256), 0, stream, ds.adj, ds.adj_off, xoff, sig, nn, adjx);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(stream));
    for (void* p : {(void*)k0, (void*)k1, (void*)v0, (void*)v1, (void*)len, (void*)pos, tmp}) HIPC(hipFree(p));
  } else if (n_set_edges) {
    hipLaunchKernelGGL(k_build_adjx, dim3(2048), dim3(256), 0, stream, ds.adj, ds.adj_off, sig, n_set_edges, adjx);
    HIPC(hipGetLastError());
  }
  ds.adjx = adjx;
  ds.adjx_off = xoff;
  const uint64_t n_rows = n_check_rows;
  // load <= 0.25 keys per slot: a miss (the common probe) reads one bucket with probability ~0.9.
  // A table that would take more than a fifth of the device's HBM runs at 0.375 instead (and the
  // node map at 0.625 past an eighth), so the largest graphs leave room for batches in flight.
  size_t hbm_free = 0, hbm_total = 0;
  if (hipMemGetInfo(&hbm_free, &hbm_total) != hipSuccess) hbm_total = 288ull << 30;
  (void)hipGetLastError();
  uint64_t buckets = std::max<uint64_t>(1, (n_rows * 4 + DSET_BUCKET - 1) / DSET_BUCKET);
  if (buckets * DSET_BUCKET * 8 > hbm_total / 5) buckets = std::max<uint64_t>(1, (n_rows * 8 + 2) / 3 / DSET_BUCKET);
  if (buckets >= (1ull << 32)) {  // dset_home scales by a 32-bit bucket count
    if (n_rows * 2 >= (0xFFFFFFFFull - 1) * DSET_BUCKET) return set_error(KG_ERR_RESOURCE_CODE, "check rows exceed dset");
    buckets = 0xFFFFFFFFull;
  }
  uint64_t* dset = nullptr;
  if (alloc((void**)&dset, buckets * DSET_BUCKET * 8)) return -1;
  HIPC(hipMemsetAsync(dset, 0xFF, buckets * DSET_BUCKET * 8, stream));
  uint64_t slots = std::max<uint64_t>(16, (uint64_t)ds.n_nodes * 2);
  if (slots * sizeof(NSlot) > hbm_total / 8) slots = std::max<uint64_t>(16, (uint64_t)ds.n_nodes * 8 / 5);
  NSlot* nm = nullptr;
  if (alloc((void**)&nm, slots * sizeof(NSlot))) return -1;
  HIPC(hipMemsetAsync(nm, 0xFF, slots * sizeof(NSlot), stream));
  uint32_t grid = (ds.n_nodes + 255) / 256;
  if (ds.n_nodes) {
    if (n_rows)
      hipLaunchKernelGGL(k_dset_insert_rows, dim3((uint32_t)std::min<uint64_t>(65536, (n_rows + 64 * 256 - 1) / (64 * 256))), dim3(256), 0,
                         stream, dset, buckets, coff, csub, ds.n_nodes, n_rows);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_nmap_insert, dim3(grid), dim3(256), 0, stream, nm, slots, ds.nd_ns, ds.nd_obj,
                       ds.nd_rel, ds.adj_off, xoff, sig, ds.nflags, ds.n_nodes, coff, csub);
    HIPC(hipGetLastError());
  }
  HIPC(hipStreamSynchronize(stream));
  HIPC(hipFree(sig));
  ds.dset = dset;
  ds.dset_nb = buckets;
  ds.nmap = nm;
  ds.nmap_n = slots;
  ds.shard_rank = shard_rank;
  ds.shard_n = shard_n;
  ds.nowner = nullptr;
  if (shard_n > 1 && ds.n_nodes) {
    uint8_t* no = nullptr;
    if (alloc((void**)&no, ds.n_nodes)) return -1;
    hipLaunchKernelGGL(k_node_owner, dim3(grid), dim3(256), 0, stream, ds.nd_ns, ds.nd_obj, ds.n_nodes, shard_n, no);
    HIPC(hipGetLastError());
    ds.nowner = no;
  }
  HIPC(hipStreamSynchronize(stream));
  return build_reverse();
}

// Reverse indexes for the backward tier: parents through set-adjacency, and the holders of every
// subject (its row entries sorted by subject, plus a subject -> range hash).  Skipped (tier off)
// when row positions do not fit u32.
int Snapshot::build_reverse() {
  const uint32_t nn = ds.n_nodes;
  const uint64_t E = n_set_edges, R = n_check_rows;
  const uint64_t* coff = ds.crow_off ? ds.crow_off : ds.row_off;
  const uint32_t* csub = ds.crow_off ? ds.crow_subj : ds.row_subj;
  ds.radj = nullptr;
  ds.hbits = nullptr;
  ds.hbits_n = 0;
  if (R >= 0xFFFFFFFFull || nn == 0) return 0;
  uint64_t* roff = nullptr;
  uint32_t* radj = nullptr;
  if (alloc((void**)&roff, ((size_t)nn + 1) * 8) || alloc((void**)&radj, (E + 1) * 4)) return -1;
  unsigned long long* deg = nullptr;
  HIPC(hipMalloc(&deg, ((size_t)nn + 1) * 8));
  HIPC(hipMemsetAsync(deg, 0, ((size_t)nn + 1) * 8, stream));
  const uint32_t grid = (nn + 255) / 256;
  if (E) hipLaunchKernelGGL(k_indeg, dim3(4096), dim3(256), 0, stream, ds.adj, E, deg);
  HIPC(hipGetLastError());
  size_t tmp_bytes = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, (uint64_t*)deg, roff, (size_t)nn + 1, stream));
  void* tmp = nullptr;
  HIPC(hipMalloc(&tmp, tmp_bytes + 16));
  HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (uint64_t*)deg, roff, (size_t)nn + 1, stream));
  HIPC(hipMemcpyAsync(deg, roff, ((size_t)nn + 1) * 8, hipMemcpyDeviceToDevice, stream));
  if (E) {
    uint32_t* src = nullptr;
    HIPC(hipMalloc(&src, E * 4));
    hipLaunchKernelGGL(k_row_nodes, dim3((uint32_t)std::min<uint64_t>(65536, (E + 64 * 256 - 1) / (64 * 256))), dim3(256),
                       0, stream, ds.adj_off, nn, E, src);
    hipLaunchKernelGGL(k_fill_radj, dim3((uint32_t)std::min<uint64_t>(65536, (E + 255) / 256)), dim3(256), 0, stream,
                       ds.adj, (const uint32_t*)src, E, deg, radj);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(stream));
    HIPC(hipFree(src));
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(stream));
  HIPC(hipFree(tmp));
  HIPC(hipFree(deg));
  // holders: sort (subject, node) by subject
  uint32_t *k0, *k1, *v0, *v1;
  HIPC(hipMalloc(&k0, R * 4 + 4));
  HIPC(hipMalloc(&k1, R * 4 + 4));
  HIPC(hipMalloc(&v0, R * 4 + 4));
  HIPC(hipMalloc(&v1, R * 4 + 4));
  HIPC(hipMemcpyAsync(k0, csub, R * 4, hipMemcpyDeviceToDevice, stream));
  if (R)
    hipLaunchKernelGGL(k_row_nodes, dim3((uint32_t)std::min<uint64_t>(65536, (R + 64 * 256 - 1) / (64 * 256))), dim3(256), 0, stream,
                       coff, nn, R, v0);
  HIPC(hipGetLastError());
  hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
  tmp_bytes = 0;
  HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kb, vb, (size_t)R, 0, 32, stream));
  HIPC(hipMalloc(&tmp, tmp_bytes + 16));
  HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kb, vb, (size_t)R, 0, 32, stream));
  unsigned long long* cnt;
  HIPC(hipMalloc(&cnt, 16));
  HIPC(hipMemsetAsync(cnt, 0, 16, stream));
  if (R) {
    hipLaunchKernelGGL(k_count_runs, dim3(4096), dim3(256), 0, stream, kb.Current(), R, cnt);
    hipLaunchKernelGGL(k_hold_maxid, dim3(4096), dim3(256), 0, stream, kb.Current(), R, (uint32_t*)(cnt + 1));
  }
  unsigned long long hcnt[2] = {0, 0};
  HIPC(hipMemcpyAsync(hcnt, cnt, 16, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  const unsigned long long distinct = hcnt[0];
  const uint32_t nbits = (uint32_t)hcnt[1];  // max held subject id + 1 (0: no subject ids)
  uint32_t* hbits = nullptr;
  if (nbits) {
    const size_t words = ((size_t)nbits + 31) / 32;
    if (alloc((void**)&hbits, words * 4)) return -1;
    HIPC(hipMemsetAsync(hbits, 0, words * 4, stream));
    hipLaunchKernelGGL(k_hold_bits, dim3(4096), dim3(256), 0, stream, kb.Current(), R, hbits);
    HIPC(hipGetLastError());
  }
  const uint64_t slots = pow2_at_least(std::max<uint64_t>(16, distinct * 2));
  uint32_t* hold;
  HSlot* hs;
  if (alloc((void**)&hs, slots * sizeof(HSlot)) || alloc((void**)&hold, R * 4 + 4)) return -1;
  HIPC(hipMemsetAsync(hs, 0xFF, slots * sizeof(HSlot), stream));
  if (R) {
    hipLaunchKernelGGL(k_hold_insert, dim3(4096), dim3(256), 0, stream, kb.Current(), R, hs, slots - 1);
    hipLaunchKernelGGL(k_hold_count, dim3(4096), dim3(256), 0, stream, kb.Current(), R, hs, slots - 1);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(hold, vb.Current(), R * 4, hipMemcpyDeviceToDevice, stream));
  }
  HIPC(hipStreamSynchronize(stream));
  for (void* p : {(void*)k0, (void*)k1, (void*)v0, (void*)v1, tmp, (void*)cnt}) HIPC(hipFree(p));
  ds.radj_off = roff;
  ds.radj = radj;
  ds.hold = hold;
  ds.hslots = hs;
  ds.hmask = slots - 1;
  ds.hbits = hbits;
  ds.hbits_n = nbits;
  return 0;
}

// Upload the rewrite program and the (ns,rel) flag table (dense n_ns x n_rel).
int Snapshot::upload_program(const kg_dict* dict, const kg_rewrite_prog* prog) {
  prog_copy = ProgCopy{};
  prog_copy.have = true;
  if (dict) prog_copy.dict = *dict;
  else prog_copy.dict = kg_dict{0, 0, 0xFFFFFFFFu};
  if (prog) {
    prog_copy.ns_has_rel.assign(prog->ns_has_rel, prog->ns_has_rel + prog->n_ns);
    prog_copy.rel_ns.assign(prog->rel_ns, prog->rel_ns + prog->n_rel);
    prog_copy.rel_rel.assign(prog->rel_rel, prog->rel_rel + prog->n_rel);
    prog_copy.rel_root.assign(prog->rel_root, prog->rel_root + prog->n_rel);
    prog_copy.rw.assign(prog->rw, prog->rw + prog->n_rw);
    prog_copy.child.assign(prog->child, prog->child + prog->n_child);
  }
  ds.n_ns = std::max<uint32_t>(dict ? dict->n_namespaces : 0, prog ? prog->n_ns : 0);
  ds.n_rel = dict ? dict->n_relations : 0;
  if (prog)
    for (uint32_t j = 0; j < prog->n_rel; j++) {
      ds.n_rel = std::max(ds.n_rel, prog->rel_rel[j] + 1);
      ds.n_ns = std::max(ds.n_ns, prog->rel_ns[j] + 1);
    }
  has_program = false;
  if (prog)
    for (uint32_t i = 0; i < prog->n_ns; i++) has_program |= prog->ns_has_rel[i] != 0;
  ds.relflags = nullptr;
  ds.ns_has_rel = nullptr;
  ds.relroot = nullptr;
  ds.rw = nullptr;
  ds.rwchild = nullptr;
  ds.n_rw = 0;
  if (!has_program) return 0;
  if ((uint64_t)ds.n_ns * ds.n_rel > (64ull << 20))
    return set_error(KG_ERR_RESOURCE_CODE, "namespace x relation table too large (%u x %u)", ds.n_ns, ds.n_rel);
  size_t nt = (size_t)ds.n_ns * ds.n_rel;
  h_relflags.assign(nt, 0);
  h_relroot.assign(nt, -1);
  for (uint32_t ns = 0; ns < prog->n_ns; ns++)
    if (prog->ns_has_rel[ns])
      for (uint32_t r = 0; r < ds.n_rel; r++) h_relflags[(size_t)ns * ds.n_rel + r] = 2;  // undeclared -> error
  for (uint32_t j = 0; j < prog->n_rel; j++) {
    size_t at = (size_t)prog->rel_ns[j] * ds.n_rel + prog->rel_rel[j];
    if (prog->rel_ns[j] < prog->n_ns && !prog->ns_has_rel[prog->rel_ns[j]]) continue;
    h_relflags[at] = prog->rel_root[j] >= 0 ? 1 : 0;
    h_relroot[at] = prog->rel_root[j];
  }
  h_rw.assign((const RwNode*)prog->rw, (const RwNode*)prog->rw + prog->n_rw);
  h_rwchild.assign(prog->child, prog->child + prog->n_child);
  std::vector<uint8_t> nshas(ds.n_ns, 0);
  for (uint32_t ns = 0; ns < prog->n_ns && ns < ds.n_ns; ns++) nshas[ns] = prog->ns_has_rel[ns] ? 1 : 0;
  uint8_t *rf, *nh;
  int32_t* rr;
  RwNode* rw;
  int32_t* rc;
  if (alloc((void**)&rf, nt) || alloc((void**)&rr, nt * 4) || alloc((void**)&rw, (h_rw.size() + 1) * sizeof(RwNode)) ||
      alloc((void**)&rc, (h_rwchild.size() + 1) * 4) || alloc((void**)&nh, ds.n_ns + 1))
    return -1;
  HIPC(hipMemcpy(nh, nshas.data(), ds.n_ns, hipMemcpyHostToDevice));
  ds.ns_has_rel = nh;
  HIPC(hipMemcpy(rf, h_relflags.data(), nt, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(rr, h_relroot.data(), nt * 4, hipMemcpyHostToDevice));
  if (!h_rw.empty()) HIPC(hipMemcpy(rw, h_rw.data(), h_rw.size() * sizeof(RwNode), hipMemcpyHostToDevice));
  if (!h_rwchild.empty()) HIPC(hipMemcpy(rc, h_rwchild.data(), h_rwchild.size() * 4, hipMemcpyHostToDevice));
  ds.relflags = rf;
  ds.relroot = rr;
  ds.rw = rw;
  ds.rwchild = rc;
  ds.n_rw = (uint32_t)h_rw.size();
  return 0;
}

uint8_t Snapshot::host_relflag(uint32_t ns, uint32_t rel) const {
  if (!has_program || ns >= ds.n_ns || rel >= ds.n_rel) return 0;
  return h_relflags[(size_t)ns * ds.n_rel + rel];
}

int Snapshot::create_from_tuples(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                                 const uint64_t* keys) {
  wildcard_rel = dict ? dict->wildcard_rel : NONE;
  ds.wildcard_rel = wildcard_rel;
  // 1. intern nodes (ns, obj, rel) in first-appearance order
  HostMap& m = hmap;
  m.init(n + 16);
  std::vector<uint32_t> lhs(n), sub(n);
  auto intern = [&](uint32_t ns, uint32_t obj, uint32_t rel) -> uint32_t {
    uint32_t id = (uint32_t)h_nd_ns.size();
    uint32_t got = m.put(nmap_key(ns, rel, obj), id);
    if (got == id) {
      h_nd_ns.push_back(ns);
      h_nd_obj.push_back(obj);
      h_nd_rel.push_back(rel);
    }
    return got;
  };
  for (size_t i = 0; i < n; i++) {
    const kg_tuple& t = rows[i];
    if (t.ns >= 0xFFFF || t.rel >= 0xFFFF || t.obj >= 0x7FFFFFFF)
      return set_error(-2, "tuple %zu: id out of range", i);
    lhs[i] = intern(t.ns, t.obj, t.rel);
    if (t.sns == KG_SUBJECT_ID) {
      if (t.sobj >= 0x7FFFFFFF) return set_error(-2, "tuple %zu: subject id out of range", i);
      sub[i] = t.sobj;
    } else {
      if (t.sns >= 0xFFFF || t.srel >= 0xFFFF || t.sobj >= 0x7FFFFFFF)
        return set_error(-2, "tuple %zu: subject set id out of range", i);
      sub[i] = SET_BIT | intern(t.sns, t.sobj, t.srel);
    }
  }
  uint32_t nn = (uint32_t)h_nd_ns.size();
  ds.n_nodes = nn;
  // 2. rows per node in tuple (shard) order: counting sort; in the hash-sharded mode only the rows
  // of nodes this rank owns are kept (node ids stay global)
  if (shard_n > 1)
    for (size_t i = 0; i < n; i++)
      if (shard_owner(h_nd_ns[lhs[i]], h_nd_obj[lhs[i]], shard_n) != shard_rank) lhs[i] = NONE;
  h_row_off.assign((size_t)nn + 1, 0);
  h_adj_off.assign((size_t)nn + 1, 0);
  for (size_t i = 0; i < n; i++) {
    if (lhs[i] == NONE) continue;
    h_row_off[lhs[i] + 1]++;
    uint32_t s = sub[i];
    if ((s & SET_BIT) && h_nd_rel[s & ~SET_BIT] != wildcard_rel) h_adj_off[lhs[i] + 1]++;
  }
  for (uint32_t v = 0; v < nn; v++) {
    h_row_off[v + 1] += h_row_off[v];
    h_adj_off[v + 1] += h_adj_off[v];
  }
  h_row_subj.assign(h_row_off[nn], 0);
  std::vector<uint32_t> adj(h_adj_off[nn]);
  std::vector<uint64_t> row_key(keys ? h_row_off[nn] : 0);  // rows keep the input (key) order per node
  {
    std::vector<uint64_t> fr(h_row_off.begin(), h_row_off.end() - 1), fa(h_adj_off.begin(), h_adj_off.end() - 1);
    for (size_t i = 0; i < n; i++) {
      if (lhs[i] == NONE) continue;
      uint32_t s = sub[i], v = lhs[i];
      if (keys) row_key[fr[v]] = keys[i];
      h_row_subj[fr[v]++] = s;
      if ((s & SET_BIT) && h_nd_rel[s & ~SET_BIT] != wildcard_rel) adj[fa[v]++] = s & ~SET_BIT;
    }
  }
  h_row_off_last = h_row_off[nn];
  // 3. program + purity closure
  if (upload_program(dict, prog)) return -1;
  std::vector<uint8_t> flags;
  if (has_program) {
    flags.assign(nn, 0);
    std::vector<uint32_t> work;
    for (uint32_t v = 0; v < nn; v++) {
      uint8_t rf = host_relflag(h_nd_ns[v], h_nd_rel[v]);
      if (rf & 1) flags[v] |= NF_REWRITE;
      if (rf & 2) flags[v] |= NF_ERR;
      if (rf) {
        flags[v] |= NF_IMPURE;
        work.push_back(v);
      }
    }
    // reverse set-adjacency: a node is impure when an impure node is reachable from it
    std::vector<uint64_t> roff((size_t)nn + 1, 0);
    for (uint32_t c : adj) roff[c + 1]++;
    for (uint32_t v = 0; v < nn; v++) roff[v + 1] += roff[v];
    std::vector<uint32_t> radj(adj.size());
    {
      std::vector<uint64_t> f(roff.begin(), roff.end() - 1);
      for (uint32_t v = 0; v < nn; v++)
        for (uint64_t i = h_adj_off[v]; i < h_adj_off[v + 1]; i++) radj[f[adj[i]]++] = v;
    }
    while (!work.empty()) {
      uint32_t c = work.back();
      work.pop_back();
      for (uint64_t i = roff[c]; i < roff[c + 1]; i++) {
        uint32_t p = radj[i];
        if (!(flags[p] & NF_IMPURE)) {
          flags[p] |= NF_IMPURE;
          work.push_back(p);
        }
      }
    }
  }
  // 4. upload
  uint64_t *d_ro, *d_ao;
  uint32_t *d_rs, *d_adj, *d_ns, *d_obj, *d_rel;
  if (alloc((void**)&d_ro, ((size_t)nn + 1) * 8) || alloc((void**)&d_ao, ((size_t)nn + 1) * 8) ||
      alloc((void**)&d_rs, h_row_subj.size() * 4) || alloc((void**)&d_adj, adj.size() * 4) || alloc((void**)&d_ns, (size_t)nn * 4) ||
      alloc((void**)&d_obj, (size_t)nn * 4) || alloc((void**)&d_rel, (size_t)nn * 4))
    return -1;
  HIPC(hipMemcpy(d_ro, h_row_off.data(), ((size_t)nn + 1) * 8, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d_ao, h_adj_off.data(), ((size_t)nn + 1) * 8, hipMemcpyHostToDevice));
  if (!h_row_subj.empty())
    HIPC(hipMemcpy(d_rs, h_row_subj.data(), h_row_subj.size() * 4, hipMemcpyHostToDevice));
  if (!adj.empty()) HIPC(hipMemcpy(d_adj, adj.data(), adj.size() * 4, hipMemcpyHostToDevice));
  if (nn) {
    HIPC(hipMemcpy(d_ns, h_nd_ns.data(), (size_t)nn * 4, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_obj, h_nd_obj.data(), (size_t)nn * 4, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_rel, h_nd_rel.data(), (size_t)nn * 4, hipMemcpyHostToDevice));
  }
  ds.row_off = d_ro;
  ds.adj_off = d_ao;
  ds.row_subj = d_rs;
  ds.adj = d_adj;
  ds.nd_ns = d_ns;
  ds.nd_obj = d_obj;
  ds.nd_rel = d_rel;
  n_set_edges = adj.size();
  if (keys) {
    if (alloc((void**)&d_row_key, row_key.size() * 8 + 8)) return -1;
    if (!row_key.empty()) HIPC(hipMemcpy(d_row_key, row_key.data(), row_key.size() * 8, hipMemcpyHostToDevice));
  }
  ds.nflags = nullptr;
  if (has_program) {
    uint8_t* d_f;
    if (alloc((void**)&d_f, nn + 1)) return -1;
    if (nn) HIPC(hipMemcpy(d_f, flags.data(), nn, hipMemcpyHostToDevice));
    ds.nflags = d_f;
  }
  n_check_rows = h_row_off_last;
  if (augment_rewrites() || build_formulas()) return -1;
  return build_hash_tables();
}

int Snapshot::create_synthetic(const kg_synth_params* p, const kg_rewrite_prog* prog) {
  SynthLayout L{};
  const uint64_t T = p->n_tuples_target ? p->n_tuples_target : 10000000ull;
  if (p->preset > 1) return set_error(-2, "unknown synthetic preset %u", p->preset);
  if (!synth_make_layout(L, T, p->seed, p->n_layers, p->max_degree, p->set_fraction, p->doc_set_fraction, p->preset,
                         p->doc_alpha, p->group_alpha))
    return set_error(-2, "synthetic graph too large");
  if (const char* e = getenv("KG_SYNTH_IDENTITY")) L.pick_identity = atoi(e) ? 1u : 0u;  // experiment only
  synth = L;
  is_synth = true;
  wildcard_rel = 0;
  ds.wildcard_rel = 0;
  const uint32_t nn = L.n_nodes;
  ds.n_nodes = nn;
  uint64_t *deg, *setdeg, *d_ro, *d_ao;
  if (alloc((void**)&d_ro, ((size_t)nn + 1) * 8) || alloc((void**)&d_ao, ((size_t)nn + 1) * 8)) return -1;
  HIPC(hipMalloc(&deg, ((size_t)nn + 1) * 8));
  HIPC(hipMalloc(&setdeg, ((size_t)nn + 1) * 8));
  const uint32_t grid = (nn + 255) / 256;
  hipLaunchKernelGGL(k_synth_degrees, dim3(grid), dim3(256), 0, stream, L, nn, shard_rank, shard_n, deg, setdeg);
  HIPC(hipGetLastError());
  HIPC(hipMemsetAsync(deg + nn, 0, 8, stream));
  HIPC(hipMemsetAsync(setdeg + nn, 0, 8, stream));
  size_t tmp_bytes = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, deg, d_ro, nn + 1, stream));
  void* tmp;
  HIPC(hipMalloc(&tmp, tmp_bytes + 16));
  HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, deg, d_ro, nn + 1, stream));
  HIPC(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, setdeg, d_ao, nn + 1, stream));
  uint64_t tot[2];
  HIPC(hipMemcpyAsync(&tot[0], d_ro + nn, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipMemcpyAsync(&tot[1], d_ao + nn, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  HIPC(hipFree(tmp));
  HIPC(hipFree(deg));
  HIPC(hipFree(setdeg));
  uint32_t *d_rs, *d_adj, *d_ns, *d_obj, *d_rel;
  if (alloc((void**)&d_rs, tot[0] * 4) || alloc((void**)&d_adj, tot[1] * 4) || alloc((void**)&d_ns, (size_t)nn * 4) ||
      alloc((void**)&d_obj, (size_t)nn * 4) || alloc((void**)&d_rel, (size_t)nn * 4))
    return -1;
  hipLaunchKernelGGL(k_synth_fill, dim3(grid), dim3(256), 0, stream, L, nn, d_ro, d_ao, d_rs, d_adj, d_ns, d_obj,
                     d_rel);
  HIPC(hipGetLastError());
  ds.row_off = d_ro;
  ds.adj_off = d_ao;
  ds.row_subj = d_rs;
  ds.adj = d_adj;
  ds.nd_ns = d_ns;
  ds.nd_obj = d_obj;
  ds.nd_rel = d_rel;
  ds.nflags = nullptr;
  h_row_off_last = tot[0];
  n_set_edges = tot[1];
  kg_dict dict{4, 10, 0};
  if (upload_program(&dict, prog)) return -1;
  if (has_program && device_flags()) return -1;
  n_check_rows = h_row_off_last;
  if (augment_rewrites() || build_formulas()) return -1;
  return build_hash_tables();
}

// Purity closure on the device: seed with the relation flags, propagate "impure" backwards over
// set-adjacency to a fixed point (every round that changes something marks a node).
int Snapshot::device_flags() {
  const uint32_t nn = ds.n_nodes;
  uint8_t* f;
  uint32_t* changed;
  if (alloc((void**)&f, (size_t)nn + 1)) return -1;
  ds.nflags = nullptr;
  HIPC(hipMalloc(&changed, 4));
  const uint32_t grid = (nn + 255) / 256;
  if (nn) {
    hipLaunchKernelGGL(k_flags_init, dim3(grid), dim3(256), 0, stream, ds, f);
    for (uint64_t it = 0; it <= nn; it++) {
      uint32_t h = 0;
      HIPC(hipMemsetAsync(changed, 0, 4, stream));
      hipLaunchKernelGGL(k_flags_propagate, dim3(grid), dim3(256), 0, stream, ds, f, changed);
      HIPC(hipMemcpyAsync(&h, changed, 4, hipMemcpyDeviceToHost, stream));
      HIPC(hipStreamSynchronize(stream));
      if (!h) break;
    }
  }
  HIPC(hipFree(changed));
  ds.nflags = f;
  return 0;
}

int64_t Snapshot::export_rows(kg_tuple* out, uint64_t cap) {
  uint64_t n = h_row_off_last;
  if (!out) return (int64_t)n;
  if (cap < n) return set_error(-3, "export buffer too small (%llu < %llu)", (unsigned long long)cap,
                                (unsigned long long)n);
  uint32_t nn = ds.n_nodes;
  std::vector<uint64_t> off((size_t)nn + 1);
  std::vector<uint32_t> subj(n), ns(nn), obj(nn), rel(nn);
  HIPC(hipMemcpy(off.data(), ds.row_off, ((size_t)nn + 1) * 8, hipMemcpyDeviceToHost));
  if (n) HIPC(hipMemcpy(subj.data(), ds.row_subj, n * 4, hipMemcpyDeviceToHost));
  if (nn) {
    HIPC(hipMemcpy(ns.data(), ds.nd_ns, (size_t)nn * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(obj.data(), ds.nd_obj, (size_t)nn * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(rel.data(), ds.nd_rel, (size_t)nn * 4, hipMemcpyDeviceToHost));
  }
  for (uint32_t v = 0; v < nn; v++)
    for (uint64_t i = off[v]; i < off[v + 1]; i++) {
      kg_tuple& t = out[i];
      t.ns = ns[v];
      t.obj = obj[v];
      t.rel = rel[v];
      uint32_t s = subj[i];
      if (s & SET_BIT) {
        uint32_t c = s & ~SET_BIT;
        t.sns = ns[c];
        t.sobj = obj[c];
        t.srel = rel[c];
      } else {
        t.sns = KG_SUBJECT_ID;
        t.sobj = s;
        t.srel = 0;
      }
    }
  return (int64_t)n;
}

}  // namespace kg
