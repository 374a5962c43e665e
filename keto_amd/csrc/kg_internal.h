// kg_internal.h -- shared definitions of libketogpu (host + device).
//
// HBM layout of a snapshot (all arrays device-resident, built once, immutable afterwards):
//   adj_off[n_nodes+1] u64 / adj[] u32   set-adjacency: per node (ns,obj,rel) the subject-set
//                                        subjects that checkExpandSubject recurses into
//                                        (internal/check/engine.go:118-136: SubjectIDs and "..."
//                                        sets skipped), kept in shard_id order.
//   row_off[n_nodes+1] u64 / row_subj[]   full rows (every subject, tagged), shard_id order: expand
//                                        (internal/expand/engine.go:57-94) and tuple-to-subject-set.
//   dset                                  bucketed hash set of (node << 32 | tagged subject):
//                                        checkDirect's exact-tuple query (engine.go:159-163).
//   nmap                                  (ns,rel,obj) -> node id, for request mapping on device.
//   nflags[n_nodes] u8                    bit0 IMPURE: a rewrite / undeclared relation is reachable
//                                        through set-adjacency (needs the rewrite interpreter).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace kg {

constexpr uint32_t SET_BIT = 0x80000000u;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t EMPTY64 = ~0ull;
constexpr int DSET_BUCKET = 8;  // u64 keys per bucket = one 64-B sector

enum : uint8_t { NF_IMPURE = 1, NF_REWRITE = 2, NF_ERR = 4 };

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

__host__ __device__ __forceinline__ uint64_t nmap_key(uint32_t ns, uint32_t rel, uint32_t obj) {
  return ((uint64_t)((ns << 16) | (rel & 0xFFFFu)) << 32) | obj;
}
__host__ __device__ __forceinline__ uint64_t dset_key(uint32_t node, uint32_t subj) {
  return ((uint64_t)node << 32) | subj;
}

// Rewrite-program node (kg_rw_node layout).
struct RwNode {
  int32_t kind, rel, crel, first, count;
};
enum { RW_OR = 0, RW_AND = 1, RW_COMPUTED = 2, RW_TTU = 3, RW_NOT = 4 };

// Everything a kernel needs, passed by value.
struct DevSnap {
  uint32_t n_nodes;
  uint32_t wildcard_rel;
  const uint64_t* adj_off;
  const uint32_t* adj;
  const uint64_t* row_off;
  const uint32_t* row_subj;
  const uint64_t* dset;
  uint64_t dset_mask;  // n_buckets - 1
  const uint64_t* nmap_keys;
  const uint32_t* nmap_vals;
  uint64_t nmap_mask;  // n_slots - 1
  const uint8_t* nflags;  // nullptr: every node pure
  const uint32_t* nd_ns;
  const uint32_t* nd_obj;
  const uint32_t* nd_rel;
  // program: relation flags [n_ns * n_rel] (bit0 has rewrite, bit1 undeclared->error), roots
  uint32_t n_ns, n_rel;
  const uint8_t* ns_has_rel;  // [n_ns]: configured with relations (unknown relation ids -> error)
  const uint8_t* relflags;
  const int32_t* relroot;
  const RwNode* rw;
  const int32_t* rwchild;
  uint32_t n_rw;
};

// astRelationFor (internal/check/engine.go:209-229) as flags: bit0 = has rewrite, bit1 = the
// namespace is configured with relations and this one is not declared ("relation %q not found").
// Unknown namespaces and namespaces without relations accept every relation without rewrite.
__host__ __device__ __forceinline__ uint8_t relflag(const DevSnap& s, uint32_t ns, uint32_t rel) {
  if (!s.relflags || ns >= s.n_ns) return 0;
  if (rel >= s.n_rel) return s.ns_has_rel[ns] ? 2 : 0;
  return s.relflags[(size_t)ns * s.n_rel + rel];
}

// Resolved query as stored in HBM by the mapping kernel.
struct RQuery {
  uint32_t node;   // root node id or NONE
  uint32_t subj;   // tagged subject or NONE
  int32_t depth;   // clamped rest depth
  uint32_t route;  // ROUTE_*
};
enum : uint32_t { ROUTE_DONE = 0, ROUTE_LIGHT = 1, ROUTE_GENERAL = 2 };

// ---------------------------------------------------------------- synthetic graph
// Deterministic "Drive-like" generator: pure function of (seed, index) so
// the device build and kg_snapshot_export / the oracle see the same rows.
struct SynthLayout {
  uint64_t seed;
  uint32_t n_docs, n_groups, n_users, n_layers, group_per_layer;
  uint32_t max_degree;
  float set_frac, doc_set_frac;
  // ids
  uint32_t ns_doc, ns_group, ns_user, rel_viewer, rel_member;
};

__host__ __device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
__host__ __device__ __forceinline__ uint64_t shash(uint64_t seed, uint64_t a, uint64_t b) {
  return mix64(seed ^ mix64(a * 0x9E3779B97F4A7C15ull + b * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull));
}
// truncated power-law out-degree: floor((1-u)^(-1/(s-1))), s = 2.1 (groups, mean ~7.5) / 2.3 (docs, ~3.9)
__host__ __device__ __forceinline__ uint32_t synth_degree(const SynthLayout& L, uint32_t node) {
  bool doc = node < L.n_docs;
  double u = u01(shash(L.seed, node, 0xDE6));
  double inv = doc ? (1.0 / 1.3) : (1.0 / 1.1);
  double k = floor(pow(1.0 - u, -inv));
  if (k < 1) k = 1;
  if (k > L.max_degree) k = L.max_degree;
  return (uint32_t)k;
}
// log-uniform rank (Zipf(~1) popularity) mapped through an affine permutation of [0, n)
__host__ __device__ __forceinline__ uint32_t synth_pick(uint64_t h, uint32_t n) {
  double u = u01(h);
  uint64_t r = (uint64_t)floor(exp(u * log((double)n + 1.0))) - 1;
  if (r >= n) r = n - 1;
  return (uint32_t)((r * 2654435761ull + 12345ull) % n);
}
__host__ __device__ __forceinline__ uint32_t synth_layer(const SynthLayout& L, uint32_t node) {
  return (node - L.n_docs) / L.group_per_layer;
}
// Subject of tuple e of node: tagged (SET_BIT | group node) or a user object id.
__host__ __device__ __forceinline__ uint32_t synth_subject(const SynthLayout& L, uint32_t node, uint32_t e) {
  uint64_t h1 = shash(L.seed, ((uint64_t)node << 20) ^ e, 1);
  uint64_t h2 = shash(L.seed, ((uint64_t)node << 20) ^ e, 2);
  bool doc = node < L.n_docs;
  uint32_t layer = doc ? 0 : synth_layer(L, node);
  bool set;
  uint32_t tgt_layer;
  if (doc) {
    set = u01(h1) < L.doc_set_frac;
    tgt_layer = 0;
  } else {
    set = (layer + 1 < L.n_layers) && u01(h1) < L.set_frac;
    tgt_layer = layer + 1;
  }
  if (set) {
    uint32_t g = synth_pick(h2, L.group_per_layer);
    return SET_BIT | (L.n_docs + tgt_layer * L.group_per_layer + g);
  }
  return L.n_docs + L.n_groups + synth_pick(h2, L.n_users);  // user object id
}

}  // namespace kg
