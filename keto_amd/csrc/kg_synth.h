// kg_synth.h -- deterministic synthetic "Drive-like" tuple graphs,
// generated directly in HBM.  Every row is a pure function of (seed, node, edge index), so the
// device build and kg_snapshot_export / the CPU oracle see exactly the same rows.
//
// A graph is a list of node blocks.  Block b owns node ids [node0, node0+count); node v is the
// tuple row (ns, obj0 + (v - node0), rel).  Its out-degree follows a truncated power law (or is
// fixed / empty with probability p_empty) and each subject is, with probability p_set, a subject
// set of the block's set kind, else a user id (log-uniform = Zipf(~1) popularity, permuted).
//
//   preset 0 (C2/C4): doc#viewer -> users | L0 group#member;  group#member (8 layers, L_l -> L_l+1)
//   preset 1 (C3)   : preset 0 + doc#{editor,owner,parents,blocked}, folder#{viewer,editor,owner,
//                     parents,...} with a 4-ary folder forest (depth <= 8) and the OPL program
//                     view = viewer | edit | parents.traverse(view); edit = editor | owner |
//                     parents.traverse(edit); share = view & !blocked (built by keto_amd.synth).
#pragma once
#include <math.h>
#include <stdint.h>

#include "kg_internal.h"

namespace kg {

enum : uint8_t { SK_NONE = 0, SK_GROUP_LAYER = 1, SK_FOLDER_ANY = 2, SK_FOLDER_PARENT = 3 };

struct SynthBlock {
  uint32_t node0, count;
  uint32_t ns, rel, obj0;
  float inv_s;       // 1/(s-1) of the degree power law; 0 => fixed degree
  uint32_t fixed_deg;
  float p_empty;     // row empty with this probability
  float p_set;       // subject is a set of `set_kind` with this probability
  uint32_t set_kind, set_arg;
};

constexpr int SYNTH_MAX_BLOCKS = 24;

struct SynthLayout {
  uint64_t seed;
  uint32_t preset;
  uint32_t n_docs, n_groups, n_users, n_layers, group_per_layer, n_folders;
  uint32_t max_degree;
  uint32_t user_obj0, folder_obj0;
  uint32_t group_node0, folder_any_node0;  // first node of group layer 0 / of folder#...
  uint32_t n_nodes, n_blocks;
  SynthBlock b[SYNTH_MAX_BLOCKS];
  // ids (interned by keto_amd.synth in this order)
  uint32_t ns_doc, ns_group, ns_user, ns_folder;
  // experiment (env KG_SYNTH_IDENTITY=1, kg_snapshot.hip): popularity rank r IS the id -- hot groups and
  // users at the front of their ranges, the layout an in-degree relabelling of the snapshot would give
  uint32_t pick_identity;
  uint32_t rel_viewer, rel_member, rel_editor, rel_owner, rel_parents, rel_blocked, rel_view, rel_edit, rel_share;
};

__host__ __device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
__host__ __device__ __forceinline__ uint64_t shash(uint64_t seed, uint64_t a, uint64_t b) {
  return mix64(seed ^ mix64(a * 0x9E3779B97F4A7C15ull + b * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull));
}
// log-uniform rank (Zipf(~1) popularity) mapped through an affine permutation of [0, n)
__host__ __device__ __forceinline__ uint32_t synth_pick(uint64_t h, uint32_t n, uint32_t identity = 0) {
  double u = u01(h);
  uint64_t r = (uint64_t)floor(exp(u * log((double)n + 1.0))) - 1;
  if (r >= n) r = n - 1;
  return identity ? (uint32_t)r : (uint32_t)((r * 2654435761ull + 12345ull) % n);
}

__host__ __device__ __forceinline__ int synth_block_of(const SynthLayout& L, uint32_t v) {
  int lo = 0, hi = (int)L.n_blocks;  // blocks are contiguous and ordered by node0
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (L.b[mid].node0 <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

__host__ __device__ __forceinline__ uint32_t synth_degree(const SynthLayout& L, uint32_t v) {
  const SynthBlock& B = L.b[synth_block_of(L, v)];
  const uint64_t h = shash(L.seed, v, 0xDE6);
  if (B.p_empty > 0.f && u01(shash(L.seed, v, 0xE3)) < B.p_empty) return 0;
  if (B.set_kind == SK_FOLDER_PARENT && v - B.node0 == 0) return 0;  // forest root
  if (B.inv_s == 0.f) return B.fixed_deg;
  double k = floor(pow(1.0 - u01(h), -(double)B.inv_s));
  if (k < 1) k = 1;
  if (k > L.max_degree) k = L.max_degree;
  return (uint32_t)k;
}

// Subject of tuple e of node v: tagged (SET_BIT | node) or a user object id.
__host__ __device__ __forceinline__ uint32_t synth_subject(const SynthLayout& L, uint32_t v, uint32_t e) {
  const SynthBlock& B = L.b[synth_block_of(L, v)];
  const uint64_t h1 = shash(L.seed, ((uint64_t)v << 20) ^ e, 1);
  const uint64_t h2 = shash(L.seed, ((uint64_t)v << 20) ^ e, 2);
  if (B.set_kind != SK_NONE && u01(h1) < B.p_set) {
    switch (B.set_kind) {
      case SK_GROUP_LAYER:
        return SET_BIT | (L.group_node0 + B.set_arg * L.group_per_layer + synth_pick(h2, L.group_per_layer, L.pick_identity));
      case SK_FOLDER_ANY:
        return SET_BIT | (L.folder_any_node0 + (uint32_t)(h2 % L.n_folders));
      case SK_FOLDER_PARENT:  // 4-ary forest: folder i's parent is (i-1)/4
        return SET_BIT | (L.folder_any_node0 + (v - B.node0 - 1) / 4);
    }
  }
  return L.user_obj0 + synth_pick(h2, L.n_users, L.pick_identity);
}

__host__ __device__ __forceinline__ void synth_node(const SynthLayout& L, uint32_t v, uint32_t& ns, uint32_t& obj,
                                                    uint32_t& rel) {
  const SynthBlock& B = L.b[synth_block_of(L, v)];
  ns = B.ns;
  obj = B.obj0 + (v - B.node0);
  rel = B.rel;
}

// Builds the block list for a preset; returns false if ids would overflow.
inline bool synth_make_layout(SynthLayout& L, uint64_t T, uint64_t seed, uint32_t n_layers, uint32_t max_degree,
                              float set_frac, float doc_set_frac, uint32_t preset, float doc_alpha = 0.f,
                              float group_alpha = 0.f) {
  // out-degrees: truncated Pareto with tail index alpha (CCDF ~ k^-alpha), default 1.3 (docs) and
  // 1.1 (groups): mean ~4-10 edges per row at max_degree 1e5, so a "1 B tuples" target holds
  // ~0.95 B rows.  alpha 0.5 is the degree law P(k) ~ k^-1.5 (Zipf 1.5) SURVEY.md 8d names; its
  // mean is ~sqrt(max_degree), i.e. ~40x the rows per node (the --heavy-tail bench point)
  const float inv_doc = 1.f / (doc_alpha > 0.f ? doc_alpha : 1.3f);
  const float inv_group = 1.f / (group_alpha > 0.f ? group_alpha : 1.1f);
  L = SynthLayout{};
  L.seed = seed;
  L.preset = preset;
  L.n_layers = n_layers ? n_layers : 8;
  L.n_docs = (uint32_t)(T / 8 > 0 ? T / 8 : 1);
  L.group_per_layer = (uint32_t)(T / 16 / L.n_layers > 0 ? T / 16 / L.n_layers : 1);
  L.n_groups = L.group_per_layer * L.n_layers;
  L.n_users = (uint32_t)(T / 10 > 0 ? T / 10 : 1);
  L.n_folders = preset == 1 ? (uint32_t)(T / 100 > 4 ? T / 100 : 4) : 0;
  if (preset == 1 && L.n_folders > 87381) L.n_folders = 87381;  // 4-ary forest depth <= 8
  L.max_degree = max_degree ? max_degree : 100000;
  L.ns_doc = 0;
  L.ns_group = 1;
  L.ns_user = 2;
  L.ns_folder = 3;
  L.rel_viewer = 1;  // rel 0 = "..." (keto_amd.mapper.Interner reserves it first)
  L.rel_member = 2;
  L.rel_editor = 3;
  L.rel_owner = 4;
  L.rel_parents = 5;
  L.rel_blocked = 6;
  L.rel_view = 7;
  L.rel_edit = 8;
  L.rel_share = 9;
  L.user_obj0 = L.n_docs + L.n_groups;
  L.folder_obj0 = L.user_obj0 + L.n_users;
  if ((uint64_t)L.folder_obj0 + L.n_folders >= 0x7FFFFFFFull) return false;
  uint32_t node = 0;
  int nb = 0;
  auto add = [&](uint32_t count, uint32_t ns, uint32_t rel, uint32_t obj0, float inv_s, uint32_t fixed, float p_empty,
                 float p_set, uint32_t kind, uint32_t arg) {
    L.b[nb++] = SynthBlock{node, count, ns, rel, obj0, inv_s, fixed, p_empty, p_set, kind, arg};
    node += count;
  };
  // C2 core (identical ids and hash streams for every preset)
  add(L.n_docs, L.ns_doc, L.rel_viewer, 0, inv_doc, 0, 0.f, doc_set_frac > 0 ? doc_set_frac : 0.5f,
      SK_GROUP_LAYER, 0);
  L.group_node0 = node;
  for (uint32_t l = 0; l < L.n_layers; l++)
    add(L.group_per_layer, L.ns_group, L.rel_member, L.n_docs + l * L.group_per_layer, inv_group, 0, 0.f,
        l + 1 < L.n_layers ? (set_frac > 0 ? set_frac : 0.25f) : 0.f, l + 1 < L.n_layers ? SK_GROUP_LAYER : SK_NONE,
        l + 1);
  if (preset == 1) {
    add(L.n_docs, L.ns_doc, L.rel_editor, 0, 1.f / 2.0f, 0, 0.3f, 0.3f, SK_GROUP_LAYER, 0);
    add(L.n_docs, L.ns_doc, L.rel_owner, 0, 0.f, 1, 0.f, 0.f, SK_NONE, 0);
    add(L.n_docs, L.ns_doc, L.rel_parents, 0, 0.f, 1, 0.1f, 1.f, SK_FOLDER_ANY, 0);
    add(L.n_docs, L.ns_doc, L.rel_blocked, 0, 0.f, 1, 0.9f, 0.f, SK_NONE, 0);
    add(L.n_folders, L.ns_folder, L.rel_viewer, L.folder_obj0, 1.f / 1.3f, 0, 0.2f, 0.5f, SK_GROUP_LAYER, 0);
    add(L.n_folders, L.ns_folder, L.rel_editor, L.folder_obj0, 1.f / 2.0f, 0, 0.5f, 0.3f, SK_GROUP_LAYER, 0);
    add(L.n_folders, L.ns_folder, L.rel_owner, L.folder_obj0, 0.f, 1, 0.f, 0.f, SK_NONE, 0);
    add(L.n_folders, L.ns_folder, L.rel_parents, L.folder_obj0, 0.f, 1, 0.f, 1.f, SK_FOLDER_PARENT, 0);
    L.folder_any_node0 = node;
    add(L.n_folders, L.ns_folder, 0 /* "..." */, L.folder_obj0, 0.f, 0, 1.f, 0.f, SK_NONE, 0);
  }
  L.n_blocks = (uint32_t)nb;
  L.n_nodes = node;
  return true;
}

}  // namespace kg
