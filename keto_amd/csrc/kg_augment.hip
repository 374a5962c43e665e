// kg_augment.hip -- rewrite materialisation: monotone rewrites become plain reachability.
//
// The rewrite interpreter (kg_interp.hip) evaluates internal/check/rewrites.go one wave per query.
// Most real namespace configs are unions: C3's `view = viewer | edit | parents.traverse(view)`,
// `edit = editor | owner | parents.traverse(edit)`.  For such a relation R of namespace ns the
// reference's recursion (engine.go:183-207 + rewrites.go:30-260) at rest depth d is
//
//   checkIsAllowed((ns,obj,R), d) =   direct(r, d-1) | expand(r, d)          for r in Z(R)
//                                    | checkIsAllowed((s.ns, s.obj, c), d-1)  for (t, c) in T(R),
//                                                                             s a subject set in rows (ns,obj,t)
//
// where Z(R) is R plus every relation reachable from R's rewrite through `or` / computed subject
// sets (same object, same depth: rewrites.go:167-193) and T(R) the tuple-to-subject-set pairs met on
// the way (one hop: rewrites.go:205-260).  That is exactly checkIsAllowed of ONE plain node whose
// set-adjacency row is the union of the Z nodes' rows plus the TTU targets, and whose direct tuples
// are the union of the Z nodes' rows.  So every object with such a relation gets a virtual node
// V(ns,obj,R) with that merged row (replacing the plain node (ns,obj,R) when it exists, new id
// otherwise), and queries and subject-set edges that reach it run in the rewrite-free tiers
// (k_resolve -> k_stream2 -> k_back -> grid) instead of the interpreter.
//
// A relation is materialised only when the rewrite is a pure union (no and / not: rewrites.go:95,
// binop.go:50), its computed relations are declared (no "relation not found", engine.go:228) and
// acyclic (a computed cycle is KG_ERR_REWRITE_CYCLE), and Z / T are small.  Per object, V is pure
// only if no TTU target reaches a relation that is undeclared or an unmaterialised rewrite, and no
// node it reaches is impure -- decided by a fixpoint over the augmented graph; impure V keep the
// original rows and the interpreter evaluates them (it sees pure V below them as plain nodes).
// The raw rows (row_off / row_subj: expand, tuple-to-subject-set, export) are never changed; the
// check structures (set-adjacency, the direct-tuple set, holders, node map) are rebuilt from the
// augmented graph by build_hash_tables.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "kg_bfs.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

constexpr int AUG_Z = 12, AUG_T = 8, AUG_L = AUG_Z + AUG_T;

struct AugPlan {
  uint32_t ns, R;
  uint32_t nz, nt, nl;
  uint32_t z[AUG_Z];                 // Z(R), R first
  uint32_t tt[AUG_T], tc[AUG_T];     // T(R): (tuple relation, computed relation)
  uint32_t l[AUG_L];                 // anchor order: Z then the TTU tuple relations not in Z
};

struct AugTables {
  const AugPlan* plans;
  uint32_t n_plans;
  const uint32_t* c_off;   // [n_ns * n_rel + 1]: plans a (ns, rel) node contributes to
  const uint32_t* c_list;
  const uint8_t* virt;     // [n_ns * n_rel]: 1 = a materialised (virtualizable) rewrite relation
};

__device__ __forceinline__ uint32_t aug_pair(const DevSnap& s, uint32_t ns, uint32_t rel) {
  return (ns < s.n_ns && rel < s.n_rel) ? ns * s.n_rel + rel : NONE;
}

// A TTU target relation c in namespace tns is irreducible when checkIsAllowed on it could give an
// error or a non-monotone answer: undeclared, or a rewrite that is not materialised.
__device__ __forceinline__ bool aug_target_bad(const DevSnap& s, const AugTables& A, uint32_t tns, uint32_t c) {
  const uint8_t f = relflag(s, tns, c);
  if (f & 2) return true;
  if (f & 1) {
    const uint32_t pr = aug_pair(s, tns, c);
    return pr == NONE || !A.virt[pr];
  }
  return false;
}

// ---- 1. candidates: one per (plan, object) with any contributing node; emitted by its anchor (the
// first relation of the plan's order whose node exists), so no dedup table is needed.  Pass 1
// counts per anchor node, a scan places them: candidate order (hence new node ids) is a function of
// the node triples alone, the same on every rank of the hash-sharded mode.
template <bool FILL>
__global__ void k_aug_cands(DevSnap s, AugTables A, uint32_t n0, uint32_t* count, const uint64_t* cpos,
                            uint32_t* c_plan, uint32_t* c_obj, uint32_t* c_base) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n0) return;
  uint32_t k = 0;
  const uint32_t ns = s.nd_ns[v], rel = s.nd_rel[v], obj = s.nd_obj[v];
  const uint32_t pr = aug_pair(s, ns, rel);
  if (!FILL) count[v] = 0;
  if (pr == NONE) return;
  for (uint32_t i = A.c_off[pr]; i < A.c_off[pr + 1]; i++) {
    const uint32_t p = A.c_list[i];
    const AugPlan& P = A.plans[p];
    uint32_t pos = 0;
    while (pos < P.nl && P.l[pos] != rel) pos++;
    bool anchor = true;
    for (uint32_t j = 0; j < pos && anchor; j++)
      if (nmap_find(s, ns, P.l[j], obj) != NONE) anchor = false;
    if (!anchor) continue;
    if (FILL) {
      const uint64_t at = cpos[v] + k;
      c_plan[at] = p;
      c_obj[at] = obj;
      c_base[at] = rel == P.R ? v : NONE;  // the plain node (ns,obj,R) exists: V replaces it
    }
    k++;
  }
  if (!FILL) count[v] = k;
}

// ---- 2. ids: replaced candidates keep the plain node id, new ones are appended after n0 in
// candidate order (new_pos: exclusive scan of "is new")
__global__ void k_aug_isnew(uint32_t nc, const uint32_t* c_base, uint32_t* is_new) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nc) is_new[k] = c_base[k] == NONE ? 1u : 0u;
}
__global__ void k_aug_ids(DevSnap s, AugTables A, uint32_t nc, uint32_t n0, const uint32_t* c_plan,
                          const uint32_t* c_obj, const uint32_t* c_base, const uint64_t* new_pos, uint32_t* c_id,
                          uint32_t* cand_of, uint32_t* nd_ns, uint32_t* nd_obj, uint32_t* nd_rel) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nc) return;
  const AugPlan& P = A.plans[c_plan[k]];
  uint32_t id = c_base[k];
  if (id == NONE) {
    id = n0 + (uint32_t)new_pos[k];
    nd_ns[id] = P.ns;
    nd_obj[id] = c_obj[k];
    nd_rel[id] = P.R;
  }
  c_id[k] = id;
  cand_of[id] = k;
}

// Node map over every node (keys only: the values are filled by build_hash_tables' rebuild).
__global__ void k_aug_nmap(NSlot* nm, uint64_t slots, const uint32_t* nd_ns, const uint32_t* nd_obj,
                           const uint32_t* nd_rel, uint32_t n) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const uint64_t key = nmap_key(nd_ns[v], nd_rel[v], nd_obj[v]);
  uint64_t i = hash_home(key, slots);
  for (uint64_t p = 0; p < slots; p++) {
    const unsigned long long old =
        atomicCAS((unsigned long long*)&nm[i].key, (unsigned long long)EMPTY64, (unsigned long long)key);
    if (old == EMPTY64 || old == key) {
      nm[i].node = v;
      return;
    }
    i = hash_next(i, slots);
  }
}

// Walks the merged successor set of candidate k (Z-node set rows, then TTU targets), calling f(child).
// Returns false when a TTU target is irreducible.
template <class F>
__device__ __forceinline__ bool aug_succ(const DevSnap& s, const DevSnap& base, const AugTables& A, const AugPlan& P,
                                         uint32_t obj, F&& f) {
  bool ok = true;
  for (uint32_t j = 0; j < P.nz; j++) {
    const uint32_t u = nmap_find(s, P.ns, P.z[j], obj);
    if (u == NONE || u >= base.n_nodes) continue;  // new nodes have no rows of their own
    for (uint64_t i = base.adj_off[u], e = base.adj_off[u + 1]; i < e; i++) f(base.adj[i]);
  }
  for (uint32_t j = 0; j < P.nt; j++) {
    const uint32_t u = nmap_find(s, P.ns, P.tt[j], obj);
    if (u == NONE || u >= base.n_nodes) continue;
    for (uint64_t i = base.row_off[u], e = base.row_off[u + 1]; i < e; i++) {
      const uint32_t sub = base.row_subj[i];
      if (!(sub & SET_BIT)) continue;  // rewrites.go:228-257: subject sets only, any relation
      const uint32_t sn = sub & ~SET_BIT;
      const uint32_t tns = base.nd_ns[sn];
      if (aug_target_bad(s, A, tns, P.tc[j])) ok = false;
      const uint32_t tgt = nmap_find(s, tns, P.tc[j], base.nd_obj[sn]);
      if (tgt != NONE) f(tgt);  // no node: checkIsAllowed on it is NotMember (no rows, no rewrite)
    }
  }
  return ok;
}

// ---- 3. purity: seeds, then "impure if a successor is impure" to a fixpoint
__global__ void k_aug_seed(DevSnap s, DevSnap base, AugTables A, uint32_t n1, const uint32_t* cand_of,
                           const uint32_t* c_plan, const uint32_t* c_obj, uint8_t* imp, uint32_t rank,
                           uint32_t nranks) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n1) return;
  const uint32_t k = cand_of[v];
  if (k == NONE) {  // a plain node: a rewrite that is not materialised, or an undeclared relation
    imp[v] = relflag(s, s.nd_ns[v], s.nd_rel[v]) != 0 ? 1 : 0;
    return;
  }
  const AugPlan& P = A.plans[c_plan[k]];
  if (nranks > 1 && shard_owner(P.ns, c_obj[k], nranks) != rank) {
    // hash-sharded mode: the object's rows (its TTU tuple rows among them) live on its owner, which
    // decides; records reach a node only at its owner, so no other rank reads this flag for a check
    imp[v] = 0;
    return;
  }
  imp[v] = aug_succ(s, base, A, P, c_obj[k], [](uint32_t) {}) ? 0 : 1;
}

__global__ void k_aug_propagate(DevSnap s, DevSnap base, AugTables A, uint32_t n1, const uint32_t* cand_of,
                                const uint32_t* c_plan, const uint32_t* c_obj, uint8_t* imp, uint32_t* changed) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n1 || imp[v]) return;
  bool bad = false;
  const uint32_t k = cand_of[v];
  if (k == NONE) {
    if (v < base.n_nodes)
      for (uint64_t i = base.adj_off[v], e = base.adj_off[v + 1]; i < e && !bad; i++) bad = imp[base.adj[i]] != 0;
  } else {
    aug_succ(s, base, A, A.plans[c_plan[k]], c_obj[k], [&](uint32_t c) { bad |= imp[c] != 0; });
  }
  if (bad) {
    imp[v] = 1;
    *changed = 1;
  }
}

// ---- 4. row lengths of the augmented graph: merged rows for pure candidates, else the plain ones
__global__ void k_aug_len(DevSnap s, DevSnap base, AugTables A, uint32_t n1, const uint32_t* cand_of,
                          const uint32_t* c_plan, const uint32_t* c_obj, const uint8_t* imp, uint64_t* adeg,
                          uint64_t* cdeg) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n1) return;
  const uint32_t k = cand_of[v];
  uint64_t a = 0, c = 0;
  if (k != NONE && !imp[v]) {
    const AugPlan& P = A.plans[c_plan[k]];
    aug_succ(s, base, A, P, c_obj[k], [&](uint32_t) { a++; });
    for (uint32_t j = 0; j < P.nz; j++) {
      const uint32_t u = nmap_find(s, P.ns, P.z[j], c_obj[k]);
      if (u != NONE && u < base.n_nodes) c += base.row_off[u + 1] - base.row_off[u];
    }
  } else if (v < base.n_nodes) {
    a = base.adj_off[v + 1] - base.adj_off[v];
    c = base.row_off[v + 1] - base.row_off[v];
  }
  adeg[v] = a;
  cdeg[v] = c;
}

__global__ void k_aug_fill(DevSnap s, DevSnap base, AugTables A, uint32_t n1, const uint32_t* cand_of,
                           const uint32_t* c_plan, const uint32_t* c_obj, const uint8_t* imp, const uint64_t* aoff,
                           const uint64_t* coff, uint32_t* adj, uint32_t* crow, uint64_t* roff, uint8_t* flags) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n1) return;
  const uint32_t k = cand_of[v];
  uint64_t a = aoff[v], c = coff[v];
  if (k != NONE && !imp[v]) {
    const AugPlan& P = A.plans[c_plan[k]];
    aug_succ(s, base, A, P, c_obj[k], [&](uint32_t ch) { adj[a++] = ch; });
    for (uint32_t j = 0; j < P.nz; j++) {
      const uint32_t u = nmap_find(s, P.ns, P.z[j], c_obj[k]);
      if (u == NONE || u >= base.n_nodes) continue;
      for (uint64_t i = base.row_off[u], e = base.row_off[u + 1]; i < e; i++) crow[c++] = base.row_subj[i];
    }
    flags[v] = 0;  // a pure materialised node: the rewrite-free tiers answer it
  } else {
    if (v < base.n_nodes) {
      for (uint64_t i = base.adj_off[v], e = base.adj_off[v + 1]; i < e; i++) adj[a++] = base.adj[i];
      for (uint64_t i = base.row_off[v], e = base.row_off[v + 1]; i < e; i++) crow[c++] = base.row_subj[i];
    }
    const uint8_t rf = relflag(s, s.nd_ns[v], s.nd_rel[v]);
    flags[v] = (uint8_t)((imp[v] ? NF_IMPURE : 0) | ((rf & 1) ? NF_REWRITE : 0) | ((rf & 2) ? NF_ERR : 0));
  }
  // raw rows: new nodes have none (expand / TTU / export see the original rows only)
  roff[v + 1] = v < base.n_nodes ? base.row_off[v + 1] : base.row_off[base.n_nodes];
  if (v == 0) roff[0] = 0;
}

// ------------------------------------------------------------------ host side
// Plans from the uploaded program (host mirrors of upload_program).
static bool aug_build_plans(const Snapshot* s, std::vector<AugPlan>& plans, std::vector<uint8_t>& virt) {
  const uint32_t n_ns = s->ds.n_ns, n_rel = s->ds.n_rel;
  virt.assign((size_t)n_ns * n_rel, 0);
  if (!s->has_program) return false;
  auto flag = [&](uint32_t ns, uint32_t r) -> uint8_t { return s->host_relflag(ns, r); };
  auto root = [&](uint32_t ns, uint32_t r) -> int32_t { return s->h_relroot[(size_t)ns * n_rel + r]; };
  for (uint32_t ns = 0; ns < n_ns; ns++)
    for (uint32_t R = 0; R < n_rel; R++) {
      if (!(flag(ns, R) & 1)) continue;
      AugPlan P{};
      P.ns = ns;
      P.R = R;
      bool ok = true;
      std::vector<uint32_t> z{R};
      std::vector<std::pair<uint32_t, uint32_t>> t;
      std::vector<std::pair<uint32_t, uint32_t>> comp;  // computed edges r -> c (cycle check)
      for (size_t zi = 0; zi < z.size() && ok; zi++) {
        const uint32_t r = z[zi];
        const int32_t rt = (flag(ns, r) & 1) ? root(ns, r) : -1;
        if (rt < 0) continue;
        std::vector<int32_t> st{rt};
        while (!st.empty() && ok) {
          const int32_t idx = st.back();
          st.pop_back();
          if (idx < 0 || (size_t)idx >= s->h_rw.size()) {
            ok = false;
            break;
          }
          const RwNode w = s->h_rw[(size_t)idx];
          if (w.kind == RW_OR) {
            if (w.first < 0 || w.count < 0 || (size_t)w.first + (size_t)w.count > s->h_rwchild.size()) {
              ok = false;
              break;
            }
            for (int32_t c = 0; c < w.count; c++) st.push_back(s->h_rwchild[(size_t)(w.first + c)]);
          } else if (w.kind == RW_COMPUTED) {
            const uint32_t c = (uint32_t)w.rel;
            if (w.rel < 0 || c >= n_rel || (flag(ns, c) & 2)) {  // "relation not found"
              ok = false;
              break;
            }
            comp.emplace_back(r, c);
            if (std::find(z.begin(), z.end(), c) == z.end()) z.push_back(c);
          } else if (w.kind == RW_TTU) {
            if (w.rel < 0 || (uint32_t)w.rel >= n_rel || w.crel < 0) {
              ok = false;
              break;
            }
            const auto pr = std::make_pair((uint32_t)w.rel, (uint32_t)w.crel);
            if (std::find(t.begin(), t.end(), pr) == t.end()) t.push_back(pr);
          } else {
            ok = false;  // and / not: not a union
          }
        }
      }
      if (!ok || z.size() > (size_t)AUG_Z || t.size() > (size_t)AUG_T) continue;
      // computed cycles (a relation computed from itself at the same depth) -> not materialised
      bool cyc = false;
      for (uint32_t a : z) {
        std::vector<uint32_t> seen, st{a};
        while (!st.empty() && !cyc) {
          const uint32_t x = st.back();
          st.pop_back();
          for (auto& e : comp)
            if (e.first == x) {
              if (e.second == a) cyc = true;
              if (std::find(seen.begin(), seen.end(), e.second) == seen.end()) {
                seen.push_back(e.second);
                st.push_back(e.second);
              }
            }
        }
        if (cyc) break;
      }
      if (cyc) continue;
      P.nz = (uint32_t)z.size();
      for (size_t i = 0; i < z.size(); i++) P.z[i] = z[i];
      P.nt = (uint32_t)t.size();
      for (size_t i = 0; i < t.size(); i++) {
        P.tt[i] = t[i].first;
        P.tc[i] = t[i].second;
      }
      P.nl = 0;
      for (uint32_t r : z) P.l[P.nl++] = r;
      for (auto& pr : t)
        if (std::find(P.l, P.l + P.nl, pr.first) == P.l + P.nl) P.l[P.nl++] = pr.first;
      plans.push_back(P);
      virt[(size_t)ns * n_rel + R] = 1;
    }
  return !plans.empty();
}

int Snapshot::augment_rewrites() {
  std::vector<AugPlan> plans;
  std::vector<uint8_t> virt;
  const char* env = getenv("KG_MATERIALIZE");
  if (env && env[0] == '0') materialize = 0;
  if (!materialize || !aug_build_plans(this, plans, virt)) return 0;
  h_virt = virt;  // the formula splitter's leaves may be union relations (kg_formula.hip)
  if (alloc((void**)&d_virt, virt.size() + 1)) return -1;
  HIPC(hipMemcpy(d_virt, virt.data(), virt.size(), hipMemcpyHostToDevice));
  ds.virt = d_virt;
  if (ds.n_nodes == 0) return 0;
  const uint32_t n_ns = ds.n_ns, n_rel = ds.n_rel, n0 = ds.n_nodes;
  // contributions: (ns, rel) -> plans whose anchor order lists rel
  std::vector<std::vector<uint32_t>> contrib((size_t)n_ns * n_rel);
  for (uint32_t p = 0; p < plans.size(); p++)
    for (uint32_t j = 0; j < plans[p].nl; j++) contrib[(size_t)plans[p].ns * n_rel + plans[p].l[j]].push_back(p);
  std::vector<uint32_t> c_off(contrib.size() + 1, 0), c_list;
  for (size_t i = 0; i < contrib.size(); i++) {
    c_off[i + 1] = c_off[i] + (uint32_t)contrib[i].size();
    c_list.insert(c_list.end(), contrib[i].begin(), contrib[i].end());
  }
  std::vector<void*> tmp;  // freed at the end
  auto talloc = [&](void** p, size_t bytes) -> int {
    HIPC(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return 0;
  };
  auto cleanup = [&]() {
    for (void* p : tmp) hipFree(p);
    tmp.clear();
  };
  struct Guard {
    std::function<void()> f;
    ~Guard() { f(); }
  } guard{cleanup};
  AugPlan* d_plans;
  uint32_t *d_coff, *d_clist, *d_cnt;
  uint8_t* d_virt;
  if (talloc((void**)&d_plans, plans.size() * sizeof(AugPlan)) || talloc((void**)&d_coff, c_off.size() * 4) ||
      talloc((void**)&d_clist, c_list.size() * 4 + 4) || talloc((void**)&d_virt, virt.size()) ||
      talloc((void**)&d_cnt, 16))
    return -1;
  HIPC(hipMemcpy(d_plans, plans.data(), plans.size() * sizeof(AugPlan), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d_coff, c_off.data(), c_off.size() * 4, hipMemcpyHostToDevice));
  if (!c_list.empty()) HIPC(hipMemcpy(d_clist, c_list.data(), c_list.size() * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d_virt, virt.data(), virt.size(), hipMemcpyHostToDevice));
  const AugTables A{d_plans, (uint32_t)plans.size(), d_coff, d_clist, d_virt};
  // the base snapshot needs a node map for the anchor lookups: a keys-only one over the base nodes
  const uint64_t slots0 = std::max<uint64_t>(16, (uint64_t)n0 * 8 / 5);  // load 0.625
  NSlot* nm0;
  if (talloc((void**)&nm0, slots0 * sizeof(NSlot))) return -1;
  HIPC(hipMemsetAsync(nm0, 0xFF, slots0 * sizeof(NSlot), stream));
  hipLaunchKernelGGL(k_aug_nmap, dim3((n0 + 255) / 256), dim3(256), 0, stream, nm0, slots0, ds.nd_ns, ds.nd_obj,
                     ds.nd_rel, n0);
  DevSnap b = ds;  // the base graph (its node map: nm0)
  b.nmap = nm0;
  b.nmap_n = slots0;
  // 1. candidates: count per anchor node, scan, place
  uint32_t* ccount;
  uint64_t* cpos;
  if (talloc((void**)&ccount, ((size_t)n0 + 1) * 4) || talloc((void**)&cpos, ((size_t)n0 + 1) * 8)) return -1;
  hipLaunchKernelGGL((k_aug_cands<false>), dim3((n0 + 255) / 256), dim3(256), 0, stream, b, A, n0, ccount, nullptr,
                     nullptr, nullptr, nullptr);
  HIPC(hipMemsetAsync(ccount + n0, 0, 4, stream));
  size_t tb0 = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb0, ccount, cpos, (size_t)n0 + 1, stream));
  void* scr0;
  if (talloc(&scr0, tb0 + 16)) return -1;
  HIPC(hipcub::DeviceScan::ExclusiveSum(scr0, tb0, ccount, cpos, (size_t)n0 + 1, stream));
  uint64_t nc64 = 0;
  HIPC(hipMemcpyAsync(&nc64, cpos + n0, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  if (nc64 == 0) return 0;
  if (nc64 >= 0x7FFFFFFFull) return set_error(KG_ERR_RESOURCE_CODE, "too many union nodes");
  const uint32_t nc = (uint32_t)nc64;
  uint32_t *c_plan, *c_obj, *c_base, *c_id;
  if (talloc((void**)&c_plan, (size_t)nc * 4) || talloc((void**)&c_obj, (size_t)nc * 4) ||
      talloc((void**)&c_base, (size_t)nc * 4) || talloc((void**)&c_id, (size_t)nc * 4))
    return -1;
  hipLaunchKernelGGL((k_aug_cands<true>), dim3((n0 + 255) / 256), dim3(256), 0, stream, b, A, n0, nullptr,
                     (const uint64_t*)cpos, c_plan, c_obj, c_base);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(stream));
  tmp.erase(std::find(tmp.begin(), tmp.end(), (void*)nm0));  // the base node map is done with
  HIPC(hipFree(nm0));
  // 2. ids (new nodes after n0) and the node triples of the extended graph
  if ((uint64_t)n0 + nc >= 0x7FFFFFFFull) return set_error(KG_ERR_RESOURCE_CODE, "too many nodes after materialisation");
  const uint32_t nmax = n0 + nc;  // upper bound (replaced candidates take no new id)
  uint32_t *nd_ns, *nd_obj, *nd_rel, *cand_of;
  if (talloc((void**)&nd_ns, (size_t)nmax * 4) || talloc((void**)&nd_obj, (size_t)nmax * 4) ||
      talloc((void**)&nd_rel, (size_t)nmax * 4) || talloc((void**)&cand_of, (size_t)nmax * 4))
    return -1;
  HIPC(hipMemcpyAsync(nd_ns, ds.nd_ns, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipMemcpyAsync(nd_obj, ds.nd_obj, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipMemcpyAsync(nd_rel, ds.nd_rel, (size_t)n0 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipMemsetAsync(cand_of, 0xFF, (size_t)nmax * 4, stream));
  uint32_t* is_new;
  uint64_t* new_pos;
  if (talloc((void**)&is_new, ((size_t)nc + 1) * 4) || talloc((void**)&new_pos, ((size_t)nc + 1) * 8)) return -1;
  hipLaunchKernelGGL(k_aug_isnew, dim3((nc + 255) / 256), dim3(256), 0, stream, nc, (const uint32_t*)c_base, is_new);
  HIPC(hipMemsetAsync(is_new + nc, 0, 4, stream));
  size_t tb1 = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, is_new, new_pos, (size_t)nc + 1, stream));
  void* scr1;
  if (talloc(&scr1, tb1 + 16)) return -1;
  HIPC(hipcub::DeviceScan::ExclusiveSum(scr1, tb1, is_new, new_pos, (size_t)nc + 1, stream));
  hipLaunchKernelGGL(k_aug_ids, dim3((nc + 255) / 256), dim3(256), 0, stream, b, A, nc, n0, c_plan, c_obj, c_base,
                     (const uint64_t*)new_pos, c_id, cand_of, nd_ns, nd_obj, nd_rel);
  HIPC(hipGetLastError());
  uint64_t n_new64 = 0;
  HIPC(hipMemcpyAsync(&n_new64, new_pos + nc, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  const uint32_t n_new = (uint32_t)n_new64;
  const uint32_t n1 = n0 + n_new;
  // node map over every node of the extended graph (keys + ids) for the successor lookups
  const uint64_t slots1 = std::max<uint64_t>(16, (uint64_t)n1 * 8 / 5);
  NSlot* nm1;
  if (talloc((void**)&nm1, slots1 * sizeof(NSlot))) return -1;
  HIPC(hipMemsetAsync(nm1, 0xFF, slots1 * sizeof(NSlot), stream));
  hipLaunchKernelGGL(k_aug_nmap, dim3((n1 + 255) / 256), dim3(256), 0, stream, nm1, slots1, nd_ns, nd_obj, nd_rel,
                     n1);
  DevSnap x = ds;  // the extended graph's ids and node map
  x.n_nodes = n1;
  x.nmap = nm1;
  x.nmap_n = slots1;
  x.nd_ns = nd_ns;
  x.nd_obj = nd_obj;
  x.nd_rel = nd_rel;
  // 3. purity fixpoint
  uint8_t* imp;
  if (talloc((void**)&imp, (size_t)n1 + 16)) return -1;
  const uint32_t g1 = (n1 + 255) / 256;
  hipLaunchKernelGGL(k_aug_seed, dim3(g1), dim3(256), 0, stream, x, b, A, n1, cand_of, c_plan, c_obj, imp,
                     shard_rank, shard_n);
  HIPC(hipGetLastError());
  // hash-sharded mode: the closure needs every rank's rows, so only the seeds are marked -- by the
  // owner of each union node, from its own TTU rows (a target relation that is undeclared or an
  // unmaterialised rewrite, e.g. a formula reached through tuple-to-subject-set); a record reaches a
  // node at its owner, so the impure node (or one it leads to) ends the query as NOT_IMPLEMENTED and
  // the driver's general phase answers it (keto_amd/sharded.py)
  for (uint64_t it = 0; shard_n == 1 && it <= n1; it++) {  // every round that changes something marks a node
    uint32_t h = 0;
    HIPC(hipMemsetAsync(d_cnt + 2, 0, 4, stream));
    hipLaunchKernelGGL(k_aug_propagate, dim3(g1), dim3(256), 0, stream, x, b, A, n1, cand_of, c_plan, c_obj, imp,
                       d_cnt + 2);
    HIPC(hipMemcpyAsync(&h, d_cnt + 2, 4, hipMemcpyDeviceToHost, stream));
    HIPC(hipStreamSynchronize(stream));
    if (!h) break;
  }
  // 4. augmented set-adjacency and check rows
  uint64_t *adeg, *cdeg;
  if (talloc((void**)&adeg, ((size_t)n1 + 1) * 8) || talloc((void**)&cdeg, ((size_t)n1 + 1) * 8)) return -1;
  hipLaunchKernelGGL(k_aug_len, dim3(g1), dim3(256), 0, stream, x, b, A, n1, cand_of, c_plan, c_obj, imp, adeg, cdeg);
  HIPC(hipGetLastError());
  HIPC(hipMemsetAsync(adeg + n1, 0, 8, stream));
  HIPC(hipMemsetAsync(cdeg + n1, 0, 8, stream));
  uint64_t *aoff, *coff, *roff;
  uint8_t* flags;
  if (alloc((void**)&aoff, ((size_t)n1 + 1) * 8) || alloc((void**)&coff, ((size_t)n1 + 1) * 8) ||
      alloc((void**)&roff, ((size_t)n1 + 1) * 8) || alloc((void**)&flags, (size_t)n1 + 16))
    return -1;
  size_t tb = 0;
  HIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, adeg, aoff, (size_t)n1 + 1, stream));
  void* scratch;
  if (talloc(&scratch, tb + 16)) return -1;
  HIPC(hipcub::DeviceScan::ExclusiveSum(scratch, tb, adeg, aoff, (size_t)n1 + 1, stream));
  HIPC(hipcub::DeviceScan::ExclusiveSum(scratch, tb, cdeg, coff, (size_t)n1 + 1, stream));
  uint64_t tot[2];
  HIPC(hipMemcpyAsync(&tot[0], aoff + n1, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipMemcpyAsync(&tot[1], coff + n1, 8, hipMemcpyDeviceToHost, stream));
  HIPC(hipStreamSynchronize(stream));
  uint32_t *adj, *crow;
  if (alloc((void**)&adj, tot[0] * 4 + 4) || alloc((void**)&crow, tot[1] * 4 + 4)) return -1;
  hipLaunchKernelGGL(k_aug_fill, dim3(g1), dim3(256), 0, stream, x, b, A, n1, cand_of, c_plan, c_obj, imp, aoff, coff,
                     adj, crow, roff, flags);
  HIPC(hipGetLastError());
  // extended node triples become the snapshot's
  uint32_t *ns2, *obj2, *rel2;
  if (alloc((void**)&ns2, (size_t)n1 * 4) || alloc((void**)&obj2, (size_t)n1 * 4) || alloc((void**)&rel2, (size_t)n1 * 4))
    return -1;
  HIPC(hipMemcpyAsync(ns2, nd_ns, (size_t)n1 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipMemcpyAsync(obj2, nd_obj, (size_t)n1 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipMemcpyAsync(rel2, nd_rel, (size_t)n1 * 4, hipMemcpyDeviceToDevice, stream));
  HIPC(hipStreamSynchronize(stream));
  // the base check structures are superseded (row_subj stays: the extended raw rows index it)
  for (const void* p : {(const void*)ds.adj_off, (const void*)ds.adj, (const void*)ds.row_off, (const void*)ds.nd_ns,
                        (const void*)ds.nd_obj, (const void*)ds.nd_rel, (const void*)ds.nflags})
    free_alloc((void*)p);
  ds.n_nodes = n1;
  ds.nd_ns = ns2;
  ds.nd_obj = obj2;
  ds.nd_rel = rel2;
  ds.adj_off = aoff;
  ds.adj = adj;
  ds.row_off = roff;
  ds.crow_off = coff;
  ds.crow_subj = crow;
  ds.nflags = flags;
  n_set_edges = tot[0];
  n_check_rows = tot[1];
  // a tuple-built snapshot keeps its host node map complete (kg_snapshot_apply interns against it)
  if (n_new && h_nd_ns.size() == n0 && !hmap.k.empty()) {
    std::vector<uint32_t> a(n_new), b(n_new), c(n_new);
    HIPC(hipMemcpy(a.data(), ns2 + n0, (size_t)n_new * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(b.data(), obj2 + n0, (size_t)n_new * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(c.data(), rel2 + n0, (size_t)n_new * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n_new; i++) {
      h_nd_ns.push_back(a[i]);
      h_nd_obj.push_back(b[i]);
      h_nd_rel.push_back(c[i]);
      hmap.put(nmap_key(a[i], c[i], b[i]), n0 + i);
    }
  }
  n_virtual = nc;
  n_virtual_new = n_new;
  return 0;
}

}  // namespace kg
