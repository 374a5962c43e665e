// kg_tree.cpp -- CheckRelationTuple's Result.Tree inside the library (kg_check_tree).
//
// The reference builds the tree while it checks (internal/check/checkgroup/definitions.go:46-50,
// 101-124 WithEdge; binop.go:38-69): a check answered by checkDirect is a leaf of the request tuple
// (engine.go:165-172); one answered through a subject-set row is the tree of that row's check
// (engine.go:118-136: no node of its own); a rewrite child is wrapped in an edge node labelled with
// the request tuple and typed by the child (rewrites.go:59-92,112-139; an edge over a child without a
// tree is a leaf of the request tuple); `or` returns its first member child's tree in child order,
// `and` an intersection node without tuple over every child's tree, `not` keeps the inner tree and
// flips the membership (rewrites.go:141-160).  checkIsAllowed runs its three branches concurrently, so
// which member branch supplies the tree is schedule-dependent upstream; this walk takes direct, then
// subject-set rows in row order, then the rewrite (asserted paths: rewrites_test.go:186-205).
//
// Every membership the walk relies on is the GPU engine's: sub-checks go through kg_check_batch (one
// batched call per row of candidates, memoised) and rows through the snapshot's row reads
// (kg_snapshot_rows).  Only checks at rest depth 0 -- which read no tuple whose answer can count
// (checkDirect at depth -1 and every subject-set child at -1 are Unknown) -- are decided from the
// rewrite program alone, as checkIsAllowed(r, 0) does.  Not a hot path.  keto_amd/explain.py is the
// same walk in Python (the CPU-tested restatement).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/ketogpu.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {
namespace {

enum : int { RW_OR = 0, RW_AND = 1, RW_COMPUTED = 2, RW_TTU = 3, RW_NOT = 4 };
enum Mem : char { MM = 'M', MN = 'N', ME = 'E', MU = 'U' };

using Q6 = std::array<uint32_t, 6>;  // (ns, obj, rel, sns, sobj, srel)

struct Ans {
  Mem m;
  uint32_t e;
};

struct Node {
  uint8_t type;
  bool has_tuple;
  Q6 t;
  std::vector<int> kids;
};

struct Explain {
  Snapshot* s;
  kg_snapshot* sp;
  int32_t gdepth;
  const ProgCopy& P;
  bool prog;
  uint32_t wild;
  std::map<std::pair<uint32_t, uint32_t>, int32_t> roots;
  std::set<uint32_t> hidden;
  std::map<std::array<uint32_t, 3>, std::vector<kg_tuple>> rows_;
  std::map<std::pair<Q6, int32_t>, Ans> mem;
  std::vector<Node> pool;
  int fail = 0;  // first error code of a library call (the walk then unwinds)

  Explain(Snapshot* s_, kg_snapshot* sp_, int32_t g, const uint32_t* hid, size_t nh)
      : s(s_), sp(sp_), gdepth(g), P(s_->prog_copy) {
    prog = P.have && !P.ns_has_rel.empty();
    wild = s->wildcard_rel;
    for (size_t j = 0; j < P.rel_ns.size(); j++) roots[{P.rel_ns[j], P.rel_rel[j]}] = P.rel_root[j];
    for (size_t k = 0; k < nh; k++) hidden.insert(hid[k]);
  }

  const std::vector<kg_tuple>& rows(uint32_t ns, uint32_t obj, uint32_t rel) {
    const std::array<uint32_t, 3> k{ns, obj, rel};
    auto it = rows_.find(k);
    if (it != rows_.end()) return it->second;
    std::vector<kg_tuple>& r = rows_[k];
    kg_set key{ns, obj, rel, 0};
    uint64_t off[2] = {0, 0};
    const int64_t total = s->rows_of(&key, 1, off, nullptr, 0);
    if (total < 0) {
      fail = fail ? fail : (int)total;
      return r;
    }
    r.resize((size_t)total);
    if (total && s->rows_of(&key, 1, off, r.data(), (uint64_t)total) < 0) {
      fail = fail ? fail : -1;
      r.clear();
    }
    return r;
  }

  // astRelationFor (engine.go:209-229): 0 none, 1 rewrite (root), 2 error (code)
  int relation(uint32_t ns, uint32_t rel, int32_t* out) const {
    if (!prog || ns >= P.ns_has_rel.size() || !P.ns_has_rel[ns]) return 0;
    auto it = roots.find({ns, rel});
    if (it == roots.end()) {
      *out = KG_ERR_RELATION_NOT_FOUND;
      return 2;
    }
    if (it->second >= 0) {
      *out = it->second;
      return 1;
    }
    return 0;
  }

  // checkIsAllowed(q, d) for each q (d >= 1 through kg_check_batch)
  std::vector<Ans> member(const std::vector<Q6>& qs, int32_t d) {
    std::vector<Q6> todo;
    std::set<Q6> seen;
    for (const Q6& q : qs)
      if (!mem.count({q, d}) && seen.insert(q).second) todo.push_back(q);
    if (!todo.empty()) {
      if (d >= 1) {
        std::vector<kg_query> kq(todo.size());
        for (size_t i = 0; i < todo.size(); i++)
          kq[i] = kg_query{kg_tuple{todo[i][0], todo[i][1], todo[i][2], todo[i][3], todo[i][4], todo[i][5]}, d};
        std::vector<uint8_t> out(todo.size());
        std::vector<uint32_t> err(todo.size());
        const int rc = kg_check_batch(sp, kq.data(), kq.size(), gdepth, out.data(), err.data(), nullptr);
        if (rc) fail = fail ? fail : rc;
        for (size_t i = 0; i < todo.size(); i++)
          mem[{todo[i], d}] = rc ? Ans{MN, 0}
                                 : Ans{out[i] == KG_IS_MEMBER ? MM : (out[i] == KG_ERROR ? ME : MN), err[i]};
      } else {
        for (const Q6& q : todo) mem[{q, d}] = d == 0 ? depth0(q, {}) : Ans{MN, 0};
      }
    }
    std::vector<Ans> r;
    r.reserve(qs.size());
    for (const Q6& q : qs) r.push_back(mem[{q, d}]);
    return r;
  }

  // ---- rest depth 0: only the rewrite program can answer
  Ans depth0(const Q6& q, std::vector<Q6> stack) {
    int32_t root = 0;
    const int k = relation(q[0], q[2], &root);
    if (k == 2) return {ME, (uint32_t)root};
    if (k == 0) return {MN, 0};
    if (std::find(stack.begin(), stack.end(), q) != stack.end()) return {ME, KG_ERR_REWRITE_CYCLE};
    stack.push_back(q);
    return r0(root, q, stack);
  }
  Ans r0(int32_t idx, const Q6& q, const std::vector<Q6>& stack) {
    const kg_rw_node& n = P.rw[(size_t)idx];
    if (n.kind == RW_OR || n.kind == RW_AND) {
      if (n.count == 0) return {MN, 0};
      for (int32_t j = 0; j < n.count; j++) {
        const Ans a = c0(P.child[(size_t)(n.first + j)], q, stack);
        if (a.m == ME) return a;
        if (n.kind == RW_OR && a.m == MM) return {MM, 0};
        if (n.kind == RW_AND && a.m != MM) return {MN, 0};
      }
      return n.kind == RW_AND ? Ans{MM, 0} : Ans{MN, 0};
    }
    return c0(idx, q, stack);
  }
  Ans c0(int32_t idx, const Q6& q, const std::vector<Q6>& stack) {
    const kg_rw_node& n = P.rw[(size_t)idx];
    if (n.kind == RW_COMPUTED) return depth0(Q6{q[0], q[1], (uint32_t)n.rel, q[3], q[4], q[5]}, stack);
    if (n.kind == RW_TTU) return {MN, 0};  // every candidate is checkIsAllowed(.., -1): Unknown
    if (n.kind == RW_NOT) {
      const Ans a = c0(P.child[(size_t)n.first], q, stack);
      return a.m == MM ? Ans{MN, 0} : (a.m == MN ? Ans{MM, 0} : a);
    }
    return r0(idx, q, stack);
  }

  void inconsistent() {
    if (!fail) fail = set_error(-1, "kg_check_tree: the engine answered IsMember but no branch reproduces it");
  }

  // ---- trees
  int leaf(const Q6& q) {
    pool.push_back(Node{KG_CTREE_LEAF, true, q, {}});
    return (int)pool.size() - 1;
  }
  int edge_node(uint8_t type, const Q6& q, int kid) {
    pool.push_back(Node{type, true, q, {kid}});
    return (int)pool.size() - 1;
  }

  bool direct(const Q6& q) {
    for (const kg_tuple& t : rows(q[0], q[1], q[2]))
      if (t.sns == q[3] && t.sobj == q[4] && (t.srel == q[5] || q[3] == KG_SUBJECT_ID)) return true;
    return false;
  }
  std::vector<Q6> set_children(const Q6& q) {  // checkExpandSubject's candidates, first occurrence
    std::vector<Q6> out;
    std::set<Q6> seen;
    for (const kg_tuple& t : rows(q[0], q[1], q[2]))
      if (t.sns != KG_SUBJECT_ID && t.srel != wild) {
        const Q6 c{t.sns, t.sobj, t.srel, q[3], q[4], q[5]};
        if (seen.insert(c).second) out.push_back(c);
      }
    return out;
  }

  // the tree of checkIsAllowed(q, d), which the engine answered IsMember; -1: none (inconsistent)
  int tree(const Q6& q, int32_t d) {
    if (fail) return -1;
    if (d >= 1) {
      if (direct(q)) return leaf(q);
      const std::vector<Q6> kids = set_children(q);
      if (!kids.empty()) {
        const std::vector<Ans> a = member(kids, d - 1);
        for (size_t i = 0; i < kids.size(); i++)
          if (a[i].m == MM) return tree(kids[i], d - 1);
      }
    }
    int32_t root = 0;
    if (relation(q[0], q[2], &root) == 1) {  // at depth 0 the only branch (and it holds only through `not`)
      int t = -1;
      const Ans a = rewrite(root, q, d, &t);
      if (a.m == MM) return t;
    }
    return -1;
  }

  Ans rewrite(int32_t idx, const Q6& q, int32_t d, int* t) {  // checkSubjectSetRewrite + or / and
    *t = -1;
    if (d < 0) return {MU, 0};
    const kg_rw_node& n = P.rw[(size_t)idx];
    if (n.count == 0) return {MN, 0};
    if (n.kind == RW_OR) {
      for (int32_t j = 0; j < n.count; j++) {
        int ct = -1;
        const Ans a = edge(P.child[(size_t)(n.first + j)], q, d, &ct);
        if (a.m == ME) return a;
        if (a.m == MM) {
          *t = ct;
          return {MM, 0};
        }
      }
      return {MN, 0};
    }
    if (n.kind == RW_AND) {
      std::vector<int> trees;
      for (int32_t j = 0; j < n.count; j++) {
        int ct = -1;
        const Ans a = edge(P.child[(size_t)(n.first + j)], q, d, &ct);
        if (a.m != MM) return {a.m == ME ? ME : MN, a.e};
        trees.push_back(ct);
      }
      pool.push_back(Node{KG_CTREE_INTERSECTION, false, Q6{}, trees});
      *t = (int)pool.size() - 1;
      return {MM, 0};
    }
    return {ME, KG_ERR_NOT_IMPLEMENTED};
  }

  Ans edge(int32_t idx, const Q6& q, int32_t d, int* t) {  // one rewrite child behind WithEdge
    *t = -1;
    const kg_rw_node& n = P.rw[(size_t)idx];
    if (n.kind == RW_COMPUTED && hidden.count((uint32_t)n.rel)) {
      // a lowered tuple-to-subject-set leaf: the hidden relation holds no tuples, so its only member
      // branch is its TTU -- the reference's tree has that TTU edge right here
      int32_t root = 0;
      if (relation(q[0], (uint32_t)n.rel, &root) == 1) {
        const kg_rw_node& h = P.rw[(size_t)root];
        return edge(P.child[(size_t)h.first], q, d, t);
      }
    }
    uint8_t etype;
    Ans a{MN, 0};
    int ct = -1;
    if (n.kind == RW_COMPUTED) {
      etype = KG_CTREE_COMPUTED;
      a = computed((uint32_t)n.rel, q, d, &ct);
    } else if (n.kind == RW_TTU) {
      etype = KG_CTREE_TTU;
      a = ttu((uint32_t)n.rel, (uint32_t)n.crel, q, d, &ct);
    } else if (n.kind == RW_NOT) {
      etype = KG_CTREE_NOT;
      if (d < 0) {
        a = {MU, 0};
      } else {
        a = edge(P.child[(size_t)n.first], q, d, &ct);
        a.m = a.m == MM ? MN : (a.m == MN ? MM : a.m);
      }
    } else {
      etype = n.kind == RW_OR ? KG_CTREE_UNION : KG_CTREE_INTERSECTION;
      a = rewrite(idx, q, d, &ct);
    }
    *t = ct < 0 ? leaf(q) : edge_node(etype, q, ct);
    return a;
  }

  Ans computed(uint32_t rel, const Q6& q, int32_t d, int* t) {
    *t = -1;
    if (d < 0) return {MU, 0};
    const Q6 c{q[0], q[1], rel, q[3], q[4], q[5]};
    const Ans a = member({c}, d)[0];
    if (a.m == MM && (*t = tree(c, d)) < 0) inconsistent();
    return a;
  }

  Ans ttu(uint32_t rel, uint32_t crel, const Q6& q, int32_t d, int* t) {
    *t = -1;
    if (d < 0) return {MU, 0};
    std::vector<Q6> cands;
    std::set<Q6> seen;
    for (const kg_tuple& r : rows(q[0], q[1], rel))
      if (r.sns != KG_SUBJECT_ID) {
        const Q6 c{r.sns, r.sobj, crel, q[3], q[4], q[5]};
        if (seen.insert(c).second) cands.push_back(c);
      }
    if (cands.empty() || d - 1 < 0) return {MN, 0};
    const std::vector<Ans> res = member(cands, d - 1);
    for (size_t i = 0; i < cands.size(); i++)
      if (res[i].m == MM) {
        if ((*t = tree(cands[i], d - 1)) < 0) inconsistent();
        return {MM, 0};
      }
    for (const Ans& a : res)
      if (a.m == ME) return a;
    return {MN, 0};
  }

  // pre-order records of the tree rooted at pool[i]
  void emit(int i, std::vector<kg_check_node>* out) const {
    const Node& n = pool[(size_t)i];
    kg_check_node r{};
    r.type = n.type;
    r.has_tuple = n.has_tuple ? 1 : 0;
    r.n_children = (uint32_t)n.kids.size();
    r.t = kg_tuple{n.t[0], n.t[1], n.t[2], n.t[3], n.t[4], n.t[5]};
    out->push_back(r);
    for (int k : n.kids) emit(k, out);
  }
};

}  // namespace
}  // namespace kg

using kg::set_error;

extern "C" int kg_check_tree(kg_snapshot* sp, const kg_query* q, int32_t global_max_depth, const uint32_t* hidden_rels,
                             size_t n_hidden, kg_check_node* out, size_t cap, size_t* n_nodes, uint8_t* result,
                             uint32_t* err_code) {
  try {
    if (!sp || !q || !n_nodes || !result) return set_error(-2, "NULL argument");
    if (n_hidden && !hidden_rels) return set_error(-2, "hidden_rels is NULL");
    kg::Snapshot* s = reinterpret_cast<kg::Snapshot*>(sp);
    if (s->shard_n > 1) return set_error(-2, "kg_check_tree: not on a hash-sharded snapshot");
    *n_nodes = 0;
    if (err_code) *err_code = 0;
    if (global_max_depth < 1) global_max_depth = 5;  // config.schema.json:308-315 default
    uint8_t r = 0;
    uint32_t e = 0;
    if (int rc = kg_check_batch(sp, q, 1, global_max_depth, &r, &e, nullptr)) return rc;
    *result = r;
    if (err_code) *err_code = e;
    if (r != KG_IS_MEMBER) return 0;  // only a member has a tree (engine.go:65-80)
    int32_t d = q->max_depth;
    if (d <= 0 || global_max_depth < d) d = global_max_depth;  // engine.go:68-70
    kg::Explain x(s, sp, global_max_depth, hidden_rels, n_hidden);
    const kg::Q6 root{q->t.ns, q->t.obj, q->t.rel, q->t.sns, q->t.sobj, q->t.srel};
    const int t = x.tree(root, d);
    if (x.fail) return x.fail;
    if (t < 0) return set_error(-1, "kg_check_tree: the engine answered IsMember but no branch reproduces it");
    std::vector<kg_check_node> recs;
    x.emit(t, &recs);
    *n_nodes = recs.size();
    if (!out || cap < recs.size())
      return set_error(-3, "tree needs %zu records (capacity %zu)", recs.size(), out ? cap : (size_t)0);
    memcpy(out, recs.data(), recs.size() * sizeof(kg_check_node));
    kg::clear_error();
    return 0;
  } catch (const std::exception& ex) {
    return set_error(-5, "internal error: %s", ex.what());
  }
}
