// kg_interp.hip -- rewrite interpreter: queries whose reachable region holds subject-set rewrites
// or undeclared relations (routed GENERAL by k_resolve).
//
// One wave64 per query runs the reference recursion as an explicit stack machine (frames in HBM,
// per wave slot), evaluating children strictly in the reference's order so that "first Err or
// IsMember wins" is exact:
//   CIA  checkIsAllowed (engine.go:183-207): direct(d-1) -> expand children (d-1) in shard order ->
//        "relation not found" error (engine.go:228) | rewrite (rewrites.go:30-93)
//   RW   or / and over the rewrite children (binop.go:15-70)
//   TTU  checkTupleToSubjectSet (rewrites.go:205-260): every subject-set row (any relation,
//        "..." included) -> checkIsAllowed(set.ns, set.obj, computed, d-1)
//   NOT  checkInverted (rewrites.go:95-159): IsMember <-> NotMember, errors pass through
//   computed subject sets recurse at the same depth (rewrites.go:167-193).
// Runs of consecutive rewrite-free ("pure") children are answered together by one multi-root
// wave BFS (kg_bfs.h) -- a pure child can only answer IsMember/NotMember, so batching it keeps the
// first-decisive-result order.  (node, depth) results are memoised per query (the schedule-free
// semantics), which also detects computed-subject-set cycles.
//
// Pass 1 keeps BFS state in LDS; a query whose BFS outgrows LDS restarts in pass 2, which keeps
// it in a per-slot HBM bitmap + list sized for the whole graph.
#include <hip/hip_runtime.h>

#include "kg_bfs.h"
#include "kg_internal.h"
#include "kg_interp.h"
#include "kg_snapshot.h"

namespace kg {

enum : uint32_t { F_CIA = 0, F_RW = 1, F_TTU = 2, F_NOT = 3 };
enum : uint32_t { R_N = 0, R_M = 1, R_ERR = 2, R_NONE = 0xFF, R_INPROG = 0xFE, R_MISS = 0xFD };
constexpr uint32_t STAGE_MEMOIZED = 99;

struct Frame {
  uint32_t kind, ns, obj, rel, node;
  int32_t d;
  uint32_t a, b;
};

__device__ __forceinline__ bool decisive(uint32_t r) { return r == R_M || r == R_ERR; }

__device__ __forceinline__ int32_t relroot(const DevSnap& s, uint32_t ns, uint32_t rel) {
  return s.relroot[(size_t)ns * s.n_rel + rel];
}
// impure = a rewrite / undeclared relation is reachable from this (possibly row-less) node
__device__ __forceinline__ bool target_impure(const DevSnap& s, uint32_t ns, uint32_t rel, uint32_t node) {
  if (node != NONE) return s.nflags && (s.nflags[node] & NF_IMPURE);
  return relflag(s, ns, rel) != 0;
}

// ---------------------------------------------------------------- per-query memo (lane 0 only)
__device__ __forceinline__ uint32_t memo_get(const MemoEnt* m, uint64_t key, int32_t d, uint64_t tag) {
  uint64_t h = mix64(key ^ ((uint64_t)(uint32_t)d * 0x9E3779B97F4A7C15ull));
  for (int p = 0; p < 16; p++) {
    const MemoEnt& e = m[(h + p) & (MEMO_CAP - 1)];
    if (e.tag != tag) return R_MISS;
    if (e.key == key && e.d == d) return e.val;
  }
  return R_MISS;
}
__device__ __forceinline__ void memo_put(MemoEnt* m, uint64_t key, int32_t d, uint64_t tag, uint32_t val) {
  uint64_t h = mix64(key ^ ((uint64_t)(uint32_t)d * 0x9E3779B97F4A7C15ull));
  for (int p = 0; p < 16; p++) {
    MemoEnt& e = m[(h + p) & (MEMO_CAP - 1)];
    if (e.tag != tag || (e.key == key && e.d == d)) {
      e.key = key;
      e.d = d;
      e.val = val;
      e.tag = tag;
      return;
    }
  }  // table region full: not memoised (only costs time)
}

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

enum : int { Q_OVERFLOW = -1 };

// Evaluates one query; returns R_N / R_M / R_ERR (code in err) or Q_OVERFLOW (store tier too small).
template <class Store>
__device__ int interp_query(const DevSnap& s, Store& st, const kg_query& oq, const RQuery& q, Frame* stack,
                            MemoEnt* memo, uint64_t tag, uint32_t& err, BfsStats& bs) {
  const int lane = lane_id();
  int sp = 0;
  Frame F{F_CIA, oq.t.ns, oq.t.obj, oq.t.rel, q.node, q.depth, 0, 0};
  uint32_t ret = R_NONE;
  err = KG_ERR_NONE;
  const uint32_t subj = q.subj;

  auto push = [&](const Frame& nf) -> bool {
    if (sp >= STACK_CAP) return false;
    if (lane == 0) stack[sp] = F;
    sp++;
    F = nf;
    return true;
  };
  // multi-root BFS over pure roots at rest depth d0
  auto bfs = [&](uint32_t n_roots, int d0) -> int { return wave_bfs_run(s, st, n_roots, d0, subj, bs); };

  // every step pushes a frame (bounded by STACK_CAP), advances a cursor or returns a result;
  // the step cap is a termination guarantee against engine bugs, never reached on valid input
  for (uint64_t steps = 0;; steps++) {
    if (steps > (1ull << 34)) {
      err = KG_ERR_RESOURCE;
      return R_ERR;
    }
    bool done = false;
    uint32_t res = R_N;
    switch (F.kind) {
      case F_CIA: {
        const uint64_t key = nmap_key(F.ns, F.rel, F.obj);
        if (F.a == 0) {
          uint32_t mv = 0;
          if (lane == 0) mv = memo_get(memo, key, F.d, tag);
          mv = __shfl(mv, 0, 64);
          if (mv == R_INPROG) {  // computed-subject-set cycle at equal depth
            err = KG_ERR_REWRITE_CYCLE;
            res = R_ERR;
            done = true;
            break;
          }
          if (mv != R_MISS) {
            res = mv;
            F.a = STAGE_MEMOIZED;
            done = true;
            break;
          }
          if (lane == 0) memo_put(memo, key, F.d, tag, R_INPROG);
          if (F.node != NONE && F.d - 1 >= 0) {  // checkDirect(d-1)
            bs.probes++;
            bool hit = false;
            if (lane == 0) hit = dset_probe(s, F.node, subj);
            if (__shfl((int)hit, 0, 64)) {
              res = R_M;
              done = true;
              break;
            }
          }
          F.a = 1;
          F.b = 0;
        }
        if (F.a == 1) {  // checkExpandSubject: children at d-1 in shard order
          if (ret != R_NONE) {
            const uint32_t r = ret;
            ret = R_NONE;
            if (decisive(r)) {
              res = r;
              done = true;
              break;
            }
          }
          bool pushed = false;
          if (F.node != NONE && F.d - 1 >= 0) {
            const uint64_t rb = s.adj_off[F.node], re = s.adj_off[F.node + 1];
            if (F.b == 0) bs.rows++;
            uint32_t n_roots = 0;
            st.reset();
            for (uint64_t base = rb + F.b; base < re; base += 64) {
              const uint64_t i = base + lane;
              const bool valid = i < re;
              const uint32_t c = valid ? s.adj[i] : 0;
              const bool imp = valid && s.nflags && (s.nflags[c] & NF_IMPURE);
              const uint64_t mi = __ballot(imp);
              const uint32_t first = mi ? (uint32_t)(__ffsll((unsigned long long)mi) - 1) : 64u;
              bs.edges += __popcll(__ballot(valid && (uint32_t)lane <= first));
              if (n_roots + 64 > st.cap() || n_roots >= 256) {  // flush the batch
                const int r = bfs(n_roots, F.d - 1);
                if (r == BFS_OVERFLOW) return Q_OVERFLOW;
                if (r == BFS_M) {
                  res = R_M;
                  done = true;
                  break;
                }
                n_roots = 0;
                st.reset();
              }
              if (!wave_add_roots(st, valid && (uint32_t)lane < first, c, n_roots)) return Q_OVERFLOW;
              if (mi) {
                if (n_roots) {
                  const int r = bfs(n_roots, F.d - 1);
                  if (r == BFS_OVERFLOW) return Q_OVERFLOW;
                  if (r == BFS_M) {
                    res = R_M;
                    done = true;
                    break;
                  }
                  n_roots = 0;
                }
                const uint32_t cnode = __shfl(c, (int)first, 64);
                F.b = (uint32_t)(base - rb) + first + 1;
                Frame nf{F_CIA, s.nd_ns[cnode], s.nd_obj[cnode], s.nd_rel[cnode], cnode, F.d - 1, 0, 0};
                if (!push(nf)) {
                  err = KG_ERR_RESOURCE;
                  return R_ERR;
                }
                pushed = true;
                break;
              }
            }
            if (done) break;
            if (!pushed && n_roots) {
              const int r = bfs(n_roots, F.d - 1);
              if (r == BFS_OVERFLOW) return Q_OVERFLOW;
              if (r == BFS_M) {
                res = R_M;
                done = true;
                break;
              }
            }
          }
          if (pushed) break;
          F.a = 2;
        }
        if (F.a == 2) {  // astRelationFor: error | rewrite | nothing
          const uint8_t rf = relflag(s, F.ns, F.rel);
          if (rf & 2) {
            err = KG_ERR_RELATION_NOT_FOUND;
            res = R_ERR;
            done = true;
            break;
          }
          if (rf & 1) {
            F.a = 3;
            const int32_t root = relroot(s, F.ns, F.rel);
            Frame nf{F_RW, F.ns, F.obj, F.rel, F.node, F.d, (uint32_t)root, 0};
            if (!push(nf)) {
              err = KG_ERR_RESOURCE;
              return R_ERR;
            }
            break;
          }
          res = R_N;
          done = true;
          break;
        }
        // F.a == 3: the rewrite answered
        {
          const uint32_t r = ret;
          ret = R_NONE;
          res = decisive(r) ? r : R_N;
          done = true;
        }
        break;
      }
      case F_RW:
      case F_NOT: {
        const bool is_not = F.kind == F_NOT;
        const RwNode w = s.rw[F.a];
        if (ret != R_NONE) {
          const uint32_t r = ret;
          ret = R_NONE;
          if (is_not) {
            res = r == R_M ? R_N : (r == R_N ? R_M : r);
            done = true;
            break;
          }
          if (w.kind == RW_OR) {
            if (decisive(r)) {
              res = r;
              done = true;
              break;
            }
          } else {
            if (r == R_ERR) {
              res = R_ERR;
              done = true;
              break;
            }
            if (r != R_M) {
              res = R_N;
              done = true;
              break;
            }
          }
          F.b++;
        }
        int32_t ci;
        if (is_not) {
          if (w.count != 1) {
            err = KG_ERR_NOT_IMPLEMENTED;
            res = R_ERR;
            done = true;
            break;
          }
          ci = s.rwchild[w.first];
        } else {
          if (w.kind != RW_OR && w.kind != RW_AND) {
            err = KG_ERR_NOT_IMPLEMENTED;
            res = R_ERR;
            done = true;
            break;
          }
          if ((int32_t)F.b >= w.count) {
            res = (w.count == 0 || w.kind == RW_OR) ? R_N : R_M;
            done = true;
            break;
          }
          ci = s.rwchild[w.first + (int32_t)F.b];
        }
        // evaluate rewrite child ci of the tuple (F.ns, F.obj) at depth F.d
        const RwNode c = s.rw[ci];
        Frame nf{};
        bool need_push = true;
        switch (c.kind) {
          case RW_OR:
          case RW_AND:
            nf = Frame{F_RW, F.ns, F.obj, F.rel, F.node, F.d, (uint32_t)ci, 0};
            break;
          case RW_NOT:
            nf = Frame{F_NOT, F.ns, F.obj, F.rel, F.node, F.d, (uint32_t)ci, 0};
            break;
          case RW_COMPUTED: {  // checkIsAllowed(ns, obj, c.rel) at the same depth
            const uint32_t tn = nmap_find(s, F.ns, (uint32_t)c.rel, F.obj);
            if (!target_impure(s, F.ns, (uint32_t)c.rel, tn)) {
              need_push = false;
              if (tn == NONE) {
                ret = R_N;
              } else {
                st.reset();
                uint32_t n = 0;
                wave_add_roots(st, lane == 0, tn, n);
                const int r = bfs(n, F.d);
                if (r == BFS_OVERFLOW) return Q_OVERFLOW;
                ret = r == BFS_M ? R_M : R_N;
              }
            } else {
              nf = Frame{F_CIA, F.ns, F.obj, (uint32_t)c.rel, tn, F.d, 0, 0};
            }
            break;
          }
          case RW_TTU: {
            const uint32_t tn = nmap_find(s, F.ns, (uint32_t)c.rel, F.obj);
            nf = Frame{F_TTU, F.ns, F.obj, (uint32_t)c.crel, tn, F.d, 0, 0};
            break;
          }
          default:
            need_push = false;
            err = KG_ERR_NOT_IMPLEMENTED;
            ret = R_ERR;
            break;
        }
        if (need_push && !push(nf)) {
          err = KG_ERR_RESOURCE;
          return R_ERR;
        }
        break;  // the child's answer comes back through `ret`
      }
      case F_TTU: {  // F.rel = computed relation, F.node = node of (ns, obj, ttu.rel), F.b = row cursor
        if (ret != R_NONE) {
          const uint32_t r = ret;
          ret = R_NONE;
          if (decisive(r)) {
            res = r;
            done = true;
            break;
          }
        }
        if (F.node == NONE || F.d - 1 < 0) {
          res = R_N;
          done = true;
          break;
        }
        const uint64_t rb = s.row_off[F.node], re = s.row_off[F.node + 1];
        if (F.b == 0) bs.rows++;
        uint32_t n_roots = 0;
        bool pushed = false;
        st.reset();
        for (uint64_t base = rb + F.b; base < re; base += 64) {
          const uint64_t i = base + lane;
          const bool valid = i < re;
          const uint32_t sub = valid ? s.row_subj[i] : 0;
          const bool is_set = valid && (sub & SET_BIT);
          uint32_t tn = NONE, tns = 0, tobj = 0;
          bool imp = false;
          if (is_set) {
            const uint32_t sn = sub & ~SET_BIT;
            tns = s.nd_ns[sn];
            tobj = s.nd_obj[sn];
            tn = nmap_find(s, tns, F.rel, tobj);
            imp = target_impure(s, tns, F.rel, tn);
          }
          const uint64_t mi = __ballot(imp);
          const uint32_t first = mi ? (uint32_t)(__ffsll((unsigned long long)mi) - 1) : 64u;
          bs.edges += __popcll(__ballot(valid && (uint32_t)lane <= first));
          if (n_roots + 64 > st.cap() || n_roots >= 256) {
            const int r = bfs(n_roots, F.d - 1);
            if (r == BFS_OVERFLOW) return Q_OVERFLOW;
            if (r == BFS_M) {
              res = R_M;
              done = true;
              break;
            }
            n_roots = 0;
            st.reset();
          }
          if (!wave_add_roots(st, is_set && !imp && tn != NONE && (uint32_t)lane < first, tn, n_roots))
            return Q_OVERFLOW;
          if (mi) {
            if (n_roots) {
              const int r = bfs(n_roots, F.d - 1);
              if (r == BFS_OVERFLOW) return Q_OVERFLOW;
              if (r == BFS_M) {
                res = R_M;
                done = true;
                break;
              }
              n_roots = 0;
            }
            Frame nf{F_CIA, __shfl(tns, (int)first, 64), __shfl(tobj, (int)first, 64), F.rel,
                     __shfl(tn, (int)first, 64), F.d - 1, 0, 0};
            F.b = (uint32_t)(base - rb) + first + 1;
            if (!push(nf)) {
              err = KG_ERR_RESOURCE;
              return R_ERR;
            }
            pushed = true;
            break;
          }
        }
        if (done || pushed) break;
        if (n_roots) {
          const int r = bfs(n_roots, F.d - 1);
          if (r == BFS_OVERFLOW) return Q_OVERFLOW;
          if (r == BFS_M) {
            res = R_M;
            done = true;
            break;
          }
        }
        res = R_N;
        done = true;
        break;
      }
    }
    if (!done) continue;
    if (F.kind == F_CIA && F.a != STAGE_MEMOIZED && lane == 0)
      memo_put(memo, nmap_key(F.ns, F.rel, F.obj), F.d, tag, res);
    if (sp == 0) return (int)res;
    wave_fence();
    sp--;
    F = stack[sp];
    ret = res;
  }
}

template <class Store>
__device__ void finish_query(uint32_t qi, int r, uint32_t e, uint8_t* out, uint32_t* err) {
  if (lane_id() != 0) return;
  out[qi] = r == R_M ? KG_IS_MEMBER : (r == R_ERR ? KG_ERROR : KG_NOT_MEMBER);
  if (err) err[qi] = r == R_ERR ? e : KG_ERR_NONE;
}

// Pass 1 (LDS BFS tier): persistent grid, per-XCD dequeue over the GENERAL list.  1024-slot hash +
// 512-node list per wave (6.3 KB; a 512 / 256 variant that fits 8 workgroups per CU measured the
// same on C3: the extra resident waves were offset by more queries reaching pass 2).
constexpr int ILDS_VL2 = VIS_LOG2, ILDS_LIST = LIST;
using ILdsStore = LdsStoreT<ILDS_VL2, ILDS_LIST>;
__global__ __launch_bounds__(256) void k_interp_lds(DevSnap s, const kg_query* __restrict__ oq,
                                                    const RQuery* __restrict__ rq, const uint32_t* gen_list,
                                                    InterpCtl* ic, uint8_t* out, uint32_t* err, Frame* stacks,
                                                    MemoEnt* memos, uint64_t batch_tag) {
  __shared__ WaveLdsT<ILDS_VL2, ILDS_LIST> lds_all[4];
  const int wave = threadIdx.x >> 6, lane = lane_id();
  ILdsStore st{&lds_all[wave]};
  const uint32_t slot = blockIdx.x * 4 + wave;
  Frame* stack = stacks + (size_t)slot * STACK_CAP;
  MemoEnt* memo = memos + (size_t)slot * MEMO_CAP;
  const uint32_t count = *ic->gen_count;
  if (count == 0) return;  // nothing routed here (e.g. every rewrite materialised or split)
  uint32_t head_sel = blockIdx.x & 7;
  const uint32_t head0 = head_sel;
  BfsStats bs;
  unsigned long long done = 0;
  for (;;) {
    uint32_t li = NONE;
    if (lane == 0) {
      while (head_sel < head0 + 8) {
        const uint32_t h = head_sel & 7;
        const uint32_t lo = (uint32_t)((uint64_t)count * h / 8), hi = (uint32_t)((uint64_t)count * (h + 1) / 8);
        const uint32_t k = atomicAdd(&ic->heads[h * 32], 1u);
        if (lo + k < hi) {
          li = lo + k;
          break;
        }
        head_sel++;
      }
    }
    li = __shfl(li, 0, 64);
    if (li == NONE) break;
    const uint32_t qi = gen_list[li];
    uint32_t e = 0;
    const int r = interp_query(s, st, oq[qi], rq[qi], stack, memo, batch_tag | qi, e, bs);
    if (r == Q_OVERFLOW) {
      if (lane == 0) ic->p2_list[atomicAdd(&ic->p2_count, 1u)] = qi;
    } else {
      finish_query<ILdsStore>(qi, r, e, out, err);
      done++;
    }
  }
  if (lane == 0) {
    atomicAdd(ic->st_general, done);
    atomicAdd(ic->st_rows, bs.rows);
    atomicAdd(ic->st_edges, bs.edges);
    atomicAdd(ic->st_probes, bs.probes);
  }
}

// Pass 2 / pass 3 (HBM BFS tiers): one wave per slot, a visited bitmap over the whole graph.
// Pass 2 runs many slots with a bounded BFS list (cap entries); a query whose list overflows
// leaves stray bits in its slot's bitmap, so the wave clears the whole bitmap and hands the
// query to pass 3, one slot whose list holds every node (cannot overflow).
__device__ __forceinline__ void clear_bitmap(uint32_t* bm, uint64_t words) {
  // words is a multiple of 4 and bm 16-B aligned (launch_general)
  uint4* b4 = reinterpret_cast<uint4*>(bm);
  for (uint64_t i = lane_id(); i < words / 4; i += 64) b4[i] = make_uint4(0, 0, 0, 0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One wave per slot: dequeue from qlist, evaluate, hand overflows on (pass 2) or report them.
template <class Store>
__device__ void interp_slot_loop(const DevSnap& s, const kg_query* __restrict__ oq, const RQuery* __restrict__ rq,
                                 InterpCtl* ic, int pass, uint32_t* p3_list, uint8_t* out, uint32_t* err, Store& st,
                                 uint32_t* clear_base, uint64_t clear_words, Frame* stack, MemoEnt* memo,
                                 uint64_t batch_tag) {
  const int lane = lane_id();
  const uint32_t* qlist = pass == 2 ? ic->p2_list : p3_list;
  const uint32_t count = pass == 2 ? ic->p2_count : ic->p3_count;
  uint32_t* head = pass == 2 ? &ic->p2_head : &ic->p3_head;
  BfsStats bs;
  unsigned long long done = 0;
  for (;;) {
    uint32_t li = 0;
    if (lane == 0) li = atomicAdd(head, 1u);
    li = __shfl(li, 0, 64);
    if (li >= count) break;
    const uint32_t qi = qlist[li];
    uint32_t e = 0;
    int r = interp_query(s, st, oq[qi], rq[qi], stack, memo, batch_tag | qi, e, bs);
    if (r == Q_OVERFLOW) {
      clear_bitmap(clear_base, clear_words);  // keys inserted but never listed stay behind otherwise
      if (pass == 2) {
        if (lane == 0) p3_list[atomicAdd(&ic->p3_count, 1u)] = qi;
        continue;
      }
      r = R_ERR;  // pass 3 holds every node: only the frame stack can run out
      e = KG_ERR_RESOURCE;
    }
    finish_query<Store>(qi, r, e, out, err);
    done++;
  }
  if (lane == 0) {
    atomicAdd(ic->st_general, done);
    atomicAdd(ic->st_rows, bs.rows);
    atomicAdd(ic->st_edges, bs.edges);
    atomicAdd(ic->st_probes, bs.probes);
  }
}

// Pass 2: many slots, visited hash of tsize (power of two >= 2 cap) slots + list of cap nodes.
__global__ __launch_bounds__(64) void k_interp_hash(DevSnap s, const kg_query* __restrict__ oq,
                                                    const RQuery* __restrict__ rq, InterpCtl* ic, uint32_t* p3_list,
                                                    uint8_t* out, uint32_t* err, Frame* stacks, MemoEnt* memos,
                                                    uint32_t* tabs, uint64_t tsize, uint32_t* lists, uint64_t cap,
                                                    uint64_t batch_tag) {
  __shared__ uint32_t pref[64];
  const uint32_t slot = blockIdx.x;
  uint32_t* tab = tabs + (size_t)slot * tsize;
  HashStore st{tab, (uint32_t)(tsize - 1), lists + (size_t)slot * cap, cap, pref};
  interp_slot_loop(s, oq, rq, ic, 2, p3_list, out, err, st, tab, tsize, stacks + (size_t)slot * STACK_CAP,
                   memos + (size_t)slot * MEMO_CAP, batch_tag);
}

// Pass 3: one slot, visited bitmap over the whole graph + a list that holds every node.
__global__ __launch_bounds__(64) void k_interp_hbm(DevSnap s, const kg_query* __restrict__ oq,
                                                   const RQuery* __restrict__ rq, InterpCtl* ic, uint32_t* p3_list,
                                                   uint8_t* out, uint32_t* err, Frame* stack, MemoEnt* memo,
                                                   uint32_t* bm, uint64_t words, uint32_t* list, uint64_t cap,
                                                   uint64_t batch_tag) {
  __shared__ uint32_t pref[64];
  GlobalStore st{bm, list, cap, pref};
  interp_slot_loop(s, oq, rq, ic, 3, p3_list, out, err, st, bm, words, stack, memo, batch_tag);
}

int launch_general(Snapshot* s, Workspace* w, const kg_query* d_q, const RQuery* rq, const uint32_t* gen_list,
                   const uint32_t* gen_count, InterpCtl* ic, uint8_t* out, uint32_t* err, uint32_t n_queries,
                   hipStream_t stream) {
  if (!s->has_program) return 0;  // without rewrites nothing is ever routed GENERAL
  const uint32_t grid1 = (uint32_t)s->n_cu * (uint32_t)s->interp_wgs;
  const uint32_t slots1 = grid1 * 4;
  const uint64_t nn = std::max<uint32_t>(s->ds.n_nodes, 1);
  const uint64_t words = ((nn + 31) / 32 + 1 + 3) & ~3ull;  // 16-B multiple: clear_bitmap stores uint4
  const size_t slot_bytes = STACK_CAP * sizeof(Frame) + MEMO_CAP * sizeof(MemoEnt);
  static_assert((STACK_CAP * sizeof(Frame) + MEMO_CAP * sizeof(MemoEnt)) % 16 == 0, "tables follow the slots 16-B aligned");
  // pass 2: 4 slots per CU (8 measured the same on C3: the pass is tail-bound), each a visited hash
  // + list of cap2 nodes (default 256 Ki: ~3 MB a slot)
  const uint64_t cap2 = (std::min<uint64_t>(nn, s->interp_cap2 ? s->interp_cap2 : 1ull << 18) + 3) & ~3ull;
  uint64_t tsize = 64;
  while (tsize < 2 * cap2 + 128) tsize <<= 1;
  const uint64_t per2 = slot_bytes + (tsize + cap2) * 4;
  // pass-2 budget: 4 GiB (~800 slots of 256 Ki nodes; what reaches pass 2 is the LDS pass's
  // overflow, a small fraction of a batch), or an eighth of the free HBM when less (other streams'
  // workspaces and the snapshot share the device); a pool that already exists keeps its layout
  uint64_t budget2 = 4ull << 30;
  if (w->interp_layout == 0) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) budget2 = std::min<uint64_t>(budget2, free_b / 8);
  } else {
    budget2 = (w->interp_layout >> 40) * per2;
  }
  uint32_t slots2 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)s->n_cu * 4, budget2 / per2));
  const size_t bytes1 = (size_t)slots1 * slot_bytes;
  const size_t bytes3 = slot_bytes + (words + nn) * 4;
  const size_t tail = (size_t)std::max<uint32_t>(n_queries, 1) * 4;
  size_t need = bytes1 + (size_t)slots2 * per2 + bytes3 + tail;
  if (need > w->interp_pool_bytes) {
    if (w->interp_pool) hipFree(w->interp_pool);
    w->interp_pool = nullptr;
    w->interp_pool_bytes = 0;
    // HBM is shared with the snapshot and the other streams' workspaces: fewer pass-2 slots on OOM
    hipError_t e;
    while ((e = hipMalloc(&w->interp_pool, need)) == hipErrorOutOfMemory && slots2 > 1) {
      (void)hipGetLastError();
      slots2 = slots2 / 2;
      need = bytes1 + (size_t)slots2 * per2 + bytes3 + tail;
    }
    HIPC(e);
    HIPC(hipMemsetAsync(w->interp_pool, 0, need, stream));  // memo tags 0 = empty; tables clear
    w->interp_pool_bytes = need;
  } else if (w->interp_layout != ((uint64_t)slots2 << 40 | (uint64_t)slots1 << 24 | cap2)) {
    HIPC(hipMemsetAsync(w->interp_pool, 0, need, stream));  // regions moved: tables must start clear
  }
  w->interp_layout = (uint64_t)slots2 << 40 | (uint64_t)slots1 << 24 | cap2;
  const size_t bytes2 = (size_t)slots2 * per2;
  char* p = (char*)w->interp_pool;
  Frame* stacks1 = (Frame*)p;
  MemoEnt* memos1 = (MemoEnt*)(p + (size_t)slots1 * STACK_CAP * sizeof(Frame));
  char* p2 = p + bytes1;
  Frame* stacks2 = (Frame*)p2;
  MemoEnt* memos2 = (MemoEnt*)(p2 + (size_t)slots2 * STACK_CAP * sizeof(Frame));
  uint32_t* tabs2 = (uint32_t*)(p2 + (size_t)slots2 * slot_bytes);
  uint32_t* lists2 = tabs2 + (size_t)slots2 * tsize;
  char* p3 = p2 + bytes2;
  Frame* stack3 = (Frame*)p3;
  MemoEnt* memo3 = (MemoEnt*)(p3 + STACK_CAP * sizeof(Frame));
  uint32_t* bm3 = (uint32_t*)(p3 + slot_bytes);
  uint32_t* list3 = bm3 + words;
  uint32_t* p3_list = (uint32_t*)(p3 + bytes3);
  const uint64_t tag = (uint64_t)(++s->batch_seq) << 32;
  hipLaunchKernelGGL(k_interp_lds, dim3(grid1), dim3(256), 0, stream, s->ds, d_q, rq, gen_list, ic, out, err, stacks1,
                     memos1, tag);
  HIPC(hipGetLastError());
  hipLaunchKernelGGL(k_interp_hash, dim3(slots2), dim3(64), 0, stream, s->ds, d_q, rq, ic, p3_list, out, err, stacks2,
                     memos2, tabs2, tsize, lists2, cap2, tag);
  HIPC(hipGetLastError());
  hipLaunchKernelGGL(k_interp_hbm, dim3(1), dim3(64), 0, stream, s->ds, d_q, rq, ic, p3_list, out, err, stack3, memo3,
                     bm3, words, list3, nn, tag);
  HIPC(hipGetLastError());
  (void)gen_count;
  return 0;
}

}  // namespace kg
