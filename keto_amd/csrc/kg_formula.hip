// kg_formula.hip -- boolean rewrites over union / plain relations, answered as leaf sub-checks.
//
// A relation whose rewrite is not a union (kg_augment.hip) but a boolean formula -- and / or / not
// (internal/check/rewrites.go:30-159, binop.go:15-70) over computed subject sets
// (rewrites.go:167-193) -- e.g. C3's `share = view & !blocked`, is, at rest depth d >= 1 (always
// true for a request: engine.go:68-70 clamps to the global max depth),
//
//   checkIsAllowed((ns,obj,R), d) = direct/expand of (ns,obj,R) itself  |  f(checkIsAllowed((ns,obj,c_j), d))
//
// with f the formula over its computed leaves c_j, evaluated at the SAME depth d (computed subject
// sets keep the depth; nested rewrites do too in the restatement the oracle pins: oracle/keto_oracle.c
// eval_rw / eval_child).  When every leaf relation is plain or a materialised union, and the leaf
// nodes of this object are pure (no rewrite / error reachable), each leaf check is M or N -- never
// Unknown or an error -- so the formula is plain boolean logic over ordinary rewrite-free checks.
// A query is split when, in addition, the node (ns,obj,R) itself holds no rows (its own direct /
// expand part is then NotMember): its leaf checks run as extra queries through the rewrite-free
// tiers (k_resolve -> k_stream2 -> k_back -> grid) in the same batch, and k_fcombine evaluates f.
// Everything else (TTU leaves, impure leaves, a rewrite root that is not and/or) stays with the
// interpreter (kg_interp.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "kg_bfs.h"
#include "kg_formula.h"
#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

// ------------------------------------------------------------------ device
// One thread per request, 1024 per workgroup, ONE slot reservation per workgroup: the leaf queries go
// to one contiguous range after the batch, so every reservation hits the same counter, and same-address
// atomics serialise at the memory side (~11 ns each, MI355X_MICROARCH.md).  Per wave (round 5) that was
// 15.6 k atomics per 1 M requests, 185 us of a C3 batch (profiles/r6a_c3_timeline.txt).
constexpr uint32_t FS_BLOCK = 1024;
__global__ __launch_bounds__(FS_BLOCK) void k_fsplit(DevSnap s, const int32_t* __restrict__ fidx,
                                                const FPlan* __restrict__ plans, const kg_query* __restrict__ q,
                                                uint32_t n, int32_t global, kg_query* __restrict__ q2,
                                                uint2* __restrict__ ref, uint32_t* n_extra) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < n;
  kg_query x{};
  uint32_t take = 0, pi = NONE;
  uint32_t ln[FP_LEAVES] = {NONE, NONE, NONE, NONE};
  if (valid) {
    x = q[i];
    const uint32_t ns = x.t.ns, rel = x.t.rel, obj = x.t.obj;
    if (ns < s.n_ns && rel < s.n_rel && nmap_key_ok(ns, rel, obj)) {
      const int32_t p = fidx[(size_t)ns * s.n_rel + rel];
      if (p >= 0) {
        const FPlan& P = plans[p];
        bool ok = true;
        if (P.own_rows) {
          const uint32_t own = nmap_find(s, ns, rel, obj);
          if (own != NONE) {  // its own rows would join the answer: not split
            const uint64_t* co = s.crow_off ? s.crow_off : s.row_off;
            ok = co[own + 1] == co[own] && s.adj_off[own + 1] == s.adj_off[own];
          }
        }
        for (uint32_t j = 0; j < P.n_leaves && ok; j++) {
          if (!((P.leaf_impure >> j) & 1)) continue;  // every node of this relation is pure
          ln[j] = nmap_find(s, ns, P.leaf[j], obj);
          if (ln[j] != NONE && s.nflags && (s.nflags[ln[j]] & NF_IMPURE)) ok = false;
        }
        if (ok) {
          take = P.n_leaves;
          pi = (uint32_t)p;
        }
      }
    }
  }
  // workgroup-aggregated slot reservation for the leaf queries
  __shared__ uint32_t s_wsum[FS_BLOCK / 64], s_base;
  const uint32_t wave = threadIdx.x >> 6;
  uint32_t total = 0;
  uint32_t off = wave_excl_scan(take, &total);
  if (lane_id() == 0) s_wsum[wave] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < FS_BLOCK / 64; k++) {
      const uint32_t c = s_wsum[k];
      s_wsum[k] = t;
      t += c;
    }
    s_base = t ? atomicAdd(n_extra, t) : 0u;
  }
  __syncthreads();
  off += s_wsum[wave];
  const uint32_t wbase = s_base;
  if (!valid) return;
  uint2 r = make_uint2(NONE, NONE);
  if (take) {
    int32_t d = x.max_depth;
    if (d <= 0 || global < d) d = global;  // engine.go:68-70: the leaves run at the clamped depth
    const FPlan& P = plans[pi];
    const uint32_t base = n + wbase + off;
    for (uint32_t j = 0; j < P.n_leaves; j++) {
      kg_query y = x;
      y.t.rel = P.leaf[j];
      y.max_depth = d;
      q2[base + j] = y;
    }
    x.t.ns = 0xFFFFFFFFu;  // the original is answered by k_fcombine: k_resolve finishes it at once
    r = make_uint2(base, pi);
  }
  q2[i] = x;
  ref[i] = r;
}

__global__ __launch_bounds__(256) void k_fcombine(const FPlan* __restrict__ plans, uint32_t n,
                                                  const uint2* __restrict__ ref, const uint8_t* __restrict__ out2,
                                                  const uint32_t* __restrict__ err2, uint8_t* __restrict__ out,
                                                  uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint2 r = ref[i];
  if (r.x == NONE) {
    out[i] = out2[i];
    if (err) err[i] = err2[i];
    return;
  }
  const FPlan& P = plans[r.y];
  uint32_t e = KG_ERR_NONE, bits = 0;
  for (uint32_t j = 0; j < P.n_leaves; j++) {
    if (e == KG_ERR_NONE) e = err2[r.x + j];  // pure leaves do not fail; a resource error would surface
    bits |= (out2[r.x + j] == KG_IS_MEMBER ? 1u : 0u) << j;
  }
  const uint32_t st = fplan_eval(P, bits) ? 1u : 0u;
  out[i] = (e == KG_ERR_NONE && (st & 1u)) ? KG_IS_MEMBER : KG_NOT_MEMBER;
  if (err) err[i] = e;
}

// Per (ns, rel): bit0 some node holds rows (check rows or set-adjacency), bit1 some node is impure.
__global__ void k_relstats(DevSnap s, uint32_t* rs) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= s.n_nodes) return;
  const uint32_t ns = s.nd_ns[v], rel = s.nd_rel[v];
  if (ns >= s.n_ns || rel >= s.n_rel) return;
  const uint64_t* co = s.crow_off ? s.crow_off : s.row_off;
  const uint32_t f = ((co[v + 1] != co[v] || s.adj_off[v + 1] != s.adj_off[v]) ? 1u : 0u) |
                     ((s.nflags && (s.nflags[v] & NF_IMPURE)) ? 2u : 0u);
  uint32_t* p = rs + (size_t)ns * s.n_rel + rel;
  if (f & ~*p) atomicOr(p, f);  // read first: most nodes find their bits already set
}

// ------------------------------------------------------------------ host
int Snapshot::build_formulas() {
  n_fplans = 0;
  fp_leaves = 0;
  d_fidx = nullptr;
  d_fplans = nullptr;
  if (!materialize || !has_program) return 0;
  const uint32_t n_ns = ds.n_ns, n_rel = ds.n_rel;
  auto flag = [&](uint32_t ns, uint32_t r) -> uint8_t { return host_relflag(ns, r); };
  auto virt = [&](uint32_t ns, uint32_t r) -> bool {
    return !h_virt.empty() && h_virt[(size_t)ns * n_rel + r] != 0;
  };
  std::vector<FPlan> plans;
  std::vector<int32_t> idx((size_t)n_ns * n_rel, -1);
  for (uint32_t ns = 0; ns < n_ns; ns++)
    for (uint32_t R = 0; R < n_rel; R++) {
      if (!(flag(ns, R) & 1) || virt(ns, R)) continue;
      const int32_t root = h_relroot[(size_t)ns * n_rel + R];
      if (root < 0 || (size_t)root >= h_rw.size()) continue;
      if (h_rw[(size_t)root].kind != RW_OR && h_rw[(size_t)root].kind != RW_AND) continue;  // else an error
      FPlan P{};
      bool ok = true;
      std::function<void(int32_t, int)> emit = [&](int32_t at, int depth) {
        if (!ok) return;
        if (at < 0 || (size_t)at >= h_rw.size() || depth > 32 || P.n_ops >= (uint32_t)FP_OPS) {
          ok = false;
          return;
        }
        const RwNode w = h_rw[(size_t)at];
        if (w.kind == RW_OR || w.kind == RW_AND) {
          if (w.count < 0 || w.count > 15 || w.first < 0 || (size_t)w.first + (size_t)w.count > h_rwchild.size()) {
            ok = false;
            return;
          }
          for (int32_t c = 0; c < w.count; c++) emit(h_rwchild[(size_t)(w.first + c)], depth + 1);
          if (!ok || P.n_ops >= (uint32_t)FP_OPS) {
            ok = false;
            return;
          }
          P.ops[P.n_ops++] = (uint8_t)((w.kind == RW_AND ? FOP_AND : FOP_OR) | w.count);
        } else if (w.kind == RW_NOT) {
          if (w.count != 1 || w.first < 0 || (size_t)w.first >= h_rwchild.size()) {  // KG_ERR_NOT_IMPLEMENTED
            ok = false;
            return;
          }
          emit(h_rwchild[(size_t)w.first], depth + 1);
          if (!ok || P.n_ops >= (uint32_t)FP_OPS) {
            ok = false;
            return;
          }
          P.ops[P.n_ops++] = FOP_NOT;
        } else if (w.kind == RW_COMPUTED) {
          const uint32_t c = (uint32_t)w.rel;
          // a leaf must be a rewrite-free check: declared, no rewrite or a materialised union, and
          // not R itself (a computed cycle is an error)
          if (w.rel < 0 || c >= n_rel || c == R || (flag(ns, c) & 2) || ((flag(ns, c) & 1) && !virt(ns, c))) {
            ok = false;
            return;
          }
          uint32_t j = 0;
          while (j < P.n_leaves && P.leaf[j] != c) j++;
          if (j == P.n_leaves) {
            if (P.n_leaves >= (uint32_t)FP_LEAVES) {
              ok = false;
              return;
            }
            P.leaf[P.n_leaves++] = c;
          }
          P.ops[P.n_ops++] = (uint8_t)(FOP_LEAF | j);
        } else {
          ok = false;  // tuple-to-subject-set leaves stay with the interpreter
        }
      };
      emit(root, 0);
      if (!ok || P.n_leaves == 0) continue;
      idx[(size_t)ns * n_rel + R] = (int32_t)plans.size();
      plans.push_back(P);
      fp_leaves = std::max(fp_leaves, P.n_leaves);
    }
  if (plans.empty()) return 0;
  // which plans need per-query lookups (own rows, impure leaf nodes)
  std::vector<uint32_t> rs(idx.size(), 0);
  if (ds.n_nodes) {
    uint32_t* d_rs = nullptr;
    HIPC(hipMalloc(&d_rs, rs.size() * 4 + 4));
    HIPC(hipMemsetAsync(d_rs, 0, rs.size() * 4, stream));
    hipLaunchKernelGGL(k_relstats, dim3((ds.n_nodes + 255) / 256), dim3(256), 0, stream, ds, d_rs);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(rs.data(), d_rs, rs.size() * 4, hipMemcpyDeviceToHost, stream));
    HIPC(hipStreamSynchronize(stream));
    HIPC(hipFree(d_rs));
  }
  for (uint32_t ns = 0; ns < n_ns; ns++)
    for (uint32_t R = 0; R < n_rel; R++) {
      const int32_t p = idx[(size_t)ns * n_rel + R];
      if (p < 0) continue;
      FPlan& P = plans[(size_t)p];
      P.own_rows = rs[(size_t)ns * n_rel + R] & 1u;
      for (uint32_t j = 0; j < P.n_leaves; j++)
        if (rs[(size_t)ns * n_rel + P.leaf[j]] & 2u) P.leaf_impure |= 1u << j;
    }
  if (alloc((void**)&d_fidx, idx.size() * 4) || alloc(&d_fplans, plans.size() * sizeof(FPlan))) return -1;
  HIPC(hipMemcpy(d_fidx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d_fplans, plans.data(), plans.size() * sizeof(FPlan), hipMemcpyHostToDevice));
  n_fplans = (uint32_t)plans.size();
  return 0;
}

static size_t fal(size_t x) { return (x + 255) & ~size_t(255); }

int formula_split(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t gdepth, const kg_query** q2,
                  size_t* n2, const uint32_t** n_extra, uint8_t** out2, uint32_t** err2, const uint2** ref) {
  const size_t N2 = n * (1 + (size_t)s->fp_leaves);
  if (N2 > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  auto layout = [](size_t m, size_t m2, size_t* off) {  // q2 | out2 | err2 | ref | count
    off[0] = 0;
    off[1] = fal(m2 * sizeof(kg_query));
    off[2] = off[1] + fal(m2);
    off[3] = off[2] + fal(m2 * 4);
    off[4] = off[3] + fal(m * sizeof(uint2));
    return off[4] + 256;
  };
  size_t off[5];
  const size_t need = layout(n, N2, off);
  if (need > w->split_bytes) {  // grown geometrically like the batch scratch
    const size_t want = std::max(need, 2 * w->split_bytes);
    if (w->split) hipFree(w->split);
    w->split = nullptr;
    w->split_bytes = 0;
    HIPC(hipMalloc(&w->split, want));
    w->split_bytes = want;
  }
  char* b = (char*)w->split;
  kg_query* q = (kg_query*)(b + off[0]);
  uint2* r = (uint2*)(b + off[3]);
  uint32_t* cnt = (uint32_t*)(b + off[4]);
  HIPC(hipMemsetAsync(cnt, 0, 4, w->stream));
  hipLaunchKernelGGL(k_fsplit, dim3((uint32_t)((n + FS_BLOCK - 1) / FS_BLOCK)), dim3(FS_BLOCK), 0, w->stream, s->ds, s->d_fidx,
                     (const FPlan*)s->d_fplans, d_q, (uint32_t)n, gdepth, q, r, cnt);
  HIPC(hipGetLastError());
  *q2 = q;
  *n2 = N2;
  *n_extra = cnt;
  *out2 = (uint8_t*)(b + off[1]);
  *err2 = (uint32_t*)(b + off[2]);
  *ref = r;
  return 0;
}

int formula_combine(Snapshot* s, Workspace* w, size_t n, const uint2* ref, const uint8_t* out2, const uint32_t* err2,
                    uint8_t* d_out, uint32_t* d_err) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_fcombine, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, w->stream,
                     (const FPlan*)s->d_fplans, (uint32_t)n, ref, out2, err2, d_out, d_err);
  HIPC(hipGetLastError());
  return 0;
}

}  // namespace kg
