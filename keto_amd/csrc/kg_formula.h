// kg_formula.h -- boolean rewrite plans (kg_formula.hip): shared by the single-GPU split and the
// hash-sharded seed (kg_shard.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kg {

constexpr int FP_OPS = 16, FP_LEAVES = 4;
// postfix program: LEAF | j pushes leaf j's answer; NOT flips the top; AND | k / OR | k fold the top k
// (k = 0: NotMember for both, as eval_rw answers an empty operator)
enum : uint8_t { FOP_LEAF = 0x00, FOP_NOT = 0x40, FOP_AND = 0x80, FOP_OR = 0xC0 };

struct FPlan {
  uint32_t n_ops, n_leaves;
  uint32_t leaf[FP_LEAVES];  // computed relations (same object)
  uint8_t ops[FP_OPS];
  // from the snapshot's nodes at build: some (ns, obj, R) node holds rows (its own part must be
  // looked up per query); bit j: some node of leaf relation j is impure (leaf j looked up per query)
  uint32_t own_rows, leaf_impure;
};

// The formula over leaf answers (bit j of `leaves` = leaf j is IsMember).
__device__ __forceinline__ bool fplan_eval(const FPlan& P, uint32_t leaves) {
  uint32_t st = 0;  // answer stack as bits (top = bit sp-1)
  int sp = 0;
  for (uint32_t k = 0; k < P.n_ops; k++) {
    const uint8_t op = P.ops[k];
    const uint32_t a = op & 0x3F;
    switch (op & 0xC0) {
      case FOP_LEAF:
        st = (st & ~(1u << sp)) | (((leaves >> a) & 1u) << sp);
        sp++;
        break;
      case FOP_NOT:
        st ^= 1u << (sp - 1);
        break;
      default: {  // AND / OR over the top a entries
        const uint32_t m = a ? (((1u << a) - 1u) << (sp - (int)a)) : 0u;
        const uint32_t v = (op & 0xC0) == FOP_AND ? (a && (st & m) == m) : ((st & m) != 0);
        sp -= (int)a;
        st = (st & ~(1u << sp)) | (v << sp);
        sp++;
        break;
      }
    }
  }
  return st & 1u;
}

}  // namespace kg
