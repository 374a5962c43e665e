// kg_interp.h -- interfaces between the batch driver (kg_check.hip) and the rewrite interpreter.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/ketogpu.h"
#include "kg_internal.h"

namespace kg {

constexpr int STACK_CAP = 1024;  // frames per wave slot (HBM)
constexpr int MEMO_CAP = 2048;   // (node, depth) results per wave slot (HBM, epoch-tagged)

struct MemoEnt {
  uint64_t key;
  uint64_t tag;  // batch sequence << 32 | query index; 0 = empty
  int32_t d;
  uint32_t val;
};

// Device-side control block of the GENERAL path (zeroed per batch, part of the driver's Ctl).
struct InterpCtl {
  const uint32_t* gen_count;  // -> Ctl::gen_count
  uint32_t* p2_list;          // pass-2 query list (n entries)
  uint32_t p2_count, p2_head, p3_count, p3_head;  // pass-2 / pass-3 counters (p3 list lives in the pool)
  uint32_t heads[8 * 32];
  unsigned long long* st_general;
  unsigned long long* st_rows;
  unsigned long long* st_edges;
  unsigned long long* st_probes;
};

struct Snapshot;
struct Workspace;
int launch_general(Snapshot* s, Workspace* w, const kg_query* d_q, const RQuery* rq, const uint32_t* gen_list,
                   const uint32_t* gen_count, InterpCtl* ic, uint8_t* out, uint32_t* err, uint32_t n_queries,
                   hipStream_t stream);

}  // namespace kg
