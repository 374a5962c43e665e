// kg_grid.h -- grid tier interface (kg_grid.hip), called by the batch driver (kg_check.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kg_internal.h"

namespace kg {

struct GridStats {
  unsigned long long rows = 0, edges = 0, probes = 0, done = 0, logged = 0;
  unsigned long long ms_eload = 0, ms_wact = 0;  // k_ms_level: adjx records loaded, active (edge, word) pairs
};

// phase 1 with dsum (zeroed, 256-B aligned, GRID_SUM_WORDS): the first round keeps its counters there
// and k_grid_finish adds the list length, so they come back with the caller's one readback and need
// no memset or copy of their own; phase 2 reads them from hsum, the host copy.
constexpr uint32_t GRID_SUM_WORDS = 160;

struct Snapshot;
struct Workspace;
int grid_tier(Snapshot* s, Workspace* w, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count, int global_max_depth,
              uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs, int phase = 0, bool allow_ms = true,
              uint64_t* dsum = nullptr, const uint64_t* hsum = nullptr);
// kg_msbfs.hip: the grid tier's queries as a multi-source bit-parallel BFS (64 queries per group)
bool ms_usable(const Snapshot* s, int global_max_depth);
int ms_tier(Snapshot* s, Workspace* w, const RQuery* rq, const uint32_t* qlist, const uint32_t* d_count,
            int global_max_depth, uint8_t* out, uint32_t* err, hipStream_t stream, GridStats* gs, int phase);

}  // namespace kg
